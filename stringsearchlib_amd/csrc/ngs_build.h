// ngs_build.h — the gram CSR, gram dictionary and skip table of an index, built on the GPU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "ngs_common.h"

namespace ngs {

struct DeviceGrams {           // device arrays, owned by the caller after a successful build
    uint64_t* gram_off = nullptr;  // [G + 1]: G = kGramSpace codes, or the dictionary's ids
    uint32_t* post = nullptr;      // [n_post + 4]
    uint32_t* gram_row = nullptr;  // [G]
    uint32_t* skip = nullptr;      // [n_grams][n_buckets + 1]
    uint64_t n_post = 0, n_grams = 0;
    uint32_t n_buckets = 1, bucket_span = 1;
};

// From the normalised terms in HBM (term_off in characters, term_bytes; long terms are ids
// [n_short, n_terms)). Same arrays as the host build (ngs_index.cpp build_grams_impl).
// Dictionary mode (dict != nullptr: every shape but narrow 3-grams): a gram is the key of its g
// characters (cs bytes each, 21 bits per character), and its id is the key's rank among the
// index's distinct keys, dict[0 .. nspace) ascending (gram_keys_device).
hipError_t build_grams_device(const uint64_t* term_off, const uint8_t* term_bytes, uint32_t n_short,
                              uint32_t n_terms, DeviceGrams& out, const uint64_t* dict = nullptr,
                              uint32_t nspace = 0, uint32_t cs = 1, uint32_t g = 3);

// Dictionary mode: the distinct gram keys of the long terms, ascending, to the host (the host then
// lays out the lookup table, set_gram_dict, exactly as its own build does).
hipError_t gram_keys_device(const uint64_t* term_off, const uint8_t* term_bytes, uint32_t n_short,
                            uint32_t n_terms, uint32_t cs, uint32_t g, std::vector<uint64_t>& keys);

struct HostIndex;

// Term ids within each class (short, long) follow first appearance, or with NGS_TERM_ORDER=rank
// the terms' best key rank first (both builds read it). The rank order makes DevIndex.tk_monotone
// hold, so tier 1b stops counting one-hit terms exactly once its top-L is full of them: C2
// (thr 0) 8.8 -> 14.7 Mq/s; but it groups the terms by key length, which skews the skip buckets'
// posting mass and the sketch candidates of the lean kernel: C3 29.1 -> 20.2 Mq/s.
inline bool term_order_by_rank() {
    static const bool r = [] {
        const char* e = std::getenv("NGS_TERM_ORDER");
        return e && std::strcmp(e, "rank") == 0;
    }();
    return r;
}

// String interning, term ids, key ranks, the term -> key CSR and the wildcard weights of an index
// on the current device (ngs_intern.hip), into the host index (ix.csize, short_term_len set by the
// caller). words are char* (ix.csize 1) or UTF-32 strings (4). hipErrorNotSupported: the host
// build must decide (a 64-bit hash collision between two strings, a NaN weight, >= 2^31 words, or
// no pair at all); other codes are HIP failures.
hipError_t intern_device(HostIndex& ix, const void* const* words, uint64_t size, uint16_t rowSize,
                         const float* weight, uint32_t g);

}  // namespace ngs
