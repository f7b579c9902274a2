// ngs_index.h — host-side index build: normalise the library and lay it out for HBM.
//
// Restates the reference's index construction (nGramSearch.hpp:120-172 ctor, :54-108 init,
// :13-21/:41-46 gram build) as flat arrays instead of hash-of-hash-sets:
//   terms      normalised strings; shortLib (len < 6) gets ids [0, n_short), longLib the rest
//   keys       raw trimmed master keys, ranked by (length asc, first appearance asc): the
//              ScoreComparer's length tie-break (nGramSearch.h:262-269) plus a deterministic
//              refinement of the reference's unspecified order
//   tk         term -> (key rank, weight) CSR  (wordMap + wordWeight, nGramSearch.h:290,293)
//   gram CSR   21-bit gram code -> sorted long-term ids (ngrams, nGramSearch.h:296)
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "ngs_common.h"

namespace ngs {

// NGS_BUILD_TIMING=1 prints the index build's phases (seconds since the previous mark) to stderr
struct PhaseTimer {
    bool on = std::getenv("NGS_BUILD_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngs build] %-26s %8.3f s\n", what, std::chrono::duration<double>(n - t).count());
        t = n;
    }
};

struct HostIndex {
    bool indexed = false;                   // nGramSearch.h:301
    bool grams_built = false;               // gram CSR + skip table on the host (else the GPU builds them)
    // characters: 1 byte (indexN / indexG) or 4 (indexW, UTF-32); offsets below count characters
    uint32_t csize = 1, gsz = 3;
    // 0: gram = 21-bit code of 3 ASCII bytes, direct-indexed; 1: gram dictionary (ghash)
    uint32_t gram_mode = 0;
    uint32_t short_term_len = 6, short_query_len = 9, full_scan_len = 3;  // 2g, 3g, g
    std::vector<uint64_t> gram_keys;        // dictionary mode: the distinct gram keys, ascending (id = rank)
    std::vector<uint64_t> ghash_key;        // dictionary mode: open addressing, ~0 = empty
    std::vector<uint32_t> ghash_val;        // -> gram id (CSR row of gram_off)
    uint32_t ghash_bits = 0;
    uint32_t n_terms = 0, n_short = 0, n_keys = 0;
    uint64_t n_grams = 0;                   // distinct grams -> getLibSize
    std::vector<uint64_t> gram_off;         // gram space + 1 (kGramSpace codes, or dictionary ids)
    std::vector<uint32_t> post;
    uint32_t n_buckets = 1, bucket_span = 1; // term-id buckets of the skip table
    std::vector<uint32_t> gram_row;         // kGramSpace: row of the skip table, UINT32_MAX = empty list
    std::vector<uint32_t> skip;             // rows x (n_buckets + 1) list offsets
    std::vector<uint64_t> term_off;
    std::vector<uint8_t> term_bytes;
    std::vector<uint32_t> tk_off;
    std::vector<uint2> tk;                  // {key rank, float bits}
    std::vector<uint64_t> key_off;          // key k = key_bytes[key_off[k] .. key_off[k+1]-1), NUL at end
    std::vector<char> key_bytes;
    std::vector<float> wild_w;              // wildcard score per key (max of its pair weights)
};

// Builds the index; `threads` workers for the gram CSR (0 = hardware concurrency).
void build_index(HostIndex& ix, char* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                 unsigned threads = 0);

// Extensions (BASELINE north_star / README gSize; parity self-consistent):
// narrow strings with gram size gsz (1..3), and wide UTF-32 strings (indexW).
void build_index_g(HostIndex& ix, char* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                   uint32_t gsz, unsigned threads = 0);
void build_index_w(HostIndex& ix, const uint32_t* const* words, uint64_t size, uint16_t rowSize,
                   const float* weight, uint32_t gsz, unsigned threads = 0);

// The gram CSR and skip table of an index whose terms are laid out (grams_built == false): the
// host fallback of the device build.
void build_grams_host(HostIndex& ix, unsigned threads = 0);

// Dictionary mode: the gram ids of the sorted distinct keys (id = rank) and the open-addressing
// table the device looks them up in (ghash_key / ghash_val / ghash_bits), as build_grams_impl
// makes them; the device build (ngs_build.hip) computes the keys and hands them here.
void set_gram_dict(HostIndex& ix, std::vector<uint64_t> sorted_keys);

// Wildcard answer: keys sorted by (wild_w desc, rank asc).
void wildcard_order(const HostIndex& ix, std::vector<uint32_t>& keys, std::vector<float>& scores);

}  // namespace ngs
