// ngs_build.h — the gram CSR and skip table of a narrow 3-gram index, built on the GPU.
#pragma once

#include <hip/hip_runtime.h>

#include "ngs_common.h"

namespace ngs {

struct DeviceGrams {           // device arrays, owned by the caller after a successful build
    uint64_t* gram_off = nullptr;  // [kGramSpace + 1]
    uint32_t* post = nullptr;      // [n_post + 4]
    uint32_t* gram_row = nullptr;  // [kGramSpace]
    uint32_t* skip = nullptr;      // [n_grams][n_buckets + 1]
    uint64_t n_post = 0, n_grams = 0;
    uint32_t n_buckets = 1, bucket_span = 1;
};

// From the normalised terms in HBM (term_off in characters, term_bytes; long terms are ids
// [n_short, n_terms)). Same arrays as the host build (ngs_index.cpp build_grams_impl).
hipError_t build_grams_device(const uint64_t* term_off, const uint8_t* term_bytes, uint32_t n_short,
                              uint32_t n_terms, DeviceGrams& out);

}  // namespace ngs
