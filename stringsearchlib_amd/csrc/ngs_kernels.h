// ngs_kernels.h — launchers of the gfx950 search kernels (ngs_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "ngs_common.h"

namespace ngs {

// Normalise every query (escapeBlank -> trim -> toUpper, nGramSearch.hpp:372-376) into
// qnorm (same offsets as the raw bytes) and its length into qm (kQueryWildcard for ""/"*").
// The heavy and full lists (tier-1 routing) go through 2 x kListSlots slot lists: `slots` holds
// 2 * kListSlots * ceil(B / kListSlots) entries, `ctr` 2 * kListSlots counters 16 words apart
// (zeroed by the caller). The lists are merged on `side` after an event on s (prep_ev), so the
// main tier-1a launch queued next on s does not wait for them; lists_ev marks them done.
// A graph being built node by node (hipGraphAdd*Node, no stream capture): a launch function given
// one appends its kernels after `last` instead of queueing them. One-stream calls only (side ==
// side2 == s: no events). err keeps the first failure.
struct GraphBuild {
    hipGraph_t graph = nullptr;
    hipGraphNode_t last = nullptr;
    hipError_t err = hipSuccess;
};

hipError_t launch_prep(const uint8_t* raw, const uint64_t* off, uint32_t B, const SearchParams& P,
                       uint8_t* qnorm, uint32_t* qm, uint32_t cs, const DevIndex& X, uint32_t* heavy,
                       uint32_t* hcount, uint32_t* full, uint32_t* fcount, uint32_t* slots, uint32_t* ctr,
                       hipStream_t s, hipStream_t side, hipEvent_t prep_ev, hipEvent_t lists_ev,
                       GraphBuild* gb = nullptr);

// Fused per-query kernel: short Levenshtein scan of shortLib (4 <= m < 9), 3-gram posting
// count in an LDS hash table per term-id part, threshold, term->key weighting, per-key max
// merge and top-L in LDS. Queries it cannot take are appended to glist for the general path.
// Tier 1 (k_wave, one wave per query: <= 64 grams, limit <= 128) then tier 2 (k_fast, one block
// per query over list2: <= 255 grams, limit <= 1024); what remains goes to glist.
hipError_t launch_fast(const DevIndex& X, const SearchParams& P, const uint8_t* qnorm, const uint64_t* off,
                       const uint32_t* qm, uint32_t* out_n, uint32_t* out_k, float* out_s, uint32_t* list2,
                       uint32_t* count2, uint32_t* fb, uint32_t* fbc, uint32_t* fb2, uint32_t* fbc2,
                       const uint32_t* heavy, const uint32_t* hcount, const uint32_t* full,
                       const uint32_t* fcount, uint32_t* glist, uint32_t* gcount, DevStats* stats, hipStream_t s,
                       hipStream_t side, hipStream_t side2, hipEvent_t join, hipEvent_t join2,
                       hipEvent_t lists_ev, bool all_heavy = false, hipEvent_t main_ev = nullptr, bool main_wait = false,
                       GraphBuild* gb = nullptr);

// The low-latency server (ngsServe): kServeSlots persistent one-wave workgroups on `s`, wave i
// serving requests from blk[i] (coherent pinned host memory, device view) until blk[0].stop, or
// until no request came to any slot for idle_ms (t_any: device memory, the latest request time),
// or after life_ms in all. scratch: kServeSlots x (kStatSlots + 1) DevStats of device memory
// (statistics and the tier-2 routing count it ignores), list2: kServeSlots x 4 words.
hipError_t launch_serve(const DevIndex& X, const SearchParams& P, ServeBlock* blk, DevStats* scratch,
                        uint32_t* list2, unsigned long long* t_any, uint32_t idle_ms, uint32_t life_ms, hipStream_t s);

// Result compaction for the host entry points: pos[0..B] = exclusive prefix sum of n[0..B) (n
// holds B + 1 entries, n[B] = 0), then query q's n[q] records (k, s at q * stride) are copied to
// pk / ps at pos[q]. The host then copies pos and the pos[B] packed records, not B * stride.
size_t pack_temp_bytes(uint32_t B);
hipError_t launch_pack(const uint32_t* n, const uint32_t* k, const float* s, uint32_t B, uint32_t stride,
                       uint32_t* pos, uint32_t* pk, float* ps, void* temp, size_t temp_bytes, hipStream_t st,
                       const uint64_t* koff = nullptr, uint64_t pbase = 0, uint32_t cs = 0, uint64_t* pp = nullptr);
// ngsPackResults: counts[B] + records at i * stride -> pos[B + 1] (exclusive sum) and rec[2 * total]
// = {key, score bits} pairs (the packed multi-GPU gather, stringsearchlib_amd/shard.py)
size_t pack_pairs_temp_bytes(uint32_t B);
hipError_t launch_pack_pairs(const uint32_t* n, const uint32_t* k, const float* s, uint32_t B, uint32_t stride,
                             uint32_t* pos, uint32_t* rec, void* temp, size_t temp_bytes, hipStream_t st);

// Wildcard answer (nGramSearch.hpp:356-369): keys sorted by (weight desc, rank asc).
hipError_t build_wildcard(const float* d_w, uint32_t n_keys, uint32_t* d_keys, float* d_scores, hipStream_t s);

// DevIndex.kt_flag of an index with kt_off / kt_term under one validChar set (k_key_flags)
hipError_t build_key_flags(const DevIndex& X, const uint32_t valid[8], uint8_t* flags, hipStream_t s);

// hipcub's int item count bounds the rank lists' segmented sort
constexpr uint64_t kRankMaxPostings = 0x7FFFFFFFull;
// Rank lists of an index (DevIndex.rank_post): out[i] = tk[n_short + post[i]].x, each gram's
// segment gram_off[c] .. gram_off[c + 1] (c < n_seg) sorted ascending. out holds n_post + 4 entries.
hipError_t build_rank_post(const uint64_t* gram_off, uint32_t n_seg, const uint32_t* post, uint64_t n_post,
                           const uint2* tk, uint32_t n_short, uint32_t n_keys, uint32_t* out, hipStream_t s);

// General path: library-wide dense scoring of G queries at once (m <= 3 full-library scans,
// very long queries, limits above kFastMaxLimit).
struct GeneralBuffers {
    uint32_t G = 0;             // queries per group
    uint32_t* cnt = nullptr;    // [G][n_long] posting counts (self-clearing)
    uint32_t* kenc = nullptr;   // [G][gen_kstride(n_keys)] per-key score encoding (self-clearing)
    uint64_t* list = nullptr;   // [G][n_keys] compacted candidate records
    uint64_t* sorted = nullptr; // [n_keys] radix-sort output
    uint32_t* lcount = nullptr; // [G] candidates per query
    void* temp = nullptr;       // radix-sort scratch
    size_t temp_bytes = 0;
};
size_t general_sort_temp_bytes(uint32_t n_keys);
constexpr uint32_t kGeneralMaxGroup = 256;  // queries per group (one k_gen_select workgroup each)
// kenc's row stride: n_keys rounded up to whole 16-byte loads (the padding stays zero)
__host__ __device__ inline uint32_t gen_kstride(uint32_t n_keys) { return (n_keys + 3u) & ~3u; }

// Diagnostic build (make prof, -DNGS_PHASE_STAMPS): accumulated block-time per k_fast phase in
// 100 MHz ticks. Returns the number of phases, or -1 in the regular build.
int phase_stats(unsigned long long* out, int n, bool reset);
hipError_t run_general(const DevIndex& X, const SearchParams& P, const uint8_t* qnorm, const uint64_t* off,
                       const uint32_t* qm, const uint32_t* d_group, const uint32_t* h_group, uint32_t G,
                       GeneralBuffers& W, uint32_t* out_n, uint32_t* out_k, float* out_s, hipStream_t s);

}  // namespace ngs
