// ngs_common.h — layout of the device index and the constants of the search path.
//
// Shared by the host index builder (ngs_index.cpp), the kernels (ngs_kernels.hip) and the
// C-ABI layer (ngs_abi.cpp). Reference constants are cited (paths under /root/reference).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ngs {

// nGramSearch.hpp:82 — terms of length >= 6 go to longLib (gram search), others to shortLib.
constexpr uint32_t kShortTermLen = 6;
// nGramSearch.hpp:381 — queries shorter than 9 bytes also run the Levenshtein search.
constexpr uint32_t kShortQueryLen = 9;
// nGramSearch.hpp:235,247 — queries of <= 3 bytes Levenshtein-scan the WHOLE library.
constexpr uint32_t kFullScanQueryLen = 3;

// 3-gram code. The reference hashes c0<<16 | c1<<8 | c2 on signed chars (nGramSearch.h:147-150).
// Indexed terms only hold validChar bytes (< 0x80), so their grams are exactly the 7-bit
// triples; a query gram holding a byte >= 0x80 has a negative reference hash and can never
// match. The 21-bit code (c0<<14 | c1<<7 | c2) is therefore a lossless direct index.
constexpr uint32_t kGramBits = 21;
constexpr uint32_t kGramSpace = 1u << kGramBits;
// indexG / indexW: gram sizes 1..3 (a gram of g <= 3 code points packs into 63 bits, the
// key of the gram dictionary; grams of any other shape than narrow g=3 go through it).
constexpr uint32_t kMaxGramSize = 3;

// Score encoding shared by every stage: enc = bits(max(w*s, +0.0f)) + 1 for finite
// non-negative scores (fp32 bits of non-negative floats order like the floats), 0 = "key
// absent". An exact match promoted to 100 (nGramSearch.hpp:328-335) is the score 100 itself,
// kPromoted: ScoreComparer (nGramSearch.h:262-269) ranks a key with w*s > 100 above it and
// orders a key at exactly 100 against it by length.
constexpr uint32_t kPromoted = 0x42C80000u + 1u;  // bits(100.0f) + 1

// Candidate record = (~enc) << 32 | key: ascending order == reference order
// (score desc, then key rank asc; key ranks are assigned by (length, first appearance)).
constexpr uint64_t kNoCand = ~0ull;

// ---- fused kernel geometry (tuned on MI355X) ----
constexpr int kFastThreads = 512;        // 8 waves
constexpr int kTableSlots = 8192;        // LDS hash table, u32 slot = (term - lo + 1) << 8 | count
constexpr int kPartCap = kTableSlots / 2;// <= 50 % load: postings per term-range part
constexpr int kCandCap = 2048;           // LDS candidate buffer (u64 records)
constexpr uint32_t kFastMaxLimit = kCandCap / 2;
constexpr uint32_t kFastMaxGrams = 255;  // u8 counts in the table slot
constexpr uint32_t kMaxPartSpan = (1u << 24) - 2;  // 24-bit relative term id in the slot

// bucket skip table: K <= kMaxBuckets term-id buckets of >= kMinBucketTerms terms each
constexpr uint32_t kMaxBuckets = 256;
constexpr uint32_t kMinBucketTerms = 4096;
constexpr uint64_t kDenseBucketLen = 16;          // dense lists: postings of the longest list per bucket
constexpr uint64_t kSkipBudget = 512ull << 20;    // ... within this many bytes of skip table

// Skip-table geometry of an index (host and device builds alike): K buckets (a power of two) of
// span term ids. Up to kMaxBuckets buckets of >= kMinBucketTerms terms; more when the lists are
// dense, so that the longest list has about kDenseBucketLen postings per bucket and a query's
// parts stay whole buckets (small gram sizes: 1,369 2-grams over 40M terms), as long as the
// table stays within kSkipBudget bytes.
inline void skip_buckets(uint32_t n_long, uint32_t rows, uint64_t max_len, uint32_t& K, uint32_t& span) {
    K = 1;
    while (K < kMaxBuckets && (uint64_t)K * kMinBucketTerms < n_long) K <<= 1;
    while ((uint64_t)K * 2 <= n_long && max_len / K > kDenseBucketLen &&
           (uint64_t)rows * (K * 2 + 1) * sizeof(uint32_t) <= kSkipBudget)
        K <<= 1;
    span = n_long ? (n_long + K - 1) / K : 1;
}

// ---- wave kernel geometry (tier 1: one wave per query) ----
#ifndef NGS_SLOT_BITS
#define NGS_SLOT_BITS 10   // experiment builds override (make variant VFLAGS=-DNGS_SLOT_BITS=11)
#endif
#ifndef NGS_SKETCH_CAP
#define NGS_SKETCH_CAP 768
#endif
constexpr int kWaveSlotBits = NGS_SLOT_BITS;     // tier 1a table: 2^10 words = 4 KB
constexpr int kFullSlotBits = 11;  // tier 1b (full kernel) table: 8 KB
constexpr int kWaveSlots = 1 << kWaveSlotBits;  // wave-private LDS table (u32 words)
constexpr int kWaveCap = kWaveSlots / 2;        // entries per exact-count pass (<= 50 % table load)
constexpr int kSketchCellBits = 4;              // sketch counters: u4, 8 per table word
constexpr uint32_t kSketchMax = (1u << kSketchCellBits) - 1u;
constexpr int kSketchCap = NGS_SKETCH_CAP;      // entries per sketch part (<= 1/8 of the cells)
static_assert(kSketchCap * 8 <= kWaveSlots * (32 / kSketchCellBits), "sketch load");
constexpr int kWaveCand = 256;        // candidate buffer per query
constexpr uint32_t kGenSelThreads = 1024;       // general path: k_gen_select's workgroup (one per query)
constexpr uint32_t kGenSelCap = 1024;           // ... and the limits it takes (larger: sort per query)
constexpr uint32_t kWaveMaxLimit = 128;         // tier 1 limits (<= kWaveCand / 2)
static_assert(kWaveMaxLimit * 2 <= (uint32_t)kWaveCand, "a flush keeps at most half the buffer");
constexpr int kWaveChunks = kSketchCap / 4;     // 16-byte chunks per part and wave (sketch parts)
constexpr int kExactChunks = (kWaveCap < kSketchCap ? kWaveCap : kSketchCap) / 4;  // ... parts counted exactly (cmin <= 2)
constexpr int kDmaRounds = kWaveChunks / 64;    // dwordx4 loads per lane for one part
#ifndef NGS_WPS
#define NGS_WPS 3
#endif
constexpr int kWaveWavesPerSimd = NGS_WPS;      // occupancy target of tier 1b: 3 -> <= 168 VGPRs (C4 -7 % time against 4)
#ifndef NGS_LEAN_WPS
#define NGS_LEAN_WPS 6
#endif
constexpr int kLeanWavesPerSimd = NGS_LEAN_WPS; // tier 1a: 6 -> <= 80 VGPRs (LDS 6 KB: 24 waves per CU)
#ifndef NGS_HEAVY_LEAN_WPS
#define NGS_HEAVY_LEAN_WPS NGS_LEAN_WPS  // (5: 95 VGPRs and no scratch, measured no faster: profiles/r04_s2_ab_heavy_wps_sort64.txt)
#endif
constexpr int kHeavyLeanWavesPerSimd = NGS_HEAVY_LEAN_WPS;  // ... the heavy list's launch (packed staging)
// Tier 1a writes its survivor list (term, count) to HBM and k_emit runs calcScore and the top-L per
// query afterwards: the dependent term -> key loads and the sorts leave the occupancy-bound counting
// kernel (SearchParams.esn / est / esc).
constexpr uint32_t kListSlots = 64;             // slot lists per routing list in k_prep
constexpr uint32_t kNoEmit = 0xFFFFFFFFu;       // esn[q]: query not finished by tier 1a
constexpr uint32_t kEmitHeavy = 0x80000000u;    // esn[q] flag: finished by the heavy-list launch
// a sliced heavy query's word (SearchParams.eovf, zeroed by k_prep; heavy queries have no arena):
// survivor slots taken (low 24 bits), slices finished (kHeavyDone each), handed over (kHeavyBailed)
constexpr uint32_t kHeavySlotMask = 0xFFFFFFu;
constexpr uint32_t kHeavyDone = 1u << 24;
constexpr uint32_t kHeavyBailed = 0x80000000u;
constexpr uint32_t kHeavyCmin = 2; // queries with cmin <= this go to the heavy list from the start
// the heavy list runs through the lean kernel (its survivors spill to k_emit; short-search queries
// and cmin-1 queries without part_ones hand over to tier 1b)
constexpr uint32_t kLeanShrink2 = 1;  // tier 1a cmin-2 sketch parts: cap and target >> this
// the heavy list's launch also takes cmin-1 queries (threshold 0): part_ones
constexpr uint32_t kOnesShrink = 2;  // ... in parts of a quarter of the sketch cap
constexpr uint32_t kBackPieces = 4;              // host batches: records read back in up to this many pieces
constexpr uint32_t kBackPieceMin = 131072;        // ... of at least this many records
constexpr uint32_t kOneStreamBatch = 16384;     // batches up to this size run on one stream per call
constexpr uint32_t kHeavyGrid = 4096;           // the heavy list's launches: this many workgroups (grid-stride)
constexpr uint32_t kHeavyMaxSlices = 8;         // ... over (query, term-id slice) items, up to this many per query
constexpr uint32_t kHeavyItems = 8 * kHeavyGrid; // ... as many slices as keep about this many items
constexpr uint32_t kHeavySliceList = 1024;      // ... on indexes of at least this many postings per list
constexpr uint32_t kHeavyOverflowGrid = 1024;   // ... the overflow launch's grid (items past the hinted grid)
constexpr uint64_t kHeavySlicePostings = 3840;  // ... a slice per this many of the query's postings (~16 parts)
constexpr int kWaveTarget = kWaveCap * 5 / 8;   // postings per exact part the bucket grouping aims at
#ifndef NGS_TGT8
#define NGS_TGT8 5
#endif
constexpr int kSketchTarget = kSketchCap * NGS_TGT8 / 8;  // ... per sketch part (bucket groups aim at NGS_TGT8/8 of the cap)
constexpr int kGroupTarget = kSketchCap * NGS_TGT8 / 8;  // ... the same for tier 1a's lane-group staging (lean_query_g)
constexpr uint32_t kStray = 0xFFFFFFFFu;        // staged entry outside its list segment
constexpr int kWaveSurv = 128;                  // survivor list (term, count) before calcScore
constexpr uint32_t kEmitCap = 1024;
// threshold-0 queries on rank lists (DevIndex.rank_post): tier 1a leaves the query's lists for k_emit
// in the last slots of its survivor slots, per list lane the posting offset (2 x u32) and the length
constexpr uint32_t kRankInfo = 3 * 64;
// batches up to kEmitWideBatch queries get kEmitCapWide slots per query (5 bytes each): a
// threshold-0 query has thousands of one-hit survivors at C2 (part_ones)
constexpr uint32_t kEmitCapWide = 4096;
constexpr uint64_t kEmitWideBytes = 1ull << 30;       // ... halved until the batch's slots fit this
constexpr uint32_t kEmitCapMax = 32768;              // ... grown up to this many per query
constexpr uint32_t kArenaBlock = 1024;               // survivor arena block (entries; a multiple of 128)
constexpr uint32_t kArenaChain = 128;                // blocks one query may chain (k_emit lists them in LDS)
constexpr uint32_t kArenaCtrWord = 12;               // SearchParams.actr: this word of the path-count line
                                                     // (and the next: blocks still needed when it ran out)
constexpr uint64_t kEmitBudget = 16ull << 30;         // ... within this many bytes per context
constexpr size_t kEmitWideBatch = 262144;             // tier 1a survivors per query spilled to HBM for k_emit
constexpr uint32_t kWaveMaxGrams = 63;          // counts <= 63: one lane per count value
constexpr uint32_t kSketchMinCmin = 2;     // smallest cmin counted by the sketch (below: exact hash counting)

struct DevIndex {  // passed by value to kernels; all pointers are device pointers
    const uint64_t* gram_off;   // [kGramSpace + 1] -> post
    const uint32_t* post;       // long-term ids (0-based within longLib), sorted per gram
    const uint32_t* gram_row;   // [kGramSpace] -> row of skip (UINT32_MAX = empty)
    const uint32_t* skip;       // [rows][n_buckets + 1] offset of the first posting >= b * bucket_span
    uint32_t n_buckets, bucket_span;
    uint32_t post_per_row;      // postings per non-empty gram list (heavy_slices)
    const uint64_t* term_off;   // [n_terms + 1] -> term_bytes (normalised terms)
    const uint8_t* term_bytes;
    const uint32_t* tk_off;     // [n_terms + 1] -> tk
    const uint2* tk;            // {key rank, weight bits} — wordMap + wordWeight (h:290,293)
    const uint64_t* key_off;    // [n_keys + 1] -> key_bytes (raw trimmed keys, NUL-separated)
    const uint8_t* key_bytes;
    const uint32_t* wild_key;   // wildcard answer, pre-sorted (hpp:356-369)
    const float* wild_score;
    uint32_t n_terms, n_short, n_keys;
    uint32_t keys_unique;       // 1: every key has one (term, key) pair, so a query's records never
                                // share a key and the top-L needs no key dedup pass
    uint32_t tk_identity;       // 1: term t's pairs are exactly tk[t] (tk_off[t] == t): one load less
    float w_max;                // largest pair weight (<= 0: none positive); bounds a term's best score
    uint32_t tk_monotone;       // 1: term ids ascend with key rank (all of t's below all of t + 1's):
                                // a term loses every score tie against the records of lower terms
    // gram size and character width (indexG / indexW extensions; 3 and 1 for indexN)
    uint32_t gsz, csize, gram_mode;         // gram_mode 1: grams via the dictionary below
    uint32_t short_query_len, full_scan_len; // 3g and g (nGramSearch.hpp:381, :247)
    uint32_t ghash_bits;
    const uint64_t* ghash_key;  // dictionary mode: open addressing on packed code points, ~0 = empty
    const uint32_t* ghash_val;  // -> gram id (row of gram_off / gram_row)
    // Rank lists (threshold 0, cmin 1): when every pair has one weight, every term one pair and every
    // key one term, a one-hit term's record is (the one score of 1/n hits, its key rank), so the one-hit
    // records of a query's top-L are the smallest key ranks of its lists. rank_post holds, per gram,
    // the key ranks of its postings in ascending order (the offsets of post); null otherwise.
    const uint32_t* rank_post;
    uint32_t w_uniform;         // ... the weight's bits
    // key -> its terms (the pairs transposed), for keys with several pairs; null when every key
    // has one pair (keys_unique). kt_flag (per validChar set, k_key_flags): 1 = a long term
    // promotes the key when it is queried, after its short pairs (pair_enc drops those above 100)
    const uint32_t* kt_off;     // [n_keys + 1] -> kt_term
    const uint32_t* kt_term;
    const uint8_t* kt_flag;
};

struct ValidSet {  // a 256-bit validChar set by value (kernel argument)
    uint32_t w[8];
};

constexpr uint64_t kGramEmpty = ~0ull;

struct SearchParams {
    float thr;
    uint32_t limit;      // effective L = min(limit or 2^31-1, n_keys)
    uint32_t out_stride;
    uint32_t n_queries;
    uint32_t valid[8];   // 256-bit validChar mask (h:307-313 / setValidChar)
    uint32_t dbg;        // ablation switches for performance experiments (NGS_DEBUG); 0 in production
    uint32_t waves;      // tier 1: 0 = lean 1a + full 1b (batches), 1 = the full kernel alone (latency path)
    uint32_t lean_all;     // tier 1a also takes heavy queries (its launch over the heavy list)
    // the heavy list's launch: term-id slices per query (0: from the list's length, heavy_slices;
    // NGS_HEAVY_SLICES); a sliced query's survivors take slots from eovf[q] (heavy_slot).
    // hbase: the first (query, slice) item of a heavy launch (its overflow launch starts past the
    // first launch's grid); hgrid: the first launch's grid from the context's last call (0: none)
    uint32_t hslices, hbase, hgrid;
    // deferred calcScore (kDeferEmit): per query the survivor count (kNoEmit = none) and
    // kEmitCap survivor slots, terms and hit counts
    uint32_t* esn;
    uint32_t* est;
    uint8_t* esc;
    uint32_t ecap;       // survivor slots per query (emit_cap: kEmitCap .. kEmitCapWide, grown by the host)
    // sliced tier 1b (kSlices): the full list and the hand-over lists run as nslices term-id
    // slices of each query (one wave each, bucket ranges of the skip table); slice j of query q
    // leaves its top-L records at prec[(q * nslices + j) * limit] and their count at
    // pcnt[q * nslices + j], merged by k_merge. nslices 1: unsliced
    uint32_t nslices;
    uint64_t* prec;
    uint32_t* pcnt;
    // capacity (bytes) of the normalised-query buffer: k_prep flags (*oflow = 1) a query whose
    // bytes end past it instead of writing, and the host reruns the call with a larger buffer
    // (ngsSearchDevice does not read the batch's byte count back before launching)
    uint64_t qcap;
    uint32_t* oflow;
    // batch-wide survivor arena (the main tier-1a launch, lean_query_g): a query whose survivors outgrow
    // its ecap slots goes on in blocks of kArenaBlock entries taken from *actr (a word of the call's
    // path-count line, zeroed with it); its first block is eovf[q] - 1 (0: none, reset by k_prep),
    // a block's successor anext[b] - 1. A counter past ablocks means the arena ran out (the query
    // went to tier 1b; the host grows the arena for later calls). at == null: no arena.
    uint32_t* eovf;
    uint32_t* anext;
    uint32_t* at;
    uint8_t* ac;
    uint32_t* actr;
    uint32_t ablocks;
    // the latency path: k_prep zeroes these words (the statistics and path counts, which the
    // tier kernels after it accumulate) in place of a memset launch; null otherwise
    uint32_t* zero_stats;
    uint32_t zero_words;
    // tier 1b over a list (k_wave): a persistent grid takes its (query, slice) items from this
    // counter (zeroed with the path counts) instead of one workgroup per item; null: grid-stride
    uint32_t* qhead;
};

// Term-id slices per heavy-list query (the most; lean_query takes fewer for a query of fewer
// postings), host and device alike (the host sizes the next call's grid with it): hslices, else
// as many as keep about kHeavyItems (query, slice) items, no more than the longest heavy query is
// estimated to use (cmin <= 2: at most 2 / thr grams of post_per_row postings each, a slice per
// kHeavySlicePostings), at most kHeavyMaxSlices and one bucket per slice. None on an index of short
// lists (C2, 1M rows: ~11 parts per query, where the slices' own set-up cost more than they saved:
// 40.6 -> 36.0 Mq/s, profiles/r05_s7_ab_heavy_slices_c2.txt)
__host__ __device__ inline uint32_t heavy_slices(const SearchParams& P, uint32_t cnt, const DevIndex& X) {
    if (!P.hslices && X.post_per_row < kHeavySliceList) return 1;
    uint32_t want = P.hslices;
    if (!want) {
        const uint32_t nmax = P.thr > 0.0f && 2.0f / P.thr < (float)kWaveMaxGrams ? (uint32_t)(2.0f / P.thr) : kWaveMaxGrams;
        const uint64_t est = ((uint64_t)nmax * X.post_per_row + kHeavySlicePostings - 1) / kHeavySlicePostings;
        want = kHeavyItems / (cnt ? cnt : 1u);
        if (est < want) want = (uint32_t)(est ? est : 1u);
    }
    if (want > kHeavyMaxSlices) want = kHeavyMaxSlices;
    if (want > X.n_buckets) want = X.n_buckets;
    return want ? want : 1u;
}

// Tier 1b slices per query (SearchParams.nslices): a full-list or handed-over query is a few
// hundred to thousands of survivors in one wave; four waves on disjoint term-id ranges each keep
// their own top-L, and k_merge joins them. The key-max merge is exact: a key among the global
// top L is among the top L of the slice holding its best record.
constexpr uint32_t kSlices = 4;
constexpr uint32_t kTier1bGrid = 65536;  // cap on the persistent tier-1b grids (else one per wave slot)
constexpr uint32_t kNoPart = 0xFFFFFFFFu;  // pcnt[q * nslices]: the query was answered unsliced

// ---- low-latency score() (ngsServe, opt-in): a persistent one-wave server kernel polls a
// request block in coherent pinned host memory, answers the query with the tier-1 wave search
// and writes the results back into the same block; no launch, copy or wait per call.
constexpr uint32_t kServeMaxQuery = 256;   // normalised query characters the block holds
constexpr uint32_t kServeSlots = 8;        // server waves, one request block each (4 and 2 measured
                                           // lower past 4 / 2 concurrent callers: DESIGN.md §6)
struct alignas(64) ServeBlock {
    // host -> device
    uint64_t req_seq;          // the host stores the request's number last (release)
    uint32_t stop;             // != 0: the server exits
    uint32_t pad0;
    float thr;
    uint32_t limit;            // effective limit (<= kWaveMaxLimit)
    uint32_t m;                // normalised length, or kQueryWildcard
    uint32_t pad1;
    uint64_t off[2];           // {0, m}: the query's offsets into q (wave_query's qoff)
    uint32_t valid[8];         // the index's validChar set at the call (setValidChar)
    uint8_t q[kServeMaxQuery]; // the normalised query
    // device -> host
    uint64_t done_seq;         // the server stores the answered request's number last (release)
    uint32_t alive;            // 1 while the server runs (set at start, cleared at exit)
    uint32_t status;           // 0 answered; 1 the query needs the host path (tier 2 / general)
    uint32_t n;                // results
    uint32_t pad2[3];
    uint32_t keys[kWaveMaxLimit];
    float scores[kWaveMaxLimit];
};

// per-query normalised length sentinels written by the prep kernel
constexpr uint32_t kQueryWildcard = 0xFFFFFFFFu;

// Statistics are accumulated into kStatSlots cache-line slots (query q adds to slot q % kStatSlots)
// and summed on the host: 65,536 queries adding into one line serialised at one memory channel.
constexpr uint32_t kStatSlots = 256;
struct alignas(64) DevStats {  // accumulated by the fused kernel (one atomic per query, per slot)
    unsigned long long postings;
    unsigned long long lists;
    unsigned long long results;
    unsigned long long fast;
    unsigned long long survivors;  // scored terms that passed the threshold
    unsigned errors;  // bit 0 table overflow, 1 flush rounds, 2 part rounds: all "cannot happen"
    unsigned slot_full;  // queries tier 1a handed over because their survivor slots (ecap) were full
    unsigned long long main_postings;  // postings and lists of the queries the main tier-1a launch finished
    unsigned long long main_lists;     // (its own algorithmic bytes, bench.py's serialised roofline)
};

}  // namespace ngs
