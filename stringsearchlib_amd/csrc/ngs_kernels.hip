// ngs_kernels.hip — gfx950 kernels of the batched search() path.
//
// Reference semantics (paths under /root/reference):
//   query normalisation  nGramSearch.hpp:372-376 (escapeBlank h:93-98, trim h:243-247, toUpper h:72-76)
//   searchLong           nGramSearch.hpp:278-301   count[t] = #query grams (with multiplicity) in t
//   searchShort          nGramSearch.hpp:182-270   semi-global edit distance, |q| < 9 (whole lib if |q| <= 3)
//   calcScore            nGramSearch.hpp:310-341   s >= thr, key score = max(w*s, 0), exact -> 100
//   top-k                nGramSearch.hpp:397-401   score desc, key length asc (ScoreComparer h:262-269)
//
// Numerics (bit-exact with the reference): s = (float)count / (float)n is one correctly rounded
// fp32 division (built with -fhip-fp32-correctly-rounded-divide-sqrt); w*s one fp32 multiply
// (-ffp-contract=off); threshold `s < thr` in fp32; promotion test `(double)s > 0.999`.
#include <hipcub/hipcub.hpp>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <tuple>

#include "ngs_kernels.h"

namespace ngs {
namespace {

#ifdef NGS_PHASE_STAMPS
// Diagnostic build only (make prof): block-time per phase of k_fast, in 100 MHz ticks.
__device__ unsigned long long g_phase[48];  // [16, 32) the packed lean kernel, [32, 48) lean_query_g
#define STAMP(i)                                                          \
    if (threadIdx.x == 0) {                                               \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();   \
        atomicAdd(&g_phase[i], t_ - tp_);                                 \
        tp_ = t_;                                                         \
    }
// wave kernel: cycles (s_memtime) per phase, phases 16..31
#define WSTAMP(i)                                                         \
    {                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
        wacc_[i] += t_ - wt_;                                             \
        wt_ = t_;                                                         \
    }
#define WCOUNT(i, v) wacc_[i] += (v)
#define WPHASE_BEGIN                                       \
    unsigned long long wt_ = __builtin_amdgcn_s_memtime(); \
    unsigned long long wacc_[16] = {};
#define WPHASE_END(base) \
    if (lane_id() == 0)  \
        for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&g_phase[(base) + i_], wacc_[i_]);
#else
#define WCOUNT(i, v)
#define STAMP(i)
#define WSTAMP(i)
#define WPHASE_BEGIN
#define WPHASE_END(base)
#endif

// a global (address space 1) pointer: keeps global_load addressing where a pointer passes through
// inline asm, which hides the address space the compiler inferred from the kernel argument
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
using gptr = const T __attribute__((address_space(1)))*;
#else  // the host pass parses the device code only
template <class T>
using gptr = const T*;
#endif

__device__ __forceinline__ uint64_t min64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t max64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__device__ __forceinline__ bool dev_space(unsigned c) { return c == 32u || (c >= 9u && c <= 13u); }
__device__ __forceinline__ unsigned dev_upper(unsigned c) { return (c >= 'a' && c <= 'z') ? c - 32u : c; }
__device__ __forceinline__ unsigned esc(const uint32_t* valid, unsigned c) {
    return ((valid[c >> 5] >> (c & 31u)) & 1u) ? c : 32u;  // escapeBlank
}
// Characters are bytes (indexN / indexG) or UTF-32 code points (indexW): cs = 1 or 4. Wide code
// points below 128 are escaped like bytes; from 128 they are kept, except non-code-points
// (> 0x10FFFF), which become spaces.
__device__ __forceinline__ unsigned esc_cs(const uint32_t* valid, uint32_t c, uint32_t cs) {
    return (cs == 1 || c < 128u) ? esc(valid, c) : (c > 0x10FFFFu ? 32u : c);
}
__device__ __forceinline__ uint32_t char_at(const uint8_t* base, uint64_t i, uint32_t cs) {
    return cs == 4 ? reinterpret_cast<const uint32_t*>(base)[i] : (uint32_t)base[i];
}

// Queries tier 1a leaves to a launch of their own, known from the normalised length alone:
// 1 (heavy list) match-count threshold cmin == 2, where every term sharing a (g+1)-gram with the
//   query survives: hundreds of survivors, which the heavy list's lean launch spills to k_emit;
//   the same list takes cmin 1 (part_ones, every term sharing a gram survives);
// 2 (full list, tier 1b) a short search over shortLib (m < 3g, hpp:381).
// Both run beside tier 1a. cmin is computed exactly as the wave kernel does: the first c with
// !((float)c / n < thr).
__device__ __forceinline__ uint32_t heavy_class(const DevIndex& X, const SearchParams& P, uint32_t m) {
    if (m == kQueryWildcard || m == 0 || m <= X.full_scan_len) return 0;
    const uint32_t n = m - X.gsz + 1;
    if (n > kWaveMaxGrams || P.limit > kWaveMaxLimit) return 0;  // tier 2
    if (m < X.short_query_len && X.n_short) return 2;
    const float fn = (float)n;
    uint32_t cmin = 1000u;
    for (uint32_t c = n; c >= 1; --c)
        if (!((float)c / fn < P.thr)) cmin = c;
    if (cmin > kHeavyCmin) return 0;
    return 1;
}

// ---------------------------------------------------------------- normalisation ------
// Four queries per wave, 16 lanes each (one query per wave spent 50 us on 65,536 waves of a few
// dependent loads): 16-lane windows of the wave's ballots find the first / last character that
// survives escape + trim; the window loops run while any query of the wave still searches.
__global__ __launch_bounds__(64) void k_prep(const uint8_t* __restrict__ raw, const uint64_t* __restrict__ off,
                                             uint32_t B, SearchParams P, uint8_t* __restrict__ qnorm,
                                             uint32_t* __restrict__ qm, uint32_t cs, DevIndex X,
                                             uint32_t* __restrict__ slots, uint32_t* __restrict__ ctr, uint32_t cap) {
    const uint32_t lane = threadIdx.x, gl = lane & 15u, sh = lane & 48u;
    const uint32_t q = blockIdx.x * 4 + (lane >> 4);
    const bool live = q < B;
    if (P.zero_stats) {
        for (uint32_t i = blockIdx.x * 64 + lane; i < P.zero_words; i += gridDim.x * 64) P.zero_stats[i] = 0;
        // the path counts, but not word 6 (*oflow), which other blocks of this launch may set: the host
        // resets it (it is zero unless a call reran for the query buffer)
        if (blockIdx.x == 0 && lane < 16 && lane != 6) P.zero_stats[kStatSlots * 16 + lane] = 0;
    }
    const uint8_t* rq = raw;  // query q: characters of cs bytes from byte offset off[q]
    uint8_t* nq = qnorm;
    uint64_t n = 0;
    bool over = false;
    if (live) {
        rq = raw + off[q];
        nq = qnorm + off[q];
        n = (off[q + 1] - off[q]) / cs;
        if (gl == 0 && P.esn) P.esn[q] = kNoEmit;  // set by tier 1a when it finishes the query (DEFER)
        if (gl == 0 && P.eovf) P.eovf[q] = 0;        // no arena blocks yet
        over = off[q + 1] > P.qcap;  // the normalised bytes would not fit: the host reruns the call
        if (over) {
            if (gl == 0) atomicOr(P.oflow, 1u);
            n = 0;
        }
    }
    const bool wild = live && !over && (n == 0 || (n == 1 && char_at(rq, 0, cs) == '*'));  // nGramSearch.hpp:356
    uint64_t first = n, last = 0;
    bool seek = live && !wild;
    for (uint64_t base = 0; __ballot(seek); base += 16) {
        const uint64_t i = base + gl;
        const bool keep = seek && i < n && !dev_space(esc_cs(P.valid, char_at(rq, i, cs), cs));
        const uint32_t bal = (uint32_t)(__ballot(keep) >> sh) & 0xFFFFu;
        if (seek && bal) {
            first = base + __ffs(bal) - 1;
            seek = false;
        } else if (base + 16 >= n) {
            seek = false;
        }
    }
    const bool empty = live && !wild && first == n;  // nothing left after escape + trim, hpp:374-375
    seek = live && !wild && !empty;
    for (uint64_t base = 0; __ballot(seek); base += 16) {
        const uint64_t i = n - 1 - (base + gl);
        const bool keep = seek && base + gl < n && !dev_space(esc_cs(P.valid, char_at(rq, i, cs), cs));
        const uint32_t bal = (uint32_t)(__ballot(keep) >> sh) & 0xFFFFu;
        if (seek && bal) {
            last = n - 1 - (base + __ffs(bal) - 1);
            seek = false;
        } else if (base + 16 >= n) {
            seek = false;
        }
    }
    const uint64_t m = live && !wild && !empty ? last - first + 1 : 0;
    for (uint64_t i = gl; i < m; i += 16) {
        const uint32_t c = dev_upper(esc_cs(P.valid, char_at(rq, first + i, cs), cs));
        if (cs == 4) reinterpret_cast<uint32_t*>(nq)[i] = c; else nq[i] = (uint8_t)c;
    }
    if (live && gl == 0) {
        if (wild) {
            qm[q] = kQueryWildcard;
        } else if (empty) {
            qm[q] = 0;
        } else {
            const uint32_t mq = (uint32_t)(m > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : m);
            qm[q] = mq;
            // heavy / full lists: 64 slot lists with a counter line each (one counter for the
            // whole batch serialised 3,900 atomics at one address: 57 against 15 us), merged by k_lists
            const uint32_t hk = slots ? heavy_class(X, P, mq) : 0u;
            if (hk) {
                const uint32_t sl = (hk - 1) * kListSlots + (q & (kListSlots - 1));
                slots[(size_t)sl * cap + atomicAdd(&ctr[16 * sl], 1u)] = q;
            }
        }
    }
}


// ---------------------------------------------------------------- shared helpers -----
// libStr = escapeBlank(key); trim; libStr == query (nGramSearch.hpp:330-334: the key is NOT
// upper-cased, so only keys already in query form promote).
__device__ bool key_equals_query(const DevIndex& X, uint32_t k, const void* q, uint32_t qcs, uint32_t m,
                                 const uint32_t* valid) {
    const uint32_t cs = X.csize;
    uint64_t a = X.key_off[k], e = X.key_off[k + 1] - 1;  // drop the NUL
    while (a < e && dev_space(esc_cs(valid, char_at(X.key_bytes, a, cs), cs))) ++a;
    while (e > a && dev_space(esc_cs(valid, char_at(X.key_bytes, e - 1, cs), cs))) --e;
    if (e - a != m) return false;
    for (uint32_t i = 0; i < m; ++i)
        if (esc_cs(valid, char_at(X.key_bytes, a + i, cs), cs) != char_at((const uint8_t*)q, i, qcs)) return false;
    return true;
}

// The (key, weight) pairs [p, pe) of survivor term t (calcScore, nGramSearch.hpp:318-336), or none
// when not even the index's largest weight lifts the term's score s into the running top-L: every
// pair scores max(w * s, 0) <= max(w_max * s, 0) in fp32, and a record enters only below tau. (A
// term that can promote an exact match, s > 0.999, is never pruned.) At threshold 0 most survivors share one gram
// with the query and are dropped here without a load.
__device__ __forceinline__ void term_pairs(const DevIndex& X, uint32_t t, float s, bool promo, uint64_t tau,
                                           uint32_t& p, uint32_t& pe) {
    if (!promo && tau != kNoCand) {
        const float ub = X.w_max * s;
        const uint32_t ub_enc = ub > 0.0f ? __float_as_uint(ub) + 1u : 1u;
        if (ub_enc < ~(uint32_t)(tau >> 32)) {
            p = pe = 0;
            return;
        }
    }
    if (X.tk_identity) {
        p = t;
        pe = t + 1;
    } else {
        p = X.tk_off[t];
        pe = X.tk_off[t + 1];
    }
}

// stringMatch (nGramSearch.hpp:182-222): min over source substrings of the edit distance to q
// (m <= 8), returned as m - distance, by Myers' bit-vector algorithm (J. ACM 46(3), 1999) in its
// approximate-matching form: bit i of the vertical deltas is row i + 1 of the DP column; a free start in the source is
// a zero carried into the horizontal deltas, the score tracks the last row (the query's end), and
// its minimum over the columns is the free end. peq[c] holds the query positions holding
// character c (c < 256; others are compared with qc); ~16 operations per source character
// against ~50 for a column DP. Tested against a column DP (200k random pairs, round 2) and the
// reference's through the oracle (tests/test_gpu_parity.py short corpora, test_oracle_golden.py).
template <typename TT>
__device__ __forceinline__ uint32_t myers_match_t(const uint8_t* peq, const uint32_t (&qc)[8], uint32_t m,
                                                  const TT* s, uint32_t L) {
    const uint32_t top = 1u << (m - 1u);
    uint32_t pv = ~0u, mv = 0u, score = m, best = m;
    // byte strings are read a dword at a time, the next one in flight while the current one is
    // consumed (term_bytes is padded to whole dwords): a byte load per character was the cost
    const uint32_t* w = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(s) & ~(uintptr_t)3);
    const uint32_t skip = (uint32_t)(reinterpret_cast<uintptr_t>(s) & 3u);
    uint32_t cur = 0, nxt = 0;
    if (sizeof(TT) == 1 && L) {
        cur = w[0] >> (8u * skip);
        nxt = skip + L > 4u ? w[1] : 0u;
    }
    uint32_t avail = 4u - skip, k = 1;
    for (uint32_t j = 0; j < L; ++j) {
        uint32_t c;
        if constexpr (sizeof(TT) == 1) {
            if (!avail) {
                cur = nxt;
                avail = 4u;
                ++k;
                if (j + 4u < L) nxt = w[k];
            }
            c = cur & 255u;
            cur >>= 8;
            --avail;
        } else {
            c = s[j];
        }
        uint32_t eq;
        if (sizeof(TT) == 1 || c < 256u) {
            eq = peq[c];
        } else {
            eq = 0u;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) eq |= (i < m && qc[i] == c) ? 1u << i : 0u;
        }
        const uint32_t xv = eq | mv;
        const uint32_t xh = (((eq & pv) + pv) ^ pv) | eq;
        uint32_t ph = mv | ~(xh | pv);
        uint32_t mh = pv & xh;
        score += (ph & top) ? 1u : 0u;
        score -= (mh & top) ? 1u : 0u;
        ph <<= 1;  // row 0's horizontal delta is 0: the match may start anywhere in the source
        mh <<= 1;
        pv = mh | ~(xv | ph);
        mv = ph & xv;
        best = min(best, score);
    }
    return m - best;
}

// myers_match_t over a short narrow term (L <= 5 bytes: shortLib holds terms shorter than 2g <= 6)
// held in two dwords (x1:x0) from byte sk: its match masks read from peq all at once (five LDS reads
// in flight instead of one per character), then the recurrence; steps past L do not move `best`
__device__ __forceinline__ uint32_t myers_short(const uint8_t* peq, uint32_t m, uint32_t x0, uint32_t x1, uint32_t sk,
                                                uint32_t L) {
    const uint64_t x = (((uint64_t)x1 << 32) | x0) >> (8u * sk);
    uint32_t eq[kShortTermLen - 1];
#pragma unroll
    for (uint32_t j = 0; j + 1 < kShortTermLen; ++j) eq[j] = peq[(uint32_t)(x >> (8u * j)) & 255u];
    const uint32_t top = 1u << (m - 1u);
    uint32_t pv = ~0u, mv = 0u, score = m, best = m;
#pragma unroll
    for (uint32_t j = 0; j + 1 < kShortTermLen; ++j) {
        const uint32_t e = eq[j];
        const uint32_t xv = e | mv;
        const uint32_t xh = (((e & pv) + pv) ^ pv) | e;
        uint32_t ph = mv | ~(xh | pv);
        uint32_t mh = pv & xh;
        score += (ph & top) ? 1u : 0u;
        score -= (mh & top) ? 1u : 0u;
        ph <<= 1;
        mh <<= 1;
        pv = mh | ~(xv | ph);
        mv = ph & xv;
        best = j < L ? min(best, score) : best;
    }
    return m - best;
}

// the match-mask table of Myers' algorithm for characters < 256: peq[c] bit i = (q[i] == c);
// threads [tid0, tid0 + nthreads) of the caller fill it (the caller orders it before use)
template <class QF>
__device__ __forceinline__ void build_peq(uint8_t* peq, QF q, uint32_t m, uint32_t tid0, uint32_t nthreads) {
    for (uint32_t c = tid0; c < 256u; c += nthreads) {
        uint32_t e = 0;
        for (uint32_t i = 0; i < m && i < 8; ++i) e |= (q(i) == c) ? 1u << i : 0u;
        peq[c] = (uint8_t)e;
    }
}

// term t of the index against the query (m <= 8 characters in qc; peq its match masks)
__device__ __forceinline__ uint32_t string_match(const uint8_t* peq, const uint32_t (&qc)[8], uint32_t m,
                                                 const DevIndex& X, uint32_t t) {
    const uint64_t a = X.term_off[t], b = X.term_off[t + 1];
    if (X.csize == 4) {
        const uint32_t* s = reinterpret_cast<const uint32_t*>(X.term_bytes) + a;
        return myers_match_t(peq, qc, m, s, (uint32_t)(b - a));
    }
    const uint8_t* s = X.term_bytes + a;
    return myers_match_t(peq, qc, m, s, (uint32_t)(b - a));
}

// Gram of the query characters at position i (accessor qf), as a row of the gram space:
// the 21-bit code of three ASCII bytes (indexN), or the dictionary id of the g packed code
// points (indexG / indexW). UINT32_MAX: the gram is in no term of the index.
template <class QF>
__device__ __forceinline__ uint32_t gram_at(const DevIndex& X, QF qf, uint32_t i) {
    if (X.gram_mode == 0) {
        const uint32_t c0 = qf(i), c1 = qf(i + 1), c2 = qf(i + 2);
        return ((c0 | c1 | c2) & ~0x7Fu) ? UINT32_MAX : (c0 << 14) | (c1 << 7) | c2;
    }
    uint64_t key = 0;
    for (uint32_t j = 0; j < X.gsz; ++j) {
        const uint32_t c = qf(i + j);
        if (c > 0x1FFFFFu) return UINT32_MAX;
        key = (key << 21) | c;
    }
    const uint64_t mask = (1ull << X.ghash_bits) - 1;
    for (uint64_t h = (key * 0x9E3779B97F4A7C15ull) >> (64 - X.ghash_bits);; h = (h + 1) & mask) {
        const uint64_t k = X.ghash_key[h];
        if (k == key) return X.ghash_val[h];
        if (k == kGramEmpty) return UINT32_MAX;
    }
}

// calcScore's per-pair value (nGramSearch.hpp:326-335) as an order-preserving encoding: the
// score max(w*s, +0), or 100 for an exact match (kPromoted, an ordinary score in ScoreComparer).
// shortg: the pair's score came from the short search (searchShort, hpp:262-270). 0: the pair
// never shows: calcScore merges the short scores before the long ones (hpp:393-394) and a
// promotion overwrites what the key had, so a short pair above 100 of a key that a long term
// promotes is lost (DevIndex.kt_flag: the key has such a long term; the query is the key).
__device__ __forceinline__ uint32_t pair_enc(uint2 kw, float s, bool promo_possible, bool shortg,
                                             const DevIndex& X, const void* q, uint32_t qcs, uint32_t m,
                                             const uint32_t* valid) {
    const float sc = __uint_as_float(kw.y) * s;
    const uint32_t enc = sc > 0.0f ? __float_as_uint(sc) + 1u : 1u;  // std::max(w*s, 0.0f) (entry default)
    // one key test for both (the key is the query): promoted, or an overwritten short pair
    const bool test = promo_possible || (shortg && enc > kPromoted && X.kt_flag && X.kt_flag[kw.x]);
    if (test && key_equals_query(X, kw.x, q, qcs, m, valid)) return promo_possible ? kPromoted : 0u;
    return enc;
}

// the wildcard query's answer (nGramSearch.hpp:356-369), precomputed at index time; threads
// [tid, ...) of nthreads write it
__device__ __forceinline__ void wild_answer(const DevIndex& X, const SearchParams& P, uint32_t q, uint32_t tid,
                                            uint32_t nthreads, uint32_t* out_n, uint32_t* out_k, float* out_s) {
    const uint32_t n = min(P.limit, X.n_keys);
    const size_t ob = (size_t)q * P.out_stride;
    for (uint32_t i = tid; i < n; i += nthreads) {
        out_k[ob + i] = X.wild_key[i];
        out_s[ob + i] = X.wild_score[i];
    }
    if (tid == 0) out_n[q] = n;
}

// searchLong's lists (nGramSearch.hpp:278-301): the query's gram occurrences with postings,
// compacted to lanes 0..ng-1 (a gram repeated k times owns k lanes: counts with multiplicity), each
// with its posting range and skip-table row. Every wave that calls it computes the same plan.
template <class QF>
__device__ __forceinline__ uint32_t gram_lists(const DevIndex& X, QF qch, uint32_t n, uint32_t lane, uint64_t& gbase,
                                               uint32_t& glen, uint32_t& grow) {
    gbase = 0;
    glen = grow = 0;
    bool have = false;
    if (lane < n) {
        const uint32_t code = gram_at(X, qch, lane);
        if (code != UINT32_MAX) {
            gbase = X.gram_off[code];
            glen = (uint32_t)(X.gram_off[code + 1] - gbase);
            grow = X.gram_row[code];
            have = glen != 0;
        }
    }
    const unsigned long long hb = __ballot(have);
    const uint32_t ng = __popcll(hb);
    uint32_t src = 0;
    unsigned long long rest = hb;
    for (uint32_t k = 0; k <= lane && rest; ++k) {  // lane k takes the k-th set bit
        src = __ffsll((long long)rest) - 1;
        rest &= rest - 1;
    }
    const uint64_t b2 = __shfl(gbase, (int)src);
    const uint32_t l2 = __shfl(glen, (int)src), r2 = __shfl(grow, (int)src);
    gbase = lane < ng ? b2 : 0;
    glen = lane < ng ? l2 : 0;
    grow = lane < ng ? r2 : 0;
    return ng;
}

// ---------------------------------------------------------------- fused kernel -------
struct FastSmem {
    uint32_t table[kTableSlots];   // (term - lo + 1) << 8 | count
    uint64_t cand[kCandCap];       // (~enc) << 32 | key
    uint64_t g_base[256];          // per distinct gram: start of its posting list
    uint64_t g_cur[256];           // first posting of the current part
    uint64_t g_end[256];           // end of the current bucket range
    uint64_t g_stop[256];          // end of the current part's segment
    uint32_t g_row[256];           // skip-table row
    uint32_t g_mult[256];          // multiplicity of the gram in the query
    uint32_t g_code[256];
    uint32_t btot[kMaxBuckets];    // postings per term-id bucket
    uint2 part[kMaxBuckets];       // parts: bucket range [x, y & 0x7fffffff), y >> 31 = oversized
    uint32_t pre[260];             // segment prefix sums
    uint32_t q[264];               // the normalised query, one character (byte or code point) per entry
    uint8_t peq[256];              // Myers match masks of the query (short search)
    uint64_t tau;                  // records >= tau cannot enter the top-L
    uint64_t p_left;
    unsigned long long seg_total;
    uint32_t ng, cand_n, n_valid, survivors;
    uint32_t nparts, pad1, pad2, pad3;
};

__device__ __forceinline__ uint32_t next_pow2(uint32_t x) { return x <= 1 ? 1u : 1u << (32 - __clz(x - 1)); }

__device__ void bitonic_sort(uint64_t* a, uint32_t n) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t p = tid; p < n / 2; p += kFastThreads) {
                const uint32_t i = ((p & ~(j - 1u)) << 1) | (p & (j - 1u)), l = i + j;  // j is a power of two
                const uint64_t x = a[i], y = a[l];
                if ((x > y) == ((i & k) == 0)) { a[i] = y; a[l] = x; }
            }
            __syncthreads();
        }
    }
}

// Merge the buffer: keep each key's best record, then the best L records in order.
// The running top-L with max-merge is exact: a record evicted here is beaten by L other keys
// whose scores can only grow.
__device__ void flush(FastSmem& S, uint32_t L) {
    const uint32_t tid = threadIdx.x;
    __syncthreads();
    const uint32_t n = min(S.cand_n, (uint32_t)kCandCap);
    const uint32_t P2 = next_pow2(max(n, 2u));
    for (uint32_t i = tid; i < P2; i += kFastThreads) {
        const uint64_t r = i < n ? S.cand[i] : kNoCand;
        S.cand[i] = i < n ? ((r << 32) | (r >> 32)) : kNoCand;  // key-major for the dedup
    }
    if (tid == 0) S.n_valid = 0;
    __syncthreads();
    bitonic_sort(S.cand, P2);
    uint64_t keep[kCandCap / kFastThreads];
#pragma unroll
    for (int u = 0; u < kCandCap / kFastThreads; ++u) {
        const uint32_t i = tid + u * kFastThreads;
        keep[u] = kNoCand;
        if (i < P2) {
            const uint64_t d = S.cand[i];
            if (d != kNoCand && (i == 0 || (S.cand[i - 1] >> 32) != (d >> 32))) keep[u] = (d << 32) | (d >> 32);
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kCandCap / kFastThreads; ++u) {
        const uint32_t i = tid + u * kFastThreads;
        if (i < P2) S.cand[i] = keep[u];
    }
    __syncthreads();
    bitonic_sort(S.cand, P2);
    for (uint32_t i = tid; i < P2; i += kFastThreads)
        if (S.cand[i] != kNoCand && (i + 1 == P2 || S.cand[i + 1] == kNoCand)) S.n_valid = i + 1;
    __syncthreads();
    if (tid == 0) {
        const uint32_t nv = S.n_valid;
        S.cand_n = min(nv, L);
        S.tau = nv >= L ? S.cand[L - 1] : kNoCand;
    }
    __syncthreads();
}

struct EmitState {
    uint32_t p, pe;  // pending (key, weight) pairs of the current term
    float s;
    bool promo;
    bool shortg;     // the term's score is a short-search one
};

// Appends the pending pairs; false = buffer full (the pair is retried after a flush).
__device__ __forceinline__ bool emit_pending(EmitState& st, FastSmem& S, const DevIndex& X, uint64_t tau,
                                             uint32_t m, const uint32_t* valid) {
    while (st.p < st.pe) {
        const uint2 kw = X.tk[st.p];
        const uint32_t enc = pair_enc(kw, st.s, st.promo, st.shortg, X, S.q, 4u, m, valid);
        const uint64_t rec = ((uint64_t)(~enc) << 32) | kw.x;
        if (enc && rec < tau) {
            const uint32_t idx = atomicAdd(&S.cand_n, 1u);
            if (idx >= (uint32_t)kCandCap) return false;
            S.cand[idx] = rec;
        }
        ++st.p;
    }
    return true;
}

// Drives a per-thread stream of scored terms through calcScore into the buffer, flushing
// whenever any thread finds it full. next(st) -> 0 exhausted, 1 term loaded into st, 2 skip.
template <class Next>
__device__ void produce(FastSmem& S, const DevIndex& X, const SearchParams& P, uint32_t m, uint32_t L,
                        unsigned* err, Next next) {
    EmitState st{0, 0, 0.0f, false, false};
    bool done = false;
    for (uint32_t rounds = 0;; ++rounds) {
        bool full = false;
        const uint64_t tau = S.tau;
        while (!full) {
            if (st.p < st.pe && !emit_pending(st, S, X, tau, m, P.valid)) { full = true; break; }
            if (done) break;
            const int r = next(st);
            if (r == 0) done = true;
        }
        if (!__syncthreads_or(full)) break;
        flush(S, L);
        if (rounds > (1u << 24)) {  // each flush frees >= kCandCap - L slots: unreachable
            if (threadIdx.x == 0) atomicOr(err, 2u);
            break;
        }
    }
}

__device__ __forceinline__ void table_insert(uint32_t* T, uint32_t rel, uint32_t mult, unsigned* err) {
    uint32_t probes = 0;
    uint32_t h = (rel * 0x9E3779B1u) >> (32 - 13);
    static_assert(kTableSlots == 1 << 13, "hash width");
    const uint32_t want = rel << 8;
    for (;;) {
        uint32_t cur = T[h];
        if (cur == 0) {
            const uint32_t prev = atomicCAS(&T[h], 0u, want | mult);
            if (prev == 0) return;
            cur = prev;
        }
        if ((cur >> 8) == rel) {
            atomicAdd(&T[h], mult);
            return;
        }
        h = (h + 1) & (kTableSlots - 1);
        if (++probes > (uint32_t)kTableSlots) {  // cannot happen at <= 50 % load; never spin
            atomicOr(err, 1u);
            return;
        }
    }
}

// Sum of one value per thread for threads < 256 (waves 0..3) into *dst (zeroed by caller).
__device__ __forceinline__ void small_sum(uint64_t v, unsigned long long* dst) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && threadIdx.x < 256 && v) atomicAdd(dst, (unsigned long long)v);
}

// One term-id part of searchLong: the segments [g_cur, g_stop) of every distinct gram hold
// the postings with term ids in [lo, lo + span) (span < 2^24). Counts them in the LDS table
// (<= 50 % load), then scans the table: s = count / n, threshold, calcScore.
__device__ void long_part(FastSmem& S, const DevIndex& X, const SearchParams& P, uint32_t m, uint32_t n,
                          uint32_t L, uint32_t lo, uint32_t ng, uint32_t& surv, unsigned* err,
                          unsigned long long& tp_) {
    const uint32_t tid = threadIdx.x;
    // segment prefix sums (wave 0; ng <= 255 -> 4 entries per lane)
    if (tid < 64) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t g = tid * 4 + u;
            v[u] = g < ng ? (uint32_t)(S.g_stop[g] - S.g_cur[g]) : 0u;
            sum += v[u];
        }
        uint32_t incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)tid >= o) incl += y;
        }
        uint32_t run = incl - sum;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            S.pre[tid * 4 + u] = run;
            run += v[u];
        }
        if (tid == 63) S.pre[256] = incl;
    }
    __syncthreads();
    STAMP(6);
    const uint32_t total = S.pre[ng];
    // count: every posting of the part into the LDS table (4 loads in flight per thread)
    {
        uint32_t g = 0;
        for (uint32_t j0 = tid; j0 < total; j0 += 4 * kFastThreads) {
            uint32_t tt[4], mu[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t j = j0 + u * kFastThreads;
                mu[u] = 0;
                if (j < total) {
                    while (S.pre[g + 1] <= j) ++g;
                    tt[u] = X.post[S.g_cur[g] + (j - S.pre[g])];
                    mu[u] = S.g_mult[g];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (mu[u]) table_insert(S.table, tt[u] - lo + 1u, mu[u], err);
        }
    }
    __syncthreads();
    STAMP(7);
    // extract: s = count / n, threshold, calcScore; the scan also clears the table
    uint32_t i = 0;
    const float fn = (float)n;
    produce(S, X, P, m, L, err, [&](EmitState& st) -> int {
        if (i >= (uint32_t)(kTableSlots / kFastThreads)) return 0;
        const uint32_t slot = tid + i * kFastThreads;
        ++i;
        const uint32_t v = S.table[slot];
        if (!v) return 2;
        S.table[slot] = 0;
        const uint32_t t = X.n_short + lo + (v >> 8) - 1u;
        const float s = (float)(v & 255u) / fn;  // nGramSearch.hpp:300
        if (s < P.thr) return 2;                 // nGramSearch.hpp:315
        ++surv;
        st.s = s;
        st.promo = (double)s > 0.999;            // nGramSearch.hpp:328
        st.shortg = false;
        term_pairs(X, t, s, st.promo, S.tau, st.p, st.pe);
        return 1;
    });
    STAMP(8);
}

// Tier 2: one 512-thread block per query (queries of up to 255 grams, limits up to 1024).
__device__ void fast_one(const uint32_t q, FastSmem& S, const DevIndex& X, const SearchParams& P,
                         const uint8_t* __restrict__ qnorm, const uint64_t* __restrict__ qoff,
                         const uint32_t* __restrict__ qm, uint32_t* __restrict__ out_n, uint32_t* __restrict__ out_k,
                         float* __restrict__ out_s, uint32_t* __restrict__ glist, uint32_t* __restrict__ gcount,
                         DevStats* __restrict__ stats) {
    const uint32_t tid = threadIdx.x;
    unsigned long long tp_ = 0;
#ifdef NGS_PHASE_STAMPS
    if (tid == 0) tp_ = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t m = qm[q];
    const uint32_t L = P.limit;
    const size_t ob = (size_t)q * P.out_stride;

    if (m == kQueryWildcard) {  // nGramSearch.hpp:356-369
        wild_answer(X, P, q, tid, kFastThreads, out_n, out_k, out_s);
        return;
    }
    if (m == 0) {
        if (tid == 0) out_n[q] = 0;
        return;
    }
    // every index shape: grams of g characters (bytes or code points), looked up by gram_at (the
    // 21-bit code of indexN, the dictionary of indexG / indexW); the full-library scan (m <= g)
    // and what exceeds the block's tables go to the general path
    if (m <= X.full_scan_len || m - X.gsz + 1 > kFastMaxGrams || L > kFastMaxLimit) {
        if (tid == 0) glist[atomicAdd(gcount, 1u)] = q;  // library-wide path
        return;
    }
    const uint32_t n = m - X.gsz + 1;
    const uint32_t n_long = X.n_terms - X.n_short;
    const uint8_t* qg = qnorm + qoff[q];
    for (uint32_t i = tid; i < m; i += kFastThreads) S.q[i] = char_at(qg, i, X.csize);
    for (uint32_t i = tid; i < (uint32_t)kTableSlots; i += kFastThreads) S.table[i] = 0;
    if (tid == 0) {
        S.cand_n = 0;
        S.tau = kNoCand;
        S.ng = 0;
        S.seg_total = 0;
        S.survivors = 0;
    }
    __syncthreads();
    STAMP(0);

    uint32_t surv = 0;  // terms of this thread that passed the threshold (stats only)

    // ---- searchShort over shortLib (nGramSearch.hpp:262-270), 4 <= m < 9 ----
    if (m < X.short_query_len && X.n_short) {
        uint32_t qc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) qc[i] = (uint32_t)i < m ? S.q[i] : 0;
        build_peq(S.peq, [&](uint32_t i) { return S.q[i]; }, m, tid, kFastThreads);
        __syncthreads();
        uint32_t t = tid;
        const float fm = (float)m;
        produce(S, X, P, m, L, &stats->errors, [&](EmitState& st) -> int {
            if (t >= X.n_short) return 0;
            const uint32_t match = string_match(S.peq, qc, m, X, t);
            const float s = (float)match / fm;  // nGramSearch.hpp:244
            const uint32_t id = t;
            t += kFastThreads;
            if (s < P.thr) return 2;  // nGramSearch.hpp:315
            ++surv;
            st.s = s;
            st.promo = (double)s > 0.999;
            st.shortg = true;
            term_pairs(X, id, s, st.promo, S.tau, st.p, st.pe);
            return 1;
        });
    }

    STAMP(1);
    // ---- searchLong (nGramSearch.hpp:278-301) ----
    // distinct grams with multiplicity
    if (tid < n) S.g_code[tid] = gram_at(X, [&](uint32_t i) { return S.q[i]; }, tid);  // UINT32_MAX: no list
    if (tid < kMaxBuckets) S.btot[tid] = 0;
    __syncthreads();
    uint64_t my_len = 0;
    if (tid < n) {
        const uint32_t g = S.g_code[tid];
        bool first = true;
        uint32_t mult = 0;
        for (uint32_t j = 0; j < n; ++j) {
            if (S.g_code[j] == g) {
                first &= j >= tid;
                ++mult;
            }
        }
        if (first && g != 0xFFFFFFFFu) {
            const uint64_t a = X.gram_off[g], b = X.gram_off[g + 1];
            if (b > a) {
                const uint32_t slot = atomicAdd(&S.ng, 1u);
                S.g_base[slot] = a;
                S.g_row[slot] = X.gram_row[g];
                S.g_mult[slot] = mult;
                my_len = b - a;
            }
        }
    }
    small_sum(my_len, &S.seg_total);
    __syncthreads();
    STAMP(2);
    const uint32_t ng = S.ng;
    const uint64_t p_total = S.seg_total;
    // tier 2 plans over at most kMaxBuckets buckets: every kst-th boundary of the skip table
    // (the index may hold more, power-of-two many, for dense lists)
    const uint32_t kst = X.n_buckets > kMaxBuckets ? X.n_buckets / kMaxBuckets : 1u;
    const uint32_t K = X.n_buckets / kst, span = X.bucket_span * kst, KS = X.n_buckets;
    // postings per term-id bucket, straight from the skip table
    const bool one_part = p_total <= (uint64_t)kPartCap && n_long <= kMaxPartSpan;
    if (!one_part) {
        for (uint32_t idx = tid; idx < ng * K; idx += kFastThreads) {
            const uint32_t g = idx / K, b = idx - g * K;
            const uint32_t* sk = X.skip + (size_t)S.g_row[g] * (KS + 1);
            const uint32_t c = sk[(b + 1) * kst] - sk[b * kst];
            if (c) atomicAdd(&S.btot[b], c);
        }
    }
    __syncthreads();
    STAMP(3);
    // greedy cut of the bucket sequence into parts of <= kPartCap postings (<= 50 % table load);
    // a bucket alone above the cap becomes an "oversized" part, split by term id below
    if (tid == 0) {
        uint32_t np = 0;
        if (one_part) {
            if (p_total) S.part[np++] = make_uint2(0, K);
        } else {
            uint32_t b = 0;
            while (b < K) {
                if (S.btot[b] > (uint32_t)kPartCap || span > kMaxPartSpan) {
                    if (S.btot[b]) S.part[np++] = make_uint2(b, (b + 1) | 0x80000000u);
                    ++b;
                    continue;
                }
                const uint32_t blo = b;
                uint32_t tot = 0;
                while (b < K && tot + S.btot[b] <= (uint32_t)kPartCap &&
                       (uint64_t)(b + 1 - blo) * span <= kMaxPartSpan) tot += S.btot[b++];
                if (tot) S.part[np++] = make_uint2(blo, b);
            }
        }
        S.nparts = np;
    }
    __syncthreads();
    STAMP(4);
    const uint32_t nparts = S.nparts;
    for (uint32_t pi = 0; pi < nparts; ++pi) {
        const uint2 pr = S.part[pi];
        const bool over = pr.y >> 31;
        const uint32_t blo = pr.x, bhi = pr.y & 0x7FFFFFFFu;
        const uint32_t lo_id = blo * span;
        const uint32_t hi_id = (uint32_t)min64((uint64_t)bhi * span, n_long);
        if (tid < ng) {
            const uint32_t* sk = X.skip + (size_t)S.g_row[tid] * (KS + 1);
            S.g_cur[tid] = S.g_base[tid] + sk[blo * kst];
            S.g_end[tid] = S.g_base[tid] + sk[bhi * kst];
        }
        __syncthreads();
        STAMP(5);
        if (!over) {
            if (tid < ng) S.g_stop[tid] = S.g_end[tid];
            __syncthreads();
            long_part(S, X, P, m, n, L, lo_id, ng, surv, &stats->errors, tp_);
            continue;
        }
        // oversized bucket: adaptive term-id sub-parts, lower_bound per list (rare)
        uint32_t sub_lo = lo_id;
        uint32_t step = (uint32_t)max64(1, min64((uint64_t)(hi_id - lo_id) * (kPartCap * 3 / 4) / S.btot[blo],
                                                  kMaxPartSpan));
        for (uint32_t guard = 0; sub_lo < hi_id; ++guard) {
            if (guard > hi_id - lo_id + 1u) {
                if (tid == 0) atomicOr(&stats->errors, 4u);
                break;
            }
            uint32_t hi = 0;
            for (uint32_t tries = 0;; ++tries) {
                hi = (uint32_t)min64(hi_id, (uint64_t)sub_lo + step);
                __syncthreads();
                if (tid == 0) S.seg_total = 0;
                __syncthreads();
                uint64_t cnt = 0;
                if (tid < ng) {
                    uint64_t a = S.g_cur[tid], b = S.g_end[tid];
                    while (a < b) {  // lower_bound(post[cur..end), hi)
                        const uint64_t mid = (a + b) >> 1;
                        if (X.post[mid] < hi) a = mid + 1; else b = mid;
                    }
                    S.g_stop[tid] = a;
                    cnt = a - S.g_cur[tid];
                }
                small_sum(cnt, &S.seg_total);
                __syncthreads();
                const uint64_t seg = S.seg_total;
                if (seg <= (uint64_t)kPartCap || hi - sub_lo <= 1 || tries > 64) {
                    step = (uint32_t)max64(1, min64(seg ? (uint64_t)(hi - sub_lo) * (kPartCap * 3 / 4) / seg
                                                        : (uint64_t)(hi - sub_lo) * 4, kMaxPartSpan));
                    break;
                }
                step = (uint32_t)max64(1, min64((uint64_t)(hi - sub_lo) * (kPartCap * 3 / 4) / seg, kMaxPartSpan));
            }
            long_part(S, X, P, m, n, L, sub_lo, ng, surv, &stats->errors, tp_);
            if (tid < ng) S.g_cur[tid] = S.g_stop[tid];
            __syncthreads();
            sub_lo = hi;
        }
    }

    if (surv) atomicAdd(&S.survivors, surv);
    STAMP(9);
    flush(S, L);
    STAMP(10);
    const uint32_t nres = S.cand_n;
    for (uint32_t i = tid; i < nres; i += kFastThreads) {
        const uint64_t r = S.cand[i];
        const uint32_t enc = ~(uint32_t)(r >> 32);
        out_k[ob + i] = (uint32_t)r;
        out_s[ob + i] = __uint_as_float(enc - 1u);
    }
    if (tid == 0) {
        out_n[q] = nres;
        DevStats* sl = stats + (q & (kStatSlots - 1));
        atomicAdd(&sl->postings, (unsigned long long)p_total);
        atomicAdd(&sl->lists, (unsigned long long)ng);
        atomicAdd(&sl->results, (unsigned long long)nres);
        atomicAdd(&sl->fast, 1ull);
        atomicAdd(&sl->survivors, (unsigned long long)S.survivors);
    }
    STAMP(11);
}

__global__ __launch_bounds__(kFastThreads) void k_fast(DevIndex X, SearchParams P, const uint8_t* __restrict__ qnorm,
                                                       const uint64_t* __restrict__ qoff,
                                                       const uint32_t* __restrict__ qm, uint32_t* __restrict__ out_n,
                                                       uint32_t* __restrict__ out_k, float* __restrict__ out_s,
                                                       const uint32_t* __restrict__ qlist,
                                                       const uint32_t* __restrict__ qcount,
                                                       uint32_t* __restrict__ glist, uint32_t* __restrict__ gcount,
                                                       DevStats* __restrict__ stats) {
    __shared__ FastSmem S;
    const uint32_t cnt = *qcount;
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        fast_one(qlist[i], S, X, P, qnorm, qoff, qm, out_n, out_k, out_s, glist, gcount, stats);
        __syncthreads();
    }
}

// ---------------------------------------------------------------- wave kernel --------
// Tier 1: ONE WAVE PER QUERY with a wave-private LDS table. A query's gram lists are cut into
// term-id parts of <= kWaveChunks 16-byte chunks (bucket skip table; a bucket above the cap is
// split by lower_bound); the wave loads a part into registers, the lists' chunks packed across
// its lanes, while the previous part is counted against the LDS sketch / hash table with
// predication only. A repeated query gram is kept as a separate occurrence (its list is read once
// per occurrence), which is the reference's multiplicity (hpp:289-298). (Two and four waves per
// query sharing one table were measured slower and are gone.)
// LDS table geometry: tier 1a keeps 4 KB (occupancy), the full kernel 8 KB (its occupancy is
// set by VGPRs; a bigger sketch means fewer false candidates on the heavy queries it runs)
template <bool LEAN>
struct TableGeom {
    static constexpr int kBits = LEAN ? kWaveSlotBits : kFullSlotBits;
    static constexpr int kSlots = 1 << kBits;  // u32 words: exact hash slots, or 8 u4 sketch cells each
    static constexpr int kCap = kSlots / 2;    // entries per exact-count pass (<= 50 % load)
};

template <bool LEAN = false>
struct alignas(16) WaveSmem {
    uint32_t table[TableGeom<LEAN>::kSlots];  // exact: (term - lo + 1) << 8 | count; sketch: 8 x u4 counters
    uint64_t cand_own[LEAN ? 1 : kWaveCand];  // (~enc) << 32 | key
    // the candidate buffer; tier 1a (LEAN) fills it only after the part loop, over the dead table
    __device__ __forceinline__ uint64_t* cand() {
        if constexpr (LEAN) return reinterpret_cast<uint64_t*>(table);
        else return cand_own;
    }
    uint2 segtab[64];                // staging: per list {first chunk - position, first | end entry << 16}
    uint8_t mark[kWaveChunks];       // staging: list index + 1 at the position of its first chunk
    unsigned long long lstart[kDmaRounds];  // tier 1a staging: bit (pre - 1) per list start, 64 chunk positions a word
    uint32_t g4[LEAN ? 64 : 1];      // tier 1a: per list lane, the 16-byte chunk of its list's first posting
    uint32_t surv_t[kWaveSurv];      // survivor terms
    uint32_t cbuf[64];               // sketch candidates (terms)
    uint8_t surv_c[kWaveSurv];       // hit count, | 0x80 for a Levenshtein (short search) match count
    uint32_t q[kWaveMaxGrams + 8];   // normalised query, one code point per entry
    uint8_t peq[LEAN ? 4 : 256];     // tier 1b: Myers match masks of the query (short search)
    uint32_t surv_total;             // stats
    uint32_t ncand;                  // (unused by tier 1b)
    uint32_t x_surv_n, x_cand_n;     // tier 1a: arena blocks chained (spill_arena)
    uint32_t xcnt;                   // ... and the one before the last
    uint64_t x_tau;
};

static_assert(kWaveSlots * 4 >= kWaveCand * 8, "tier 1a keeps the candidate buffer in the table");
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

constexpr uint32_t kQueryInGlobal = 0xFFFFFFFEu;  // wave_query: read the query from qnorm / qoff / qm

// popcount of the ballot bits of the lanes below this one (v_mbcnt_lo/hi)
__device__ __forceinline__ uint32_t rank_below(unsigned long long b) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// Ordering point for the wave-private LDS. A wave's LDS instructions execute in order, so
// no barrier and no wait is needed: only keep the compiler from moving LDS accesses across.
// (__syncthreads() would also drain every outstanding global load.)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int Ctrl>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, 0xf, 0xf, false);
}

// Wave-uniform u32 sum in DPP steps (quad perms, row rotations, row broadcasts) instead of
// six dependent ds_bpermute round trips; the total is read from lane 63 into an SGPR.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += dpp_mov<0xb1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4e>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x124>(v);  // row_ror:4
    v += dpp_mov<0x128>(v);  // row_ror:8
    v += dpp_mov<0x142>(v);  // row_bcast:15
    v += dpp_mov<0x143>(v);  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

template <int Ctrl, int RowMask>
__device__ __forceinline__ uint32_t dpp_mov_rows(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, RowMask, 0xf, false);
}

// Inclusive prefix sum across the wave: row shifts within each 16-lane row, then the row
// broadcasts carry rows 0 -> 1, 2 -> 3 and (0..1) -> (2..3). Lanes without a source add 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += dpp_mov_rows<0x111, 0xf>(v);  // row_shr:1
    v += dpp_mov_rows<0x112, 0xf>(v);  // row_shr:2
    v += dpp_mov_rows<0x114, 0xf>(v);  // row_shr:4
    v += dpp_mov_rows<0x118, 0xf>(v);  // row_shr:8
    v += dpp_mov_rows<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v += dpp_mov_rows<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

// Inclusive prefix max across the wave, same DPP steps.
__device__ __forceinline__ uint32_t wave_incl_max_scan(uint32_t v) {
    v = max(v, dpp_mov_rows<0x111, 0xf>(v));
    v = max(v, dpp_mov_rows<0x112, 0xf>(v));
    v = max(v, dpp_mov_rows<0x114, 0xf>(v));
    v = max(v, dpp_mov_rows<0x118, 0xf>(v));
    v = max(v, dpp_mov_rows<0x142, 0xa>(v));
    v = max(v, dpp_mov_rows<0x143, 0xc>(v));
    return v;
}

// OR of v over the wave (the inclusive-scan steps of wave_incl_scan; lane 63 holds the total)
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    v |= dpp_mov_rows<0x111, 0xf>(v);
    v |= dpp_mov_rows<0x112, 0xf>(v);
    v |= dpp_mov_rows<0x114, 0xf>(v);
    v |= dpp_mov_rows<0x118, 0xf>(v);
    v |= dpp_mov_rows<0x142, 0xa>(v);
    v |= dpp_mov_rows<0x143, 0xc>(v);
    return __builtin_amdgcn_readlane(v, 63);
}

// Radix select of the limit cutoff (hpp:397-401 keeps the first L of the ScoreComparer order):
// the buffer's n >= L records (all distinct: DevIndex.keys_unique, one record per key) are
// trimmed to the L smallest, unsorted, and tau becomes the L-th. The records sit in registers (4
// per lane); each pass histograms one 8-bit digit of the records still tied with the L-th (a
// 256-bin LDS histogram over the buffer's own first KB), taken just below the highest bit in
// which those records differ (OR / AND-NOT reductions), so equal score bits cost no pass; the
// boundary bin's prefix sum fixes 8 more bits of the L-th record, until one record is left. At
// threshold 0 (thousands of equal-score survivors, C2) this replaces a 256-record bitonic sort
// per buffer refill with ~3 histogram passes; the final order comes from one sort of the L.
template <class SM>
__device__ void wave_select(SM& S, uint32_t& cand_n, uint64_t& tau, uint32_t L) {
    static_assert(kWaveCand == 256, "wave_select holds the buffer as 4 records per lane");
    const uint32_t lane = lane_id();
    const uint32_t n = min(cand_n, (uint32_t)kWaveCand);
    uint64_t r[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) r[u] = lane + 64 * u < n ? S.cand()[lane + 64 * u] : kNoCand;
    wave_sync();  // the buffer is free: its first KB holds the histogram
    uint32_t* hist = reinterpret_cast<uint32_t*>(S.cand());
    uint64_t pre = 0, pm = 0;  // bits of the L-th record fixed so far (mask pm)
    uint32_t k = L;            // rank of the L-th record among the records matching pre
    uint64_t kth = kNoCand;
    for (;;) {
        uint32_t o_lo = 0, o_hi = 0, z_lo = 0, z_hi = 0;  // OR of the matches and of their complements
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            if (lane + 64 * u < n && (r[u] & pm) == pre) {
                o_lo |= (uint32_t)r[u];
                o_hi |= (uint32_t)(r[u] >> 32);
                z_lo |= ~(uint32_t)r[u];
                z_hi |= ~(uint32_t)(r[u] >> 32);
            }
        }
        const uint64_t o = ((uint64_t)wave_or_u32(o_hi) << 32) | wave_or_u32(o_lo);
        const uint64_t a = ~(((uint64_t)wave_or_u32(z_hi) << 32) | wave_or_u32(z_lo));  // AND of the matches
        const uint64_t d = o ^ a;  // bits in which the matching records differ
        if (!d) {                  // one record left: the L-th
            kth = o;
            break;
        }
        const uint32_t top = 63u - (uint32_t)__clzll((long long)d);
        const uint32_t sh = top >= 7u ? top - 7u : 0u;
        const uint64_t above = top == 63u ? 0ull : ~((2ull << top) - 1ull);  // shared by every match
        reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0, 0, 0, 0);
        wave_sync();
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
            if (lane + 64 * u < n && (r[u] & pm) == pre) atomicAdd(&hist[(uint32_t)(r[u] >> sh) & 255u], 1u);
        wave_sync();
        const uint4 h = reinterpret_cast<const uint4*>(hist)[lane];
        const uint32_t e0 = h.x, e1 = e0 + h.y, e2 = e1 + h.z, e3 = e2 + h.w;
        const uint32_t incl = wave_incl_scan(e3), excl = incl - e3;
        const unsigned long long hit = __ballot(excl < k && k <= incl);  // the lane holding the boundary bin
        const uint32_t src = (uint32_t)__ffsll((long long)hit) - 1u;
        const uint32_t j = k <= excl + e0 ? 0u : k <= excl + e1 ? 1u : k <= excl + e2 ? 2u : 3u;
        const uint32_t below = excl + (j == 0u ? 0u : j == 1u ? e0 : j == 2u ? e1 : e2);
        const uint32_t b = 4u * src + __builtin_amdgcn_readlane(j, (int)src);
        k -= __builtin_amdgcn_readlane(below, (int)src);
        pre = (o & above) | ((uint64_t)b << sh);
        pm = above | (0xFFull << sh);
        wave_sync();  // the histogram is read before the next pass clears it
    }
    // the L smallest: every record <= the L-th (distinct records: exactly L of them)
    uint32_t base = 0;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
        const bool f = lane + 64 * u < n && r[u] <= kth;
        const unsigned long long b = __ballot(f);
        if (f) S.cand()[base + rank_below(b)] = r[u];
        base += (uint32_t)__popcll(b);
    }
    wave_sync();
    cand_n = L;
    tau = kth;
}

// A buffer of n <= 64 distinct records sorted in registers, one record per lane: a bitonic network
// over lane shuffles (log2 P2 (log2 P2 + 1) / 2 stages for P2 = next_pow2(n)), no LDS round trip
// and barrier per stage as in the LDS sort below. The final flush of most queries (C3: ~35
// survivors, 20 results) is this one.
template <class SM>
__device__ __forceinline__ void wave_sort64(SM& S, uint32_t n) {
    const uint32_t lane = lane_id();
    const uint32_t P2 = next_pow2(max(n, 2u));
    uint64_t r = lane < n ? S.cand()[lane] : kNoCand;
    for (uint32_t k = 2; k <= P2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)r, (int)j);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(r >> 32), (int)j);
            const uint64_t p = ((uint64_t)hi << 32) | lo;
            const bool keep_min = ((lane & k) == 0) == ((lane & j) == 0);
            r = keep_min ? min64(r, p) : max64(r, p);
        }
    }
    wave_sync();  // every lane has read the buffer
    if (lane < P2) S.cand()[lane] = r;
    wave_sync();
}

// Wave-local running top-L over the candidate buffer (same algorithm as flush()), sorted.
// unique: no two records share a key (DevIndex.keys_unique): only the second pass runs, after a
// radix select has cut a buffer of more than L records to its L smallest (wave_select).
// (RADIX: the deferred emit and merge kernels; the fused tier-1b kernel keeps the sort alone,
// since the select's registers would push its calcScore out of line)
template <bool RADIX = false, class SM>
__device__ void wave_flush(SM& S, uint32_t& cand_n, uint64_t& tau, uint32_t L, bool unique = false) {
    const uint32_t lane = lane_id();
    if (RADIX && unique && cand_n > L && L) wave_select(S, cand_n, tau, L);
    if (unique && cand_n <= 64) {  // distinct records: sorted in registers
        const uint32_t n = cand_n;
        wave_sort64(S, n);
        cand_n = min(n, L);
        tau = n >= L && L ? S.cand()[L - 1] : kNoCand;
        return;
    }
    const uint32_t n = min(cand_n, (uint32_t)kWaveCand);
    const uint32_t P2 = next_pow2(max(n, 2u));
    for (uint32_t i = lane; i < P2; i += 64) {
        const uint64_t r = i < n ? S.cand()[i] : kNoCand;
        S.cand()[i] = i < n ? (unique ? r : ((r << 32) | (r >> 32))) : kNoCand;  // key-major for the dedup
    }
    wave_sync();
    for (int pass = unique ? 1 : 0; pass < 2; ++pass) {
        for (uint32_t k = 2; k <= P2; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t p = lane; p < P2 / 2; p += 64) {
                    const uint32_t i = ((p & ~(j - 1u)) << 1) | (p & (j - 1u)), l = i + j;  // j is a power of two
                    const uint64_t x = S.cand()[i], y = S.cand()[l];
                    if ((x > y) == ((i & k) == 0)) { S.cand()[i] = y; S.cand()[l] = x; }
                }
                wave_sync();
            }
        }
        if (pass == 1) break;
        uint64_t keep[kWaveCand / 64];
#pragma unroll
        for (int u = 0; u < kWaveCand / 64; ++u) {
            const uint32_t i = lane + u * 64;
            keep[u] = kNoCand;
            if (i < P2) {
                const uint64_t d = S.cand()[i];
                if (d != kNoCand && (i == 0 || (S.cand()[i - 1] >> 32) != (d >> 32))) keep[u] = (d << 32) | (d >> 32);
            }
        }
        wave_sync();
#pragma unroll
        for (int u = 0; u < kWaveCand / 64; ++u) {
            const uint32_t i = lane + u * 64;
            if (i < P2) S.cand()[i] = keep[u];
        }
        wave_sync();
    }
    uint32_t mine = 0;
    for (uint32_t i = lane; i < P2; i += 64) mine += S.cand()[i] != kNoCand;
    const uint32_t nv = wave_sum(mine);
    cand_n = min(nv, L);
    tau = nv >= L ? S.cand()[L - 1] : kNoCand;
    wave_sync();
}

// The refill of a full buffer (and raised_cmin's settling of tau): only the L smallest records
// and tau are needed, not their order, so distinct-key buffers take the radix select alone.
template <bool RADIX = false, class SM>
__device__ __forceinline__ void wave_trim(SM& S, uint32_t& cand_n, uint64_t& tau, uint32_t L, bool unique) {
    if (RADIX && unique && cand_n >= L && L)
        wave_select(S, cand_n, tau, L);
    else
        wave_flush(S, cand_n, tau, L, unique);
}

// (defined below)
template <class SM>
__device__ void wave_emit(SM& S, const DevIndex& X, const SearchParams& P, uint32_t m, uint32_t L,
                          float sc_long, float sc_short, uint32_t& surv_n, uint32_t& cand_n, uint64_t& tau);

// The smallest hit count a term of the next part needs to enter the running top-L (>= cmin). A
// count-c term scores at most max(w_max * c / n, 0) in fp32 (term_pairs' bound), so once the top-L
// is full every count whose bound encodes below tau's score is out; with DevIndex.tk_monotone also
// the count whose bound ties it: a later part's terms have larger ids, hence larger key ranks than
// every record so far, and lose the tie (ScoreComparer, nGramSearch.h:262-269). A count that can
// be an exact match (s > 0.999, promoted to 100) is never excluded. At thr 0 (cmin 1) on a large
// library this turns the exact counting of every posting into the sketch at cmin 2 after the
// first parts have filled the top-L with one-hit records of the shortest keys.
template <class SM>
__device__ uint32_t raised_cmin(SM& S, const DevIndex& X, const SearchParams& P, uint32_t m, uint32_t n, uint32_t L,
                                uint32_t cmin, float sc_long, float sc_short, uint32_t& surv_n, uint32_t& cand_n,
                                uint64_t& tau) {
    if (tau == kNoCand && cand_n + surv_n >= L) {  // full enough: settle tau now
        if (surv_n) wave_emit(S, X, P, m, L, sc_long, sc_short, surv_n, cand_n, tau);
        if (tau == kNoCand && cand_n >= L) wave_trim(S, cand_n, tau, L, X.keys_unique != 0);
    }
    if (tau == kNoCand) return cmin;
    const uint32_t lane = lane_id(), te = ~(uint32_t)(tau >> 32);
    const float ub = X.w_max * sc_long;  // lane c: the bound of c hits
    const uint32_t ue = ub > 0.0f ? __float_as_uint(ub) + 1u : 1u;
    const bool out = lane >= 1 && lane <= n && !((double)sc_long > 0.999) && (ue < te || (X.tk_monotone && ue == te));
    const unsigned long long om = __ballot(out);  // a prefix of the counts: the bound grows with c
    return max(cmin, om ? 64u - (uint32_t)__clzll((long long)om) : 0u);
}

// calcScore (nGramSearch.hpp:310-341) over the survivor list: term -> (key, weight) pairs,
// max(w*s, 0), exact-match promotion, into the running top-L.
template <class SM>
__device__ void wave_emit(SM& S, const DevIndex& X, const SearchParams& P, uint32_t m, uint32_t L,
                          float sc_long, float sc_short, uint32_t& surv_n, uint32_t& cand_n, uint64_t& tau) {
    const uint32_t lane = lane_id();
    S.surv_total += surv_n;
    wave_sync();
    for (uint32_t base = 0; base < surv_n; base += 64) {
        const uint32_t i = base + lane;
        uint32_t p = 0, pe = 0, code = 0, t = 0;
        if (i < surv_n) {
            t = S.surv_t[i];
            code = S.surv_c[i];
        }
        const float s_l = __shfl(sc_long, (int)(code & 63u)), s_s = __shfl(sc_short, (int)(code & 63u));
        const float s = (code & 0x80u) ? s_s : s_l;
        const bool promo = (double)s > 0.999;  // nGramSearch.hpp:328
        if (i < surv_n) term_pairs(X, t, s, promo, tau, p, pe);
        while (__ballot(p < pe)) {
            uint64_t rec = kNoCand;
            if (p < pe) {
                const uint2 kw = X.tk[p++];
                const uint32_t enc = pair_enc(kw, s, promo, (code & 0x80u) != 0, X, S.q, 4u, m, P.valid);
                if (enc) rec = ((uint64_t)(~enc) << 32) | kw.x;
            }
            if (cand_n + 64 > (uint32_t)kWaveCand) wave_trim(S, cand_n, tau, L, X.keys_unique != 0);
            const bool want = rec < tau;
            const unsigned long long b = __ballot(want);
            if (want) S.cand()[cand_n + rank_below(b)] = rec;
            cand_n += __popcll(b);
        }
    }
    surv_n = 0;
    wave_sync();
}

template <bool LEAN>
__device__ __forceinline__ void surv_append(WaveSmem<LEAN>& S, bool pass, uint32_t t, uint32_t code, uint32_t& surv_n) {
    const unsigned long long b = __ballot(pass);
    if (pass) {
        const uint32_t i = surv_n + rank_below(b);
        S.surv_t[i] = t;
        S.surv_c[i] = (uint8_t)code;
    }
    surv_n += __popcll(b);
}

// zero the wave's LDS table (16-byte stores, lane-strided)
template <bool LEAN>
__device__ __forceinline__ void clear_table(WaveSmem<LEAN>& S, uint32_t lane) {
    uint4* T4 = reinterpret_cast<uint4*>(S.table);
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)TableGeom<LEAN>::kSlots / 256; ++i) T4[lane + 64 * i] = make_uint4(0, 0, 0, 0);
}

// Exact counts of a sketch part's nc <= 64 candidate entries (S.cbuf; lane l < nc takes entry l):
// a term's count is the number of candidates holding it (every entry of a term lands in the same
// cell), owned by the first of them. Terms whose count reaches cmin become survivors.
template <bool LEAN>
__device__ __forceinline__ void cand_counts(WaveSmem<LEAN>& S, uint32_t nc, uint32_t cmin, uint32_t n_short,
                                            uint32_t n_terms, uint32_t& surv_n) {
    const uint32_t lane = lane_id();
    uint32_t lc = lane;  // opaque: the slot address is made here, not kept across the part loop (spilled)
    asm volatile("" : "+v"(lc));
    const uint32_t t = lc < nc ? S.cbuf[lc] : kStray;
    uint32_t cnt = 0;
    bool first = true;
    for (uint32_t j = 0; j < nc; ++j) {
        const uint32_t tj = __builtin_amdgcn_readlane(t, j);
        const bool eq = t == tj;
        cnt += eq;
        first &= !(eq && j < lane);
    }
    surv_append(S, lane < nc && first && cnt >= cmin, min(n_short + t, n_terms - 1u), cnt, surv_n);
}

template <bool LEAN>
__device__ __forceinline__ uint32_t wave_insert_slot(uint32_t* T, uint32_t rel, unsigned* err) {
    constexpr uint32_t kSlots = TableGeom<LEAN>::kSlots;
    uint32_t probes = 0;
    uint32_t h = (rel * 0x9E3779B1u) >> (32 - TableGeom<LEAN>::kBits);
    const uint32_t want = rel << 8;
    for (;;) {
        uint32_t cur = T[h];
        if (cur == 0) {
            const uint32_t prev = atomicCAS(&T[h], 0u, want | 1u);
            if (prev == 0) return h;
            cur = prev;
        }
        if ((cur >> 8) == rel) {
            atomicAdd(&T[h], 1u);
            return h;
        }
        h = (h + 1) & (kSlots - 1);
        if (++probes > kSlots) {
            atomicOr(err, 1u);
            return h;
        }
    }
}

// sketch cell of a term: full-rate shift/xor (v_mul_lo_u32 is quarter rate). Term ids of a part
// are spread over a range much wider than the table, and consecutive ids get distinct cells.
// Tier 1a takes the low bits alone (the xor fold measured 10 % slower there): its parts are contiguous term-id ranges
// whose few hundred entries are spread over an id span far wider than the table.
template <bool LEAN>
__device__ __forceinline__ uint32_t sketch_cell(uint32_t t) {  // u4 counter index: 8 per table word
    constexpr uint32_t kBits = TableGeom<LEAN>::kBits + 3;
    if constexpr (LEAN) return t & ((1u << kBits) - 1u);
    return (t ^ (t >> kBits)) & ((1u << kBits) - 1u);
}
// the table word holding t's cell; tier 1a's low-bit cells address it as the byte offset
// (t >> 1) & 0xffc, two instructions (the word index form takes three)
template <bool LEAN>
__device__ __forceinline__ uint32_t* sketch_word(uint32_t* table, uint32_t t) {
    constexpr uint32_t kBits = TableGeom<LEAN>::kBits + 3;
    if constexpr (LEAN)
        return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(table) + ((t >> 1) & (((1u << kBits) - 1u) >> 1 & ~3u)));
    return table + (sketch_cell<LEAN>(t) >> 3);
}
// (sketch_cell(t) & 7) * 4 in the low 5 bits, higher bits arbitrary: v_lshlrev and v_bfe_u32 read
// only the low 5 bits of a shift / offset, so the mask is never materialised (the tier-1a kernel
// is VALU-issue bound)
template <bool LEAN>
__device__ __forceinline__ uint32_t sketch_sh4(uint32_t t) {
    constexpr uint32_t kBits = TableGeom<LEAN>::kBits + 3;
    if constexpr (LEAN) return t << 2;
    return (t ^ (t >> kBits)) << 2;
}

// Loads one part into registers. Lane g < ng contributes entries [cur, cur + len) of its list
// (list base gbase, a0 = gbase % 4); the part's 16-byte chunks are numbered across all lists (DPP
// prefix sum), lane l holding chunks l, 64 + l, ... in v[0], v[1], ...: about one load
// instruction per 256 postings whatever the number of lists (MI355X issues scattered loads at
// a fixed rate per instruction). A chunk finds its list through a marker per list
// start plus a max-scan; vmask bit 4r+e says whether entry e of v[r] belongs to the part (chunk
// edges hold up to 3 entries of neighbouring lists). Returns the part's chunk count.
template <bool LEAN>
__device__ __forceinline__ uint32_t stage_part(WaveSmem<LEAN>& S, const uint4* __restrict__ post4, uint64_t gbase,
                                               uint32_t a0, uint32_t cur, uint32_t len,
                                               uint4 (&v)[kDmaRounds], uint32_t& vmask) {
    const uint32_t lane = lane_id();
    const uint32_t head = (a0 + cur) & 3u;
    const uint32_t nch = len ? (head + len + 3) >> 2 : 0u;
    const uint32_t incl = wave_incl_scan(nch);
    const uint32_t pre = incl - nch;
    const uint32_t tch = __builtin_amdgcn_readlane(incl, 63);
    const uint32_t mt = __builtin_amdgcn_readfirstlane(min(tch, (uint32_t)kWaveChunks));
    uint8_t* mk = S.mark;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r)
        if (64 * r < mt) mk[64 * r + lane] = 0;
    wave_sync();
    if (nch) {
        if (pre < kWaveChunks) mk[pre] = (uint8_t)(lane + 1);
        const uint32_t first = (uint32_t)((gbase + cur) >> 2);
        S.segtab[lane] = make_uint2(first - pre, (4 * pre + head) | ((4 * pre + head + len) << 16));
    }
    wave_sync();
    uint32_t carry = 0;
    // all rounds' max-scans are independent; the carries chain only through their lane-63
    // values, so the LDS reads and loads of the rounds can be in flight together
    uint32_t scn[kDmaRounds];
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        const uint32_t lc = 64 * r + lane;
        scn[r] = 64 * r < mt ? wave_incl_max_scan(lc < mt ? (uint32_t)mk[lc] : 0u) : 0u;
    }
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        const uint32_t top = __builtin_amdgcn_readlane(scn[r], 63);
        scn[r] = max(scn[r], carry);
        carry = max(carry, top);
    }
    vmask = 0;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        if (64 * r < mt) {
            const uint32_t c = 64 * r + lane;
            const bool ok = c < mt;
            const uint2 seg = S.segtab[(scn[r] - 1u) & 63u];
            // inactive lanes must not load: a shared fallback address would be read by every wave
            // of the GPU and serialise on one L2 channel
            if (ok) v[r] = post4[seg.x + c];
            // entries [lo_e, hi_e) of this chunk are in the list segment [y, z)
            const int y = (int)(seg.y & 0xFFFFu), z = (int)(seg.y >> 16);
            const uint32_t lo_e = (uint32_t)min(max(y - (int)(4 * c), 0), 4);
            const uint32_t hi_e = (uint32_t)min(max(z - (int)(4 * c), 0), 4);
            const uint32_t bits = ((1u << hi_e) - 1u) & ~((1u << lo_e) - 1u);
            vmask |= (ok ? bits : 0u) << (4 * r);
        }
    }
    return mt;
}

// Exact count of the part's entries with term ids in [ta, tb) (at most kWaveCap of them): LDS
// hash table term -> count. Each such entry's register is replaced by
// its slot, tagged with the pass number (bit 31 | pass << 16 | slot; term ids stay below 2^31),
// so later passes over other term ranges skip it; the extraction exchanges the slot with 0,
// so the first holder of a term owns its count (no table scan; the table ends empty).
template <bool LEAN>
__device__ __forceinline__ void part_exact(WaveSmem<LEAN>& S, uint4 (&v)[kDmaRounds], uint32_t vmask, uint32_t mt,
                                           uint32_t ta, uint32_t tb, uint32_t pass, const DevIndex& X,
                                           const SearchParams& P, uint32_t m, uint32_t L, uint32_t cmin,
                                           float sc_long, float sc_short, uint32_t& surv_n, uint32_t& cand_n,
                                           uint64_t& tau, unsigned* err) {
    mt = __builtin_amdgcn_readfirstlane(mt);
    const uint32_t tag = 0x80000000u | (pass << 16);
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        if (64 * r < mt) {
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) {
                uint32_t& x = e == 0 ? v[r].x : e == 1 ? v[r].y : e == 2 ? v[r].z : v[r].w;
                if (((vmask >> (4 * r + e)) & 1u) && x - ta < tb - ta)
                    x = tag | wave_insert_slot<LEAN>(S.table, x - ta + 1u, err);
            }
        }
    }
    wave_sync();
    {
        {
            uint32_t sn = surv_n, cn = cand_n;
            uint64_t ta2 = tau;
            // one element slot per step (a single wave_emit call site keeps the registers out of scratch)
            for (uint32_t k = 0; k < 4 * (uint32_t)kDmaRounds && 64 * (k >> 2) < mt; ++k) {
                if (sn + 64 > (uint32_t)kWaveSurv) wave_emit(S, X, P, m, L, sc_long, sc_short, sn, cn, ta2);
                uint32_t x = kStray;
                if (k < 16) {  // 16-way selects (k is uniform)
#pragma unroll
                    for (uint32_t j = 0; j < 16; ++j) {
                        const uint32_t y = (j & 3) == 0 ? v[j >> 2].x : (j & 3) == 1 ? v[j >> 2].y : (j & 3) == 2 ? v[j >> 2].z : v[j >> 2].w;
                        x = j == k ? y : x;
                    }
                } else {
#pragma unroll
                    for (uint32_t j = 16; j < 4 * (uint32_t)kDmaRounds; ++j) {
                        const uint32_t y = (j & 3) == 0 ? v[j >> 2].x : (j & 3) == 1 ? v[j >> 2].y : (j & 3) == 2 ? v[j >> 2].z : v[j >> 2].w;
                        x = j == k ? y : x;
                    }
                }
                const bool mine = (x >> 16) == (tag >> 16);
                const uint32_t c = mine ? atomicExch(&S.table[x & 0xFFFFu], 0u) : 0u;
                const uint32_t cnt = c & 255u;  // s = cnt / n; s >= thr <=> cnt >= cmin (nGramSearch.hpp:300,315)
                surv_append(S, c != 0 && cnt >= cmin, min(X.n_short + ta + (c >> 8) - 1u, X.n_terms - 1u), cnt, sn);
            }
            surv_n = sn;
            cand_n = cn;
            tau = ta2;
        }
        wave_sync();
    }
}

// Sketch count of a part held in registers (2 <= cmin <= 15): 8 x u4 counters per table word,
// never an undercount (an increment that wraps a counter past 15 is seen in the value the atomic
// returns and sends the part to exact counting). Entries whose cell reaches cmin are candidates;
// the wave gets their exact counts by comparing the <= 64 candidates with each other. Returns the number of candidate entries; above 64 the caller counts the part exactly
// (the table is clean again). (u16 counters with no-return adds were measured: the 4x fewer
// cells per KB cost more in false candidates than the returns cost in waits.)
template <bool LEAN, int NR = kDmaRounds>
__device__ __forceinline__ uint32_t part_sketch(WaveSmem<LEAN>& S, const uint4 (&v)[NR], uint32_t vmask,
                                                uint32_t mt, uint32_t cmin, uint32_t n_short, uint32_t n_terms,
                                                uint32_t& surv_n) {
    const uint32_t lane = lane_id();
    mt = __builtin_amdgcn_readfirstlane(mt);
    const uint32_t cm1 = __builtin_amdgcn_readfirstlane(cmin - 1u);
    // the add pass also counts the <= 3 entries of neighbouring lists at each segment edge (never an
    // undercount; the candidate pass below masks them out), so an add needs no per-entry mask bit,
    // and one running max of the counters it saw stands for both tests: >= cmin - 1 (an add took a
    // cell to cmin: candidates; every cell that ends at >= cmin had exactly one such add in this part,
    // the table starting clear and the adds being 0/1) and == 15 (a counter wrapped)
    uint32_t seen = 0;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)NR; ++r) {
        if (64 * r < mt && 64 * r + lane < mt) {
            const uint32_t t[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            // the round's four returning adds issued together, then their values read (one LDS wait
            // per round: +3 % once the VALU diet left latency to hide, 31.5 -> 32.4 Mq/s)
            uint32_t old[4];
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e)
                old[e] = atomicAdd(sketch_word<LEAN>(S.table, t[e]), 1u << (sketch_sh4<LEAN>(t[e]) & 31u));
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) seen = max(seen, __builtin_amdgcn_ubfe(old[e], sketch_sh4<LEAN>(t[e]), 4u));
        }
    }
    const bool ovf = seen == kSketchMax, hot = seen >= cm1;
    wave_sync();
    if (!__ballot(hot || ovf)) {  // no cell reached cmin: no candidates
        clear_table(S, lane);
        wave_sync();
        return 0;
    }
    const uint32_t ov = __ballot(ovf) ? 65u : 0u;  // a wrapped counter forces exact counting
    // candidates are rare (~3.5 of ~410 entries), so each entry slot is a compare into a ballot and a
    // uniform branch, taken by the few slots holding one, which write their terms in place (no
    // per-lane mask, prefix sum or register select)
    uint32_t nw = 0;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)NR; ++r) {
        if (64 * r < mt) {
            const uint32_t t[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            uint32_t w[4];
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) w[e] = *sketch_word<LEAN>(S.table, t[e]);
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) {
                // the entry's mask bit is tested only in the (rare) branch taken when some cell of the
                // slot reached cmin
                bool f = __builtin_amdgcn_ubfe(w[e], sketch_sh4<LEAN>(t[e]), 4u) >= cmin;
                if (__ballot(f)) {
                    f = f && ((vmask >> (4 * r + e)) & 1u);
                    const unsigned long long b = __ballot(f);
                    const uint32_t pos = nw + rank_below(b);
                    if (f && pos < 64u) S.cbuf[pos] = t[e];
                    nw += (uint32_t)__popcll(b);
                }
            }
        }
    }
    wave_sync();
    const uint32_t nc = __builtin_amdgcn_readfirstlane(nw + ov);
    clear_table(S, lane);
    if (nc && nc <= 64) cand_counts(S, nc, cmin, n_short, n_terms, surv_n);
    wave_sync();
    return nc;
}

// Tier 1a at cmin 1 (threshold 0: every term sharing a gram with the query survives): the sketch
// adds of part_sketch, then every entry alone in its cell is a one-hit term, written straight to
// the query's survivor slots in HBM (et / ec at `spilled`, for k_emit), and the entries of cells
// that reached 2 (terms with more hits, and the few colliding pairs of one-hit terms) are
// resolved exactly by comparing them with each other. Returns the number of those candidates;
// above 64, a wrapped counter, or survivor slots running out (kEmitCap) it returns 65: the
// caller hands the query to tier 1b. Parts are cut to a quarter of a sketch part so that pairs
// colliding in the 8,192 cells stay few.
template <int NR = kDmaRounds>
__device__ __forceinline__ uint32_t part_ones(WaveSmem<true>& S, const uint4 (&v)[NR], uint32_t vmask, uint32_t mt,
                                              uint32_t n_short, uint32_t n_terms, uint32_t& surv_n,
                                              uint32_t* __restrict__ et, uint8_t* __restrict__ ec, uint32_t& spilled,
                                              uint32_t ecap) {
    const uint32_t lane = lane_id();
    mt = __builtin_amdgcn_readfirstlane(mt);
    uint32_t seen = 0;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)NR; ++r) {
        if (64 * r < mt && 64 * r + lane < mt) {
            const uint32_t t[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            uint32_t old[4];  // (the four adds issued together, as in part_sketch)
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e)
                old[e] = atomicAdd(sketch_word<true>(S.table, t[e]), 1u << (sketch_sh4<true>(t[e]) & 31u));
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) seen = max(seen, __builtin_amdgcn_ubfe(old[e], sketch_sh4<true>(t[e]), 4u));
        }
    }
    const bool ovf = __ballot(seen == kSketchMax) != 0;
    wave_sync();
    uint32_t nw = 0;
    if (!ovf) {
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)NR; ++r) {
            if (64 * r < mt) {
                const uint32_t t[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
                uint32_t w[4];
#pragma unroll
                for (uint32_t e = 0; e < 4; ++e) w[e] = *sketch_word<true>(S.table, t[e]);
#pragma unroll
                for (uint32_t e = 0; e < 4; ++e) {
                    const uint32_t c = ((vmask >> (4 * r + e)) & 1u) ? __builtin_amdgcn_ubfe(w[e], sketch_sh4<true>(t[e]), 4u) : 0u;
                    const bool one = c == 1, two = c >= 2;
                    const unsigned long long b1 = __ballot(one);
                    if (b1) {
                        const uint32_t pos = spilled + rank_below(b1);
                        if (one && pos < ecap) {
                            et[pos] = min(n_short + t[e], n_terms - 1u);
                            ec[pos] = 1;
                        }
                        spilled += (uint32_t)__popcll(b1);
                    }
                    const unsigned long long b2 = __ballot(two);
                    if (b2) {
                        const uint32_t pos = nw + rank_below(b2);
                        if (two && pos < 64u) S.cbuf[pos] = t[e];
                        nw += (uint32_t)__popcll(b2);
                    }
                }
            }
        }
    }
    wave_sync();
    clear_table(S, lane);
    if (ovf || nw > 64 || spilled + surv_n > ecap) {
        wave_sync();
        return 65;
    }
    if (nw) cand_counts(S, nw, 1u, n_short, n_terms, surv_n);  // (every candidate a survivor)
    wave_sync();
    return nw;
}

// One query on one wave: tier 1b (the full wave kernel, k_wave) and the server kernel. Tier 1a's
// lean kernel has part loops of its own (lean_query, lean_query_g).
__device__ __forceinline__ void wave_query(WaveSmem<>& S, const uint32_t q, const DevIndex& X, const SearchParams& P,
                                           const uint8_t* __restrict__ qnorm, const uint64_t* __restrict__ qoff,
                                           const uint32_t* __restrict__ qm, uint32_t* __restrict__ out_n,
                                           uint32_t* __restrict__ out_k, float* __restrict__ out_s,
                                           uint32_t* __restrict__ list2, uint32_t* __restrict__ count2,
                                           DevStats* __restrict__ stats, uint32_t* __restrict__ fb,
                                           uint32_t* __restrict__ fbc, const uint32_t slice = 0,
                                           const uint32_t nsl = 1, const uint32_t m_in_lds = kQueryInGlobal) {
    const uint32_t lane = lane_id(), tid = threadIdx.x;
    // sliced tier 1b: this wave takes the term ids of skip-table buckets [K * slice / nsl,
    // K * (slice + 1) / nsl) and leaves its top-L records for k_merge (SearchParams.prec)
    const bool sliced = nsl > 1;
    if (sliced) {  // queries answered without the long search: slice 0 answers, k_merge skips them
        const uint32_t m0 = qm[q];
        const bool direct = m0 == kQueryWildcard || m0 == 0 || m0 <= X.full_scan_len ||
                            m0 - X.gsz + 1 > kWaveMaxGrams || P.limit > kWaveMaxLimit;
        if (direct) {
            if (slice != 0) return;
            if (tid == 0) P.pcnt[(size_t)q * nsl] = kNoPart;
        }
    }
    (void)fb;
    (void)fbc;
    // m_in_lds: the caller (k_serve) put the normalised query in S.q already
    const uint32_t m = m_in_lds != kQueryInGlobal ? m_in_lds : qm[q];
    const uint32_t L = P.limit;
    const size_t ob = (size_t)q * P.out_stride;
    if (m == kQueryWildcard) {  // nGramSearch.hpp:356-369
        wild_answer(X, P, q, tid, 64, out_n, out_k, out_s);
        return;
    }
    if (m == 0) {  // nothing left after normalisation, nGramSearch.hpp:374-375
        if (tid == 0) out_n[q] = 0;
        return;
    }
    if (m <= X.full_scan_len || m - X.gsz + 1 > kWaveMaxGrams || L > kWaveMaxLimit) {
        if (tid == 0) list2[atomicAdd(count2, 1u)] = q;  // tier 2 / library-wide path
        return;
    }
    const uint32_t n = m - X.gsz + 1;  // grams of the query (hpp:29-36; 3-grams: m - 2)
    const uint32_t n_long = X.n_terms - X.n_short;
    WPHASE_BEGIN
    if (m_in_lds == kQueryInGlobal) {
        const uint8_t* qg = qnorm + qoff[q];
        for (uint32_t i = tid; i < m; i += 64) S.q[i] = char_at(qg, i, X.csize);
    }
    if (tid == 0) {
        S.surv_total = 0;
        S.ncand = 0;
        S.xcnt = 0;
    }
    clear_table(S, lane);
    wave_sync();
    uint32_t cand_n = 0, surv_n = 0;
    uint64_t tau = kNoCand;
    unsigned* err = &stats->errors;
    // lane c holds the fp32 score of c hits: (float)c / n (hpp:300) and (float)c / m (hpp:244)
    const float sc_long = lane <= n ? (float)lane / (float)n : 0.0f;
    const float sc_short = lane <= m ? (float)lane / (float)m : 0.0f;
    // the smallest hit count whose score passes the threshold (hpp:300,315)
    const unsigned long long pm = __ballot(lane <= n && lane > 0 && !(sc_long < P.thr));
    const uint32_t cmin = pm ? (uint32_t)(__ffsll((long long)pm) - 1) : 1000u;

    // ---- searchShort over shortLib (nGramSearch.hpp:262-270), 4 <= m < 9, wave 0 ----
    if (slice == 0 && m < X.short_query_len && X.n_short) {
        uint32_t qc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) qc[i] = (uint32_t)i < m ? S.q[i] : 0;
        const unsigned long long okm = __ballot(lane <= m && !(sc_short < P.thr));  // hpp:315
        const uint32_t cmin_s = okm ? (uint32_t)(__ffsll((long long)okm) - 1) : 64u;
        build_peq(S.peq, [&](uint32_t i) { return S.q[i]; }, m, lane, 64u);
        wave_sync();
        const uint32_t ns = X.n_short;
        // narrow corpora: rounds of 64 terms (lane: term 64 r + lane) in a software pipeline; while
        // round r is matched, the bytes of round r + 1 and the offsets of round r + 2 are in flight
        // (a term is two dependent loads, offsets then bytes; one round at a time left both
        // exposed). Wide corpora match through string_match. One loop, so wave_emit keeps a
        // single call site here (a second one stops it inlining and puts X and P in scratch).
        const bool narrow = X.csize == 1;
        const uint64_t* to = X.term_off;
        const uint8_t* tbase = X.term_bytes;  // (padded by two dwords: the second dword is always readable)
        auto offs = [&](uint32_t t, uint64_t& a, uint64_t& b) {
            const uint32_t u = min(t, ns - 1u);
            a = to[u];
            b = to[u + 1];
        };
        auto bytes = [&](uint64_t a, uint64_t b, uint32_t& y0, uint32_t& y1, uint32_t& sk, uint32_t& len) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(tbase + (a & ~3ull));
            y0 = w[0];
            y1 = w[1];
            sk = (uint32_t)a & 3u;
            len = (uint32_t)(b - a);
        };
        uint64_t a1 = 0, b1 = 0;
        uint32_t x0 = 0, x1 = 0, xs = 0, xl = 0;
        if (narrow) {
            uint64_t a0, b0;
            offs(lane, a0, b0);
            offs(64u + lane, a1, b1);
            bytes(a0, b0, x0, x1, xs, xl);
        }
        for (uint32_t t0 = 0; t0 < ns; t0 += 64) {
            uint32_t y0 = 0, y1 = 0, ys = 0, yl = 0;
            uint64_t a2 = 0, b2 = 0;
            if (narrow) {
                bytes(a1, b1, y0, y1, ys, yl);   // round r + 1
                offs(t0 + 128u + lane, a2, b2);  // round r + 2
            }
            if (surv_n + 64 > (uint32_t)kWaveSurv) wave_emit(S, X, P, m, L, sc_long, sc_short, surv_n, cand_n, tau);
            const uint32_t t = t0 + lane;
            uint32_t match = 0;
            if (narrow) match = myers_short(S.peq, m, x0, x1, xs, xl);
            else if (t < ns) match = string_match(S.peq, qc, m, X, t);
            surv_append(S, t < ns && match >= cmin_s, t, match | 0x80u, surv_n);
            x0 = y0, x1 = y1, xs = ys, xl = yl;
            a1 = a2, b1 = b2;
        }
    }
    WSTAMP(0);

    // ---- searchLong (nGramSearch.hpp:278-301) ----
    // lane i: occurrence i of a query gram; lanes 0..ng-1 then own the occurrences whose gram
    // has postings (a gram repeated k times owns k lanes: count with multiplicity). Every wave
    // computes the same plan.
    uint64_t gbase;
    uint32_t glen, grow;
    const uint32_t ng = gram_lists(X, [&](uint32_t i) { return S.q[i]; }, n, lane, gbase, glen, grow);
    const uint64_t p_total = wave_sum((uint64_t)glen);
    uint64_t p_stat = p_total;  // postings this wave reads (its slice's)
    // sketch counting for 2 <= cmin <= 15; at cmin 2 two colliding entries already make a false
    // candidate, so those parts are cut at half the size
    const bool sketch = cmin >= kSketchMinCmin && cmin <= kSketchMax;
    const uint32_t shrink = 0;  // (tier 1b counts cmin-2 parts in full: half-size parts measured no faster)
    // part cap: a sketch part holds twice the entries of an exact pass (u8 vs u32 cells)
    const uint32_t kChunks = (sketch ? (uint32_t)kWaveChunks : (uint32_t)kExactChunks) >> shrink;
    WSTAMP(1);
    if (p_total && cmin <= n) {
        const uint32_t K = X.n_buckets, span = X.bucket_span;
        const uint32_t wmax = (uint32_t)max64(1, min64(K, kMaxPartSpan / max(span, 1u)));
        const uint32_t w = (uint32_t)max64(1, min64(wmax, (uint64_t)K * ((sketch ? kSketchTarget : kWaveTarget) >> shrink) / p_total));
        const uint32_t* sk = X.skip + (size_t)grow * (K + 1);
        const uint4* post4 = reinterpret_cast<const uint4*>(X.post);
        const uint32_t a0 = (uint32_t)gbase & 3u;  // list start within its 16-byte chunk
        // entries [s, e) of this lane's list cover 16-byte chunks [(a0 + s) / 4, (a0 + e + 3) / 4)
        auto chunks = [a0](uint32_t s, uint32_t e) -> uint32_t { return e > s ? ((a0 + e + 3) >> 2) - ((a0 + s) >> 2) : 0u; };
        // end of the next bucket part: skip[row][min(K, bn + w)]; idle lanes load nothing (a shared
        // row would be a hot spot). (Preloading every boundary of the query into LDS was measured
        // slower: the LDS it takes costs occupancy.)
        // this wave's buckets [b_lo, b_hi): all of them unless sliced
        const uint32_t b_lo = sliced ? (uint32_t)((uint64_t)K * slice / nsl) : 0u;
        const uint32_t b_hi = sliced ? (uint32_t)((uint64_t)K * (slice + 1) / nsl) : K;
        auto next_end = [&](uint32_t bn) -> uint32_t { return sk[min(b_hi, bn + w)]; };
        // part iterator: buckets [bnext, bnext + w) unless they exceed kChunks, then term-id sub-parts
        uint32_t cur = 0, bnext = b_lo;
        if (sliced) {
            cur = lane < ng ? sk[b_lo] : 0u;
            p_stat = wave_sum((uint64_t)(lane < ng ? sk[b_hi] - cur : 0u));
        }
        uint32_t e_pre = 0;
        if (lane < ng) e_pre = next_end(b_lo);
        uint32_t in_sub = 0;
        uint32_t sub_lo = 0, hi_lim = 0, sub_end = 0, sub_bnext = 0, step = 1;
        // software pipeline in registers: part i+1's loads are in flight while part i is counted
        uint4 pv[kDmaRounds];
        uint32_t p_vm = 0, p_mt = 0, p_lo = 0, p_hi = 0;
        bool have_p = false;
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) pv[r] = make_uint4(0, 0, 0, 0);
        for (uint32_t guard = 0;;) {
            // the part to count: the one staged last iteration (double buffer; one buffer with the
            // loads waited for in place was measured slower)
            uint4 cv[kDmaRounds];
            uint32_t c_vm = 0, c_mt = 0, c_lo = 0, c_hi = 0;
            bool have_c = false;
            auto take = [&]() {
#pragma unroll
                for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) cv[r] = pv[r];
                c_vm = p_vm;
                c_mt = p_mt;
                c_lo = p_lo;
                c_hi = p_hi;
                have_c = have_p;
            };
            take();
            WSTAMP(2);
            // ---- next part: [lo, ...) with per-lane segments [gbase + cur, gbase + cur + len) ----
            uint32_t lo = 0, hi_t = 0, len = 0;  // part: term ids [lo, hi_t)
            have_p = false;
            in_sub = __builtin_amdgcn_readfirstlane(in_sub);
            bnext = __builtin_amdgcn_readfirstlane(bnext);
            // common case, straight-line: the next group of w buckets is non-empty and fits
            // (span * w <= kMaxPartSpan holds by the choice of w)
            bool fast = false;
            if (!in_sub && bnext < b_hi) {
                const uint32_t e = lane < ng ? e_pre : cur;
                const uint32_t tot = wave_sum_u32(chunks(cur, e));
                if (tot && tot <= kChunks) {
                    lo = bnext * span;
                    len = e - cur;
                    bnext = min(b_hi, bnext + w);
                    hi_t = (uint32_t)min64((uint64_t)bnext * span, n_long);
                    if (lane < ng) e_pre = next_end(bnext);
                    have_p = true;
                    fast = true;
                }
            }
            for (; !fast;) {
                // loop-carried part state is wave-uniform: keep it in SGPRs
                guard = __builtin_amdgcn_readfirstlane(guard);
                bnext = __builtin_amdgcn_readfirstlane(bnext);
                    sub_lo = __builtin_amdgcn_readfirstlane(sub_lo);
                step = __builtin_amdgcn_readfirstlane(step);
                if (++guard > 8u * K + 4096u) {
                    atomicOr(err, 4u);  // every lane (idempotent): a lane-0 branch would make the loop divergent
                    break;
                }
                if (!in_sub) {
                    if (bnext >= b_hi) break;
                    const uint32_t bhi = min(b_hi, bnext + w), e = lane < ng ? e_pre : cur;
                    const uint32_t tot = wave_sum_u32(chunks(cur, e));
                    if (tot <= kChunks) {
                        lo = bnext * span;
                        len = e - cur;
                        bnext = bhi;
                            hi_t = (uint32_t)min64((uint64_t)bhi * span, n_long);
                        if (lane < ng) e_pre = next_end(bnext);
                        if (tot) { have_p = true; break; }
                        continue;
                    }
                    in_sub = 1;
                    sub_lo = bnext * span;
                    hi_lim = (uint32_t)min64((uint64_t)bhi * span, n_long);
                    sub_end = e;
                    sub_bnext = bhi;
                    step = (uint32_t)max64(1, min64((uint64_t)(hi_lim - sub_lo) * (kChunks * 3 / 4) / max(tot, 1u),
                                                    kMaxPartSpan));
                }
                const uint32_t hi = (uint32_t)min64(hi_lim, (uint64_t)sub_lo + step);
                // lower_bound(list, hi) per lane, as a ballot-controlled (uniform) loop: a divergent
                // loop here would make the whole part iterator divergent for the compiler
                uint32_t a = cur, b = lane < ng ? sub_end : cur;
                while (__ballot(a < b)) {
                    const bool act = a < b;
                    const uint32_t mid = (a + b) >> 1;
                    uint32_t pv = 0;
                    if (act) pv = X.post[gbase + mid];
                    const bool below = pv < hi;
                    a = act && below ? mid + 1 : a;
                    b = act && !below ? mid : b;
                }
                const uint32_t t2 = wave_sum_u32(lane < ng ? chunks(cur, a) : 0u);
                if (t2 > kChunks && hi - sub_lo > 1) {
                    step = max(1u, (uint32_t)((uint64_t)(hi - sub_lo) * (kChunks * 3 / 4) / t2));
                    continue;
                }
                lo = sub_lo;
                hi_t = hi;
                len = lane < ng ? a - cur : 0u;
                sub_lo = hi;
                if (sub_lo >= hi_lim) {
                    in_sub = 0;
                    bnext = sub_bnext;
                    if (lane < ng) e_pre = next_end(bnext);
                }
                if (t2) { have_p = true; break; }
                cur = a;
            }
            WSTAMP(3);
            have_p = __builtin_amdgcn_readfirstlane(have_p ? 1u : 0u) != 0;  // uniform: scalar loop exit
            // ---- part i+1: issue this wave's loads ----
            if (have_p) {
                p_mt = stage_part(S, post4, gbase, a0, cur, len, pv, p_vm);
                p_lo = lo;
                p_hi = hi_t;
                cur += len;
            }
            WSTAMP(4);
            // ---- count part i while part i+1 is in flight ----
            if (have_c) {
                if (surv_n + 64 > (uint32_t)kWaveSurv) wave_emit(S, X, P, m, L, sc_long, sc_short, surv_n, cand_n, tau);
                // the count this part must reach: cmin, raised once the running top-L is full and
                // a term of fewer hits could not enter it
                const uint32_t ceff = raised_cmin(S, X, P, m, n, L, cmin, sc_long, sc_short, surv_n, cand_n, tau);
                // (survivors must pass the threshold exactly: no sketch past its u4 range)
                const bool sk = ceff >= kSketchMinCmin && ceff <= kSketchMax;
                const uint32_t nc = sk ? part_sketch(S, cv, c_vm, c_mt, ceff, X.n_short, X.n_terms, surv_n) : 65u;
                const bool done = nc <= 64;
                WCOUNT(11, 1);
                WCOUNT(12, done ? 0 : 1);
                WCOUNT(13, sketch ? nc : 0);
                WCOUNT(14, c_mt);
                WSTAMP(5);
                if (!done) {
                    // exact count in term-id ranges of <= kWaveCap entries (one range unless a sketch
                    // part overflowed)
                    const uint32_t mtu = __builtin_amdgcn_readfirstlane(c_mt);
                    uint32_t ta = c_lo, pass = 0;
                    while (ta < c_hi) {
                        uint32_t tb = c_hi;
                        for (;;) {
                            uint32_t cnt = 0;
#pragma unroll
                            for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
                                if (64 * r < mtu) {
                                    const uint32_t t4[4] = {cv[r].x, cv[r].y, cv[r].z, cv[r].w};
#pragma unroll
                                    for (uint32_t e = 0; e < 4; ++e)
                                        cnt += ((c_vm >> (4 * r + e)) & 1u) && t4[e] - ta < tb - ta ? 1u : 0u;
                                }
                            }
                            cnt = wave_sum_u32(cnt);
                            if (cnt <= (uint32_t)TableGeom<false>::kCap || tb - ta <= 1) break;
                            tb = ta + (tb - ta) / 2;
                        }
                        part_exact(S, cv, c_vm, c_mt, ta, tb, pass++, X, P, m, L, ceff, sc_long, sc_short, surv_n,
                                   cand_n, tau, err);
                        ta = tb;
                    }
                }
                WSTAMP(6);
            }
            if (!have_p) break;
        }
    }
    WSTAMP(7);
    if (surv_n) wave_emit(S, X, P, m, L, sc_long, sc_short, surv_n, cand_n, tau);
    WSTAMP(8);
    wave_flush(S, cand_n, tau, L, X.keys_unique != 0);
    WSTAMP(9);
    if (sliced) {  // this slice's top-L records, in order, for k_merge
        uint64_t* pr = P.prec + ((size_t)q * nsl + slice) * L;
        for (uint32_t i = lane; i < cand_n; i += 64) pr[i] = S.cand()[i];
        if (lane == 0) {
            P.pcnt[(size_t)q * nsl + slice] = cand_n;
            if (!(P.dbg & 32u)) {
                DevStats* sl = stats + (q & (kStatSlots - 1));
                atomicAdd(&sl->postings, (unsigned long long)p_stat);
                atomicAdd(&sl->survivors, (unsigned long long)S.surv_total);
                if (slice == 0) {
                    atomicAdd(&sl->lists, (unsigned long long)ng);
                    atomicAdd(&sl->fast, 1ull);
                }
            }
        }
        return;
    }
    for (uint32_t i = lane; i < cand_n; i += 64) {
        const uint64_t r = S.cand()[i];
        const uint32_t enc = ~(uint32_t)(r >> 32);
        out_k[ob + i] = (uint32_t)r;
        out_s[ob + i] = __uint_as_float(enc - 1u);
    }
    if (lane == 0) out_n[q] = cand_n;
    if (lane == 0 && !(P.dbg & 32u)) {  // dbg 32: no stats atomics
        DevStats* sl = stats + (q & (kStatSlots - 1));
        atomicAdd(&sl->postings, (unsigned long long)p_total);
        atomicAdd(&sl->lists, (unsigned long long)ng);
        atomicAdd(&sl->results, (unsigned long long)cand_n);
        atomicAdd(&sl->fast, 1ull);
        atomicAdd(&sl->survivors, (unsigned long long)S.surv_total);
    }
    WSTAMP(10);
    WPHASE_END(16)
}

// Tier 1a's staging of one part into registers. Lane g < ng brings entries [cur, cur + len)
// of its list: nch 16-byte chunks from position pre = incl - nch of the part's packed chunk
// numbering on (incl: the planner's inclusive prefix sum, mt chunks in all). Lane l loads chunks
// l, 64 + l, ... . A chunk finds its list by counting the list starts below it: every non-empty
// list but the first sets bit (pre - 1) of a 192-bit map, so the ordinal of chunk c's list is the
// map's bits below lane l in word c / 64 (v_mbcnt_lo/hi) plus those of the earlier words; the
// non-empty lists' {first chunk - pre, entry bounds} sit in segtab by ordinal. (stage_part, the
// full kernel's staging, spends a marker array and a max-scan per round on the same lookup.)
template <bool G4>
__device__ __forceinline__ void lean_stage(WaveSmem<true>& S, gptr<uint4> post4, uint64_t gbase,
                                           uint32_t a0, uint32_t cur, uint32_t len, uint32_t nch, uint32_t incl,
                                           uint32_t mt, uint4 (&v)[kDmaRounds], uint32_t& vmask) {
    const uint32_t lane = lane_id();
    const uint32_t head = (a0 + cur) & 3u;
    const uint32_t pre = incl - nch;
    const uint32_t ord = rank_below(__ballot(nch != 0));
    mt = __builtin_amdgcn_readfirstlane(mt);
    uint32_t g4 = 0;
    if constexpr (G4) {
        // the list's chunk base lives in LDS (S.g4, written once per query): values the part loop
        // keeps in registers past 80 VGPRs were spilled to scratch, and a scratch reload's
        // vmcnt(0) waited for every load in flight, the next part's included (the heavy list's
        // launch, with part_ones beside the sketch path, is over the budget; the main one is not)
        uint32_t lz = lane;  // opaque: the slot's address is made here, not kept (and spilled)
        asm volatile("" : "+v"(lz));
        if (nch) g4 = S.g4[lz];
        (void)gbase;
    } else {
        g4 = (uint32_t)(gbase >> 2);
    }
    {
        // the zero and its address made here, for the same reason
        uint32_t z, l = lane;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z), "+v"(l));
        if (l < (uint32_t)kDmaRounds) S.lstart[l] = (unsigned long long)z;
    }
    wave_sync();
    if (nch) {
        if (pre) atomicOr(&S.lstart[(pre - 1) >> 6], 1ull << ((pre - 1) & 63u));
        const uint32_t first = g4 + ((a0 + cur) >> 2);  // the list's chunk base (u32: chunk ids < 2^32)
        S.segtab[ord] = make_uint2(first - pre, (4 * pre + head) | ((4 * pre + head + len) << 16));
    }
    wave_sync();
    uint32_t below = 0;  // list starts in the earlier words
    vmask = 0;
    uint32_t lo = lane;  // opaque: chunk positions are made per round, not hoisted (and spilled)
    asm volatile("" : "+v"(lo));
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        if (64 * r < mt) {
            const unsigned long long wd = S.lstart[r];
            const uint32_t wlo = __builtin_amdgcn_readfirstlane((uint32_t)wd);
            const uint32_t whi = __builtin_amdgcn_readfirstlane((uint32_t)(wd >> 32));
            const uint32_t idx = __builtin_amdgcn_mbcnt_hi(whi, __builtin_amdgcn_mbcnt_lo(wlo, below));
            below += (uint32_t)__popc(wlo) + (uint32_t)__popc(whi);
            const uint32_t c = 64 * r + lo;
            const bool ok = c < mt;
            const uint2 seg = S.segtab[idx & 63u];
            if (ok) v[r] = post4[seg.x + c];  // inactive lanes load nothing
            // entries [lo_e, hi_e) of this chunk are in the list segment [y, z)
            const int y = (int)(seg.y & 0xFFFFu), z = (int)(seg.y >> 16);
            const uint32_t lo_e = (uint32_t)min(max(y - (int)(4 * c), 0), 4);
            const uint32_t hi_e = (uint32_t)min(max(z - (int)(4 * c), 0), 4);
            const uint32_t bits = ((1u << hi_e) - 1u) & ~((1u << lo_e) - 1u);
            vmask |= (ok ? bits : 0u) << (4 * r);
        }
    }
}

// Tier 1a's routing of query q (both lean paths; slice slc of a sliced heavy query): the
// wildcard, empty queries and those past tier 1's gram and limit bounds are answered or listed
// for tier 2 by slice 0, and queries of the other launch (heavy_class: same test, same cmin) are
// left to it. Returns kLeanDone for those, kLeanShort for a short-search query (tier 1b), and
// kLeanCount otherwise, with S.q holding the query, the table clear, and lanes 0..ng-1 its lists.
constexpr uint32_t kLeanDone = 0, kLeanShort = 1, kLeanCount = 2;
struct LeanPlan {
    uint32_t m, n, cmin, ng, glen, grow;
    bool rank;
    uint64_t gbase, p_total;
};
__device__ __forceinline__ uint32_t lean_route(WaveSmem<true>& S, const uint32_t q, const DevIndex& X,
                                               const SearchParams& P, const uint8_t* __restrict__ qnorm,
                                               const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qm,
                                               uint32_t* __restrict__ out_n, uint32_t* __restrict__ out_k,
                                               float* __restrict__ out_s, uint32_t* __restrict__ list2,
                                               uint32_t* __restrict__ count2, uint32_t slc, LeanPlan& lp) {
    const uint32_t lane = lane_id();
    const uint32_t m = qm[q];
    if (m == kQueryWildcard) {  // nGramSearch.hpp:356-369
        if (!slc) wild_answer(X, P, q, lane, 64, out_n, out_k, out_s);
        return kLeanDone;
    }
    if (m == 0) {  // nothing left after normalisation, nGramSearch.hpp:374-375
        if (lane == 0 && !slc) out_n[q] = 0;
        return kLeanDone;
    }
    if (m <= X.full_scan_len || m - X.gsz + 1 > kWaveMaxGrams || P.limit > kWaveMaxLimit) {
        if (lane == 0 && !slc) list2[atomicAdd(count2, 1u)] = q;  // tier 2 / library-wide path
        return kLeanDone;
    }
    const uint32_t n = m - X.gsz + 1;  // grams of the query (hpp:29-36)
    // lane c holds the fp32 score of c hits, (float)c / n (hpp:300); the smallest passing count
    const float sc_long = lane <= n ? (float)lane / (float)n : 0.0f;
    const unsigned long long pm = __ballot(lane <= n && lane > 0 && !(sc_long < P.thr));
    // threshold 0 with rank lists: the multi-hit terms only, k_emit adds the one-hit records
    // (emit_rank_prefix)
    const bool rank = X.rank_post && (pm & 2ull);
    const uint32_t cmin = pm ? (rank ? 2u : (uint32_t)(__ffsll((long long)pm) - 1)) : 1000u;
    const bool short_search = m < X.short_query_len && X.n_short;
    if (!P.lean_all && (cmin <= kHeavyCmin || short_search)) return kLeanDone;
    if (short_search) return kLeanShort;
    const uint8_t* qg = qnorm + qoff[q];
    for (uint32_t i = lane; i < m; i += 64) S.q[i] = char_at(qg, i, X.csize);
    if (lane == 0) S.x_surv_n = 0;  // no arena blocks chained (spill_arena)
    clear_table(S, lane);
    wave_sync();
    // ---- searchLong (nGramSearch.hpp:278-301) ----
    lp.ng = gram_lists(X, [&](uint32_t i) { return S.q[i]; }, n, lane, lp.gbase, lp.glen, lp.grow);
    lp.p_total = wave_sum((uint64_t)lp.glen);
    lp.m = m;
    lp.n = n;
    lp.cmin = cmin;
    lp.rank = rank;
    return kLeanCount;
}

// Tier 1a (LEAN, DEFER): one wave per query, sketch counting only, survivors spilled to HBM for
// k_emit. The full kernel's part loop (bucket groups, term-id sub-parts, loads one part ahead)
// with its own staging (lean_stage) and the sketch counter part_sketch; a query that needs exact
// counting, a short search or more than kEmitCap survivor slots is handed to tier 1b untouched.
template <bool ONES>
__device__ __forceinline__ void lean_query(WaveSmem<true>& S, const uint32_t q, const DevIndex& X,
                                           const SearchParams& P, const uint8_t* __restrict__ qnorm,
                                           const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qm,
                                           uint32_t* __restrict__ out_n, uint32_t* __restrict__ out_k,
                                           float* __restrict__ out_s, uint32_t* __restrict__ list2,
                                           uint32_t* __restrict__ count2, DevStats* __restrict__ stats,
                                           uint32_t* __restrict__ fb, uint32_t* __restrict__ fbc,
                                           const uint32_t slc = 0, const uint32_t nsl = 1) {
    const uint32_t lane = lane_id();
    // term-id slice slc of nsl (the heavy list's launch): the query's slices run on separate waves,
    // take survivor slots from a per-query word (heavy_slot) and the last to finish publishes the
    // count; a slice that hands the query over marks it there, and only the first one lists it
    uint32_t nslq = 1;  // slices of this query (cmin-1 queries run whole, in slice 0)
    auto finish_slice = [&]() {
        uint32_t old = 0;
        if (lane == 0) old = atomicAdd(&P.eovf[q], kHeavyDone);
        old = __builtin_amdgcn_readfirstlane(old);
        if (((old / kHeavyDone) & 127u) == nslq - 1u && !(old & kHeavyBailed) && lane == 0)
            P.esn[q] = (old & kHeavySlotMask) | kEmitHeavy;  // the query's last slice
    };
    auto bail = [&]() {  // hand the query to tier 1b (nothing of it was written yet)
        if (nslq > 1) {
            uint32_t old = 0;
            if (lane == 0) old = atomicOr(&P.eovf[q], kHeavyBailed);
            old = __builtin_amdgcn_readfirstlane(old);
            if (!(old & kHeavyBailed) && lane == 0) fb[atomicAdd(fbc, 1u)] = q;
            finish_slice();
        } else if (lane == 0) {
            fb[atomicAdd(fbc, 1u)] = q;
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    };
    WPHASE_BEGIN
    LeanPlan lp;
    const uint32_t route = lean_route(S, q, X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, slc, lp);
    if (route != kLeanCount) {
        if (route == kLeanShort && !slc) bail();  // short search: tier 1b
        return;
    }
    const uint32_t L = P.limit, n = lp.n, cmin = lp.cmin, ng = lp.ng, glen = lp.glen, grow = lp.grow;
    const uint32_t n_long = X.n_terms - X.n_short;
    const bool rank = lp.rank;
    const uint64_t gbase = lp.gbase, p_total = lp.p_total;
    WSTAMP(0);
    const bool sketch = cmin >= kSketchMinCmin && cmin <= kSketchMax;
    const bool ones = ONES && cmin == 1;  // part_ones (the heavy list's launch only)
    constexpr bool kG4 = ONES;  // list chunk bases in LDS (lean_stage; for every query: 1.5 % slower)
    if (p_total && cmin <= n && !sketch && !ones) {  // exact counting: tier 1b
        if (!slc) bail();
        return;
    }
    // (a slice per kHeavySlicePostings postings, unless NGS_HEAVY_SLICES forces them)
    nslq = ones || !p_total || cmin > n ? 1u
         : P.hslices ? nsl : (uint32_t)min64(nsl, max64(1, p_total / kHeavySlicePostings));
    if (slc >= nslq) return;
    uint32_t surv_n = 0, spilled = 0;
    // rank lists: the query's lists for k_emit (emit_rank_prefix) in its last kRankInfo slots
    const uint32_t ecap_q = P.ecap - (rank ? kRankInfo : 0u);
    if (rank && !slc) {
        uint32_t* ri = P.est + (size_t)q * P.ecap + ecap_q;
        ri[lane] = (uint32_t)gbase;
        ri[64 + lane] = (uint32_t)(gbase >> 32);
        ri[128 + lane] = min(glen, L);
    }
    // the LDS survivor list to this query's kEmitCap slots in HBM; false if they are full
    auto spill = [&]() -> bool {
        uint32_t at = spilled;
        if (nslq > 1 && surv_n) {  // a sliced query's slots are shared: take them from its word
            uint32_t b0 = 0;
            if (lane == 0) b0 = atomicAdd(&P.eovf[q], surv_n);
            at = __builtin_amdgcn_readfirstlane(b0) & kHeavySlotMask;
        }
        if (at + surv_n > ecap_q) return false;
        uint32_t qs = q, l0 = lane;  // opaque: the slot pointers are made here, not kept (and spilled)
        asm volatile("" : "+s"(qs), "+v"(l0));
        uint32_t* et = P.est + (size_t)qs * P.ecap + at;
        uint8_t* ec = P.esc + (size_t)qs * P.ecap + at;
        for (uint32_t i = l0; i < surv_n; i += 64) {
            et[i] = S.surv_t[i];
            ec[i] = S.surv_c[i];
        }
        spilled += surv_n;
        surv_n = 0;
        return true;
    };
    // counted for the host, which grows the slots of later calls (ensure_queries)
    auto slot_full = [&]() {
        if (lane == 0 && !(P.dbg & 32u)) atomicAdd(&stats[q & (kStatSlots - 1)].slot_full, 1u);
    };
    if (p_total && cmin <= n) {
        // cmin 2: every colliding pair is a false candidate, so those parts are cut at half the size;
        // a gram the query repeats makes every term of its list a candidate, so a list held by mu
        // lanes cuts them further (the part's candidates stay within the 64 a part resolves)
        uint32_t shrink = ones ? kOnesShrink : cmin == 2 ? kLeanShrink2 : 0u;
        if (cmin == 2) {
            uint32_t mu = 0;
            for (uint32_t k = 0; k < ng; ++k)
                mu += gbase == (((uint64_t)__builtin_amdgcn_readlane((uint32_t)(gbase >> 32), (int)k) << 32) |
                                __builtin_amdgcn_readlane((uint32_t)gbase, (int)k)) ? 1u : 0u;
            const unsigned long long dup = __ballot(lane < ng && mu >= 2), dup3 = __ballot(lane < ng && mu >= 3);
            shrink += (dup ? 1u : 0u) + (dup3 ? 1u : 0u);
        }
        const uint32_t kChunks = (uint32_t)kWaveChunks >> shrink;  // part cap in 16-byte chunks
        const uint32_t K = X.n_buckets, span = X.bucket_span;
        const uint32_t wmax = (uint32_t)max64(1, min64(K, kMaxPartSpan / max(span, 1u)));
        const uint32_t w = (uint32_t)max64(1, min64(wmax, (uint64_t)K * (kSketchTarget >> shrink) / p_total));
        const uint32_t* sk = X.skip + (size_t)grow * (K + 1);
        // this slice's buckets [b0, Kend)
        const uint32_t b0 = K * slc / nslq, Kend = K * (slc + 1) / nslq;
        // an opaque SGPR pair: otherwise the compiler keeps it inside the 8-dword kernarg tuple it
        // loaded it with and reloads all 8 dwords from VGPR lanes (v_readlane, VALU) every round
        gptr<uint4> post4 = (gptr<uint4>)reinterpret_cast<const uint4*>(X.post);
        asm volatile("" : "+s"(post4));
        const uint32_t a0 = (uint32_t)gbase & 3u;  // list start within its 16-byte chunk
        if (kG4) S.g4[lane] = (uint32_t)(gbase >> 2);  // ... and its chunk (post holds < 2^34 entries)
        // entries [s, e) of this lane's list cover 16-byte chunks [(a0 + s) / 4, (a0 + e + 3) / 4)
        auto chunks = [a0](uint32_t s, uint32_t e) -> uint32_t { return e > s ? ((a0 + e + 3) >> 2) - ((a0 + s) >> 2) : 0u; };
        // end of the next bucket group: skip[row][min(K, bn + w)]; idle lanes load nothing
        auto next_end = [&](uint32_t bn) -> uint32_t { return sk[min(Kend, bn + w)]; };
        uint32_t cur = b0 && lane < ng ? sk[b0] : 0u, bnext = b0;
        uint32_t e_pre = lane < ng ? next_end(b0) : 0u;
        uint32_t in_sub = 0, sub_lo = 0, hi_lim = 0, sub_end = 0, sub_bnext = 0, step = 1;
        // software pipeline in registers: part i+1's loads are in flight while part i is counted
        uint4 pv[kDmaRounds];
        uint32_t p_vm = 0, p_mt = 0;
        bool have_p = false;
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) pv[r] = make_uint4(0, 0, 0, 0);
        unsigned* err = &stats->errors;
        WSTAMP(1);
        for (uint32_t guard = 0;;) {
            uint4 cv[kDmaRounds];
#pragma unroll
            for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) cv[r] = pv[r];
            const uint32_t c_vm = p_vm, c_mt = p_mt;
            const bool have_c = have_p;
            // ---- next part: per list lane the segment [cur, cur + len) ----
            uint32_t len = 0, nch = 0, incl = 0, tot = 0;  // the part's per-list chunks, their prefix sum, total
            have_p = false;
            in_sub = __builtin_amdgcn_readfirstlane(in_sub);
            bnext = __builtin_amdgcn_readfirstlane(bnext);
            bool fast = false;
            if (!in_sub && bnext < Kend) {  // common case, straight-line: the next bucket group fits
                const uint32_t e = lane < ng ? e_pre : cur;
                nch = chunks(cur, e);
                incl = wave_incl_scan(nch);
                tot = __builtin_amdgcn_readlane(incl, 63);
                if (tot && tot <= kChunks) {
                    len = e - cur;
                    bnext = min(Kend, bnext + w);
                    if (lane < ng) e_pre = next_end(bnext);
                    have_p = true;
                    fast = true;  // e_pre of the next group loads after this part's loads (below)
                }
            }
            WSTAMP(2);
            for (; !fast;) {
                WCOUNT(12, 1);
                guard = __builtin_amdgcn_readfirstlane(guard);
                bnext = __builtin_amdgcn_readfirstlane(bnext);
                sub_lo = __builtin_amdgcn_readfirstlane(sub_lo);
                step = __builtin_amdgcn_readfirstlane(step);
                if (++guard > 8u * K + 4096u) {
                    atomicOr(err, 4u);  // every lane (idempotent)
                    break;
                }
                if (!in_sub) {
                    if (bnext >= Kend) break;
                    const uint32_t bhi = min(Kend, bnext + w), e = lane < ng ? e_pre : cur;
                    nch = chunks(cur, e);
                    incl = wave_incl_scan(nch);
                    tot = __builtin_amdgcn_readlane(incl, 63);
                    if (tot <= kChunks) {
                        len = e - cur;
                        bnext = bhi;
                        if (lane < ng) e_pre = next_end(bnext);
                        if (tot) { have_p = true; break; }
                        continue;
                    }
                    in_sub = 1;  // the group is over the cap: term-id sub-ranges of it
                    sub_lo = bnext * span;
                    hi_lim = (uint32_t)min64((uint64_t)bhi * span, n_long);
                    sub_end = e;
                    sub_bnext = bhi;
                    step = (uint32_t)max64(1, min64((uint64_t)(hi_lim - sub_lo) * (kChunks * 3 / 4) / max(tot, 1u),
                                                    kMaxPartSpan));
                }
                const uint32_t hi = (uint32_t)min64(hi_lim, (uint64_t)sub_lo + step);
                // lower_bound(list, hi) per lane, as a ballot-controlled (uniform) loop
                uint32_t a = cur, b = lane < ng ? sub_end : cur;
                while (__ballot(a < b)) {
                    const bool act = a < b;
                    const uint32_t mid = (a + b) >> 1;
                    uint32_t pvv = 0;
                    if (act) pvv = X.post[gbase + mid];
                    const bool below = pvv < hi;
                    a = act && below ? mid + 1 : a;
                    b = act && !below ? mid : b;
                }
                nch = lane < ng ? chunks(cur, a) : 0u;
                incl = wave_incl_scan(nch);
                const uint32_t t2 = __builtin_amdgcn_readlane(incl, 63);
                tot = t2;
                if (t2 > kChunks && hi - sub_lo > 1) {
                    step = max(1u, (uint32_t)((uint64_t)(hi - sub_lo) * (kChunks * 3 / 4) / t2));
                    continue;
                }
                len = lane < ng ? a - cur : 0u;
                sub_lo = hi;
                if (sub_lo >= hi_lim) {
                    in_sub = 0;
                    bnext = sub_bnext;
                    if (lane < ng) e_pre = next_end(bnext);
                }
                if (t2) { have_p = true; break; }
                cur = a;
            }
            WSTAMP(3);
            have_p = __builtin_amdgcn_readfirstlane(have_p ? 1u : 0u) != 0;
            // ---- part i+1: issue this wave's loads ----
            if (have_p) {
                lean_stage<kG4>(S, post4, gbase, a0, cur, len, nch, incl, tot, pv, p_vm);
                p_mt = tot;
                cur += len;
            }
            WSTAMP(4);
            // ---- count part i while part i+1 is in flight ----
            if (have_c) {
                if (surv_n + 64 > (uint32_t)kWaveSurv) {
                    if (!spill()) { slot_full(); bail(); return; }
                    wave_sync();  // the list is read before it is refilled
                }
                uint32_t nc;
                if constexpr (ONES) {
                    // the query's slot pointers made here from an opaque copy of q (SALU, per part):
                    // hoisted out of the loop they were two 64-bit VGPR pairs spilled to scratch
                    uint32_t qs = q;
                    asm volatile("" : "+s"(qs));
                    nc = ones ? part_ones(S, cv, c_vm, c_mt, X.n_short, X.n_terms, surv_n, P.est + (size_t)qs * P.ecap,
                                          P.esc + (size_t)qs * P.ecap, spilled, P.ecap)
                              : part_sketch(S, cv, c_vm, c_mt, cmin, X.n_short, X.n_terms, surv_n);
                }
                else
                    nc = part_sketch(S, cv, c_vm, c_mt, cmin, X.n_short, X.n_terms, surv_n);
                WCOUNT(11, 1);
                WCOUNT(13, (c_mt + 63) / 64);
                WCOUNT(14, nc);
                WCOUNT(15, nc == 0 ? 1 : 0);
                WSTAMP(5);
                if (nc > 64) { bail(); return; }  // wrapped counter or too many candidates: tier 1b
            }
            if (!have_p) break;
        }
    }
    if (!spill()) { slot_full(); bail(); return; }
    WSTAMP(6);
    WPHASE_END(16)
    if (nslq > 1) finish_slice();
    else if (lane == 0) P.esn[q] = spilled | (P.lean_all ? kEmitHeavy : 0u);
    if (lane == 0 && !(P.dbg & 32u)) {
        DevStats* sl = stats + (q & (kStatSlots - 1));
        if (!slc) {
            atomicAdd(&sl->postings, (unsigned long long)p_total);
            atomicAdd(&sl->lists, (unsigned long long)ng);
            atomicAdd(&sl->fast, 1ull);
        }
        atomicAdd(&sl->survivors, (unsigned long long)spilled);
    }
}

// Tier 1a with lane groups (the main launch): each of the query's lists owns a fixed group of lanes
// for the whole query, sized in proportion to its length (quota_j = 1 + (64 - ng) * len_j / P lanes).
// Lane `slot` of list j's group loads chunks slot, slot + G, slot + 2G of that list's segment in
// each part, so a chunk never has to find its list: no per-part prefix sum, list-start map or
// segment table, no LDS round trips before a load. A part fits when no list has more than
// 3 G chunks (its lanes' three register rounds). The part's entry bounds are applied only where a
// cell reached cmin (the sketch counts the <= 3 neighbouring entries at each segment edge, never an
// undercount): entry e of chunk k is in the segment iff 4k + e - head < len.

// sketch count of a part staged by lane groups (3 <= cmin <= 15): part_sketch's one-wave loose path
__device__ __forceinline__ uint32_t lean_sketch_g(WaveSmem<true>& S, const uint4 (&v)[kDmaRounds], uint32_t R,
                                                  uint32_t k0, uint32_t G, uint32_t nch, uint32_t head, uint32_t len,
                                                  uint32_t cmin, uint32_t n_short, uint32_t n_terms, uint32_t& surv_n) {
    const uint32_t lane = lane_id();
    R = __builtin_amdgcn_readfirstlane(R);
    const uint32_t cm1 = __builtin_amdgcn_readfirstlane(cmin - 1u);
    uint32_t seen = 0;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        if (r < R && k0 + r * G < nch) {
            const uint32_t t[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            uint32_t old[4];
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e)
                old[e] = atomicAdd(sketch_word<true>(S.table, t[e]), 1u << (sketch_sh4<true>(t[e]) & 31u));
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) seen = max(seen, __builtin_amdgcn_ubfe(old[e], sketch_sh4<true>(t[e]), 4u));
        }
    }
    const bool ovf = seen == kSketchMax, hot = seen >= cm1;
    wave_sync();
    if (!__ballot(hot || ovf)) {  // no cell reached cmin: no candidates
        clear_table(S, lane);
        wave_sync();
        return 0;
    }
    const uint32_t ov = __ballot(ovf) ? 65u : 0u;  // a wrapped counter: exact counting (tier 1b)
    uint32_t nw = 0;
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
        if (r < R) {
            const uint32_t t[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
            uint32_t w[4];
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) w[e] = *sketch_word<true>(S.table, t[e]);
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) {
                bool f = __builtin_amdgcn_ubfe(w[e], sketch_sh4<true>(t[e]), 4u) >= cmin;
                if (__ballot(f)) {  // rare: the entry's segment bounds (and chunks not loaded) only here
                    uint32_t kk = k0;  // opaque: the round's entry offset is made here, not kept across the part loop
                    asm volatile("" : "+v"(kk));
                    f = f && 4u * (kk + r * G) + e - head < len;
                    const unsigned long long b = __ballot(f);
                    const uint32_t pos = nw + rank_below(b);
                    if (f && pos < 64u) S.cbuf[pos] = t[e];
                    nw += (uint32_t)__popcll(b);
                }
            }
        }
    }
    const uint32_t nc = nw + ov;
    wave_sync();
    clear_table(S, lane);
    if (nc && nc <= 64) cand_counts(S, nc, cmin, n_short, n_terms, surv_n);
    wave_sync();
    return nc;
}

// a staged part of lean_query_g: its chunks per lane's list, first entry in the first chunk, entries,
// rounds (0: no part)
struct PartGroups {
    uint32_t nch, head, len, R;
};

__device__ __forceinline__ void lean_query_g(WaveSmem<true>& S, const uint32_t q, const DevIndex& X,
                                             const SearchParams& P, const uint8_t* __restrict__ qnorm,
                                             const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qm,
                                             uint32_t* __restrict__ out_n, uint32_t* __restrict__ out_k,
                                             float* __restrict__ out_s, uint32_t* __restrict__ list2,
                                             uint32_t* __restrict__ count2, DevStats* __restrict__ stats,
                                             uint32_t* __restrict__ fb, uint32_t* __restrict__ fbc) {
    const uint32_t lane = lane_id();
    auto bail = [&]() {  // hand the query to tier 1b (nothing of it was written yet)
        if (lane == 0) fb[atomicAdd(fbc, 1u)] = q;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    };
    WPHASE_BEGIN
    LeanPlan lp;
    const uint32_t route = lean_route(S, q, X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, 0u, lp);
    if (route != kLeanCount) {
        if (route == kLeanShort) bail();  // short search: tier 1b
        return;
    }
    const uint32_t L = P.limit, n = lp.n, cmin = lp.cmin, ng = lp.ng, glen = lp.glen, grow = lp.grow;
    const uint32_t n_long = X.n_terms - X.n_short;
    const bool rank = lp.rank;
    const uint64_t gbase = lp.gbase, p_total = lp.p_total;
    WSTAMP(0);
    const bool sketch = cmin >= kSketchMinCmin && cmin <= kSketchMax;
    if (p_total && cmin <= n && !sketch) { bail(); return; }  // exact counting: tier 1b
    uint32_t surv_n = 0, spilled = 0;
    // rank lists: the query's lists for k_emit (emit_rank_prefix) in its last kRankInfo slots
    const uint32_t ecap_q = P.ecap - (rank ? kRankInfo : 0u);
    if (rank) {
        uint32_t* ri = P.est + (size_t)q * P.ecap + ecap_q;
        ri[lane] = (uint32_t)gbase;
        ri[64 + lane] = (uint32_t)(gbase >> 32);
        ri[128 + lane] = min(glen, L);
    }
    // the LDS survivor list to this query's ecap slots in HBM, and past them to blocks of the batch's
    // arena (SearchParams.at); false if neither has room
    // (arena blocks chained so far and the last two of them live in LDS words tier 1a does not use,
    // not in registers across the part loop: the arena is the rare path)
    uint32_t a_held = 0;  // the arena ran out for this query: 1 + the blocks it holds (arena_need)
    auto spill_arena = [&]() -> bool {  // (rare: survivors past the query's slots)
        const uint32_t end = spilled + surv_n;
        const uint32_t k1 = (end - 1u - ecap_q) / kArenaBlock;  // last chained block the spill needs
        uint32_t a_n = __builtin_amdgcn_readfirstlane(S.x_surv_n), a_last = __builtin_amdgcn_readfirstlane(S.x_cand_n);
        uint32_t a_prev = __builtin_amdgcn_readfirstlane(S.xcnt);
        while (a_n <= k1) {
            if (a_n >= kArenaChain) return false;
            uint32_t nb = 0;
            if (lane == 0) nb = atomicAdd(P.actr, 1u);
            nb = __builtin_amdgcn_readfirstlane(nb);
            if (nb >= P.ablocks) {  // the arena ran out (the counter tells the host)
                a_held = a_n + 1u;
                return false;
            }
            if (lane == 0) {
                P.anext[nb] = 0;
                if (a_n == 0) P.eovf[q] = nb + 1u;
                else P.anext[a_last] = nb + 1u;
            }
            a_prev = a_last;
            a_last = nb;
            ++a_n;
        }
        wave_sync();
        if (lane == 0) {
            S.x_surv_n = a_n;
            S.x_cand_n = a_last;
            S.xcnt = a_prev;
        }
        for (uint32_t i = lane; i < surv_n; i += 64) {
            const uint32_t p = spilled + i;
            if (p < ecap_q) {
                P.est[(size_t)q * P.ecap + p] = S.surv_t[i];
                P.esc[(size_t)q * P.ecap + p] = S.surv_c[i];
            } else {
                const uint32_t ap = p - ecap_q, k = ap / kArenaBlock;
                const size_t at = (size_t)(k + 1u == a_n ? a_last : a_prev) * kArenaBlock + (ap - k * kArenaBlock);
                P.at[at] = S.surv_t[i];
                P.ac[at] = S.surv_c[i];
            }
        }
        spilled = end;
        surv_n = 0;
        return true;
    };
    auto spill = [&]() -> bool {
        if (spilled + surv_n > ecap_q) return P.at && spill_arena();
        uint32_t qs = q, l0 = lane;  // opaque: the slot pointers are made here, not kept (and spilled)
        asm volatile("" : "+s"(qs), "+v"(l0));
        uint32_t* et = P.est + (size_t)qs * P.ecap + spilled;
        uint8_t* ec = P.esc + (size_t)qs * P.ecap + spilled;
        for (uint32_t i = l0; i < surv_n; i += 64) {
            et[i] = S.surv_t[i];
            ec[i] = S.surv_c[i];
        }
        spilled += surv_n;
        surv_n = 0;
        return true;
    };
    // counted for the host, which grows the slots of later calls (ensure_queries)
    auto slot_full = [&]() {
        if (lane == 0 && !(P.dbg & 32u)) atomicAdd(&stats[q & (kStatSlots - 1)].slot_full, 1u);
    };
    // a query the arena ran out for: the blocks it would still need, from its survivors so far and
    // the share of its postings counted (p_done of p_total), for the host's next arena size
    auto arena_need = [&](uint32_t p_done) {
        if (!a_held) return;
        const uint64_t est = (uint64_t)(spilled + surv_n) * p_total / max(p_done, 1u);
        const uint64_t need = est > ecap_q ? (est - ecap_q + kArenaBlock - 1u) / kArenaBlock : 0u;
        const uint64_t more = min64(need > a_held - 1u ? need - (a_held - 1u) : 0u, kArenaChain);
        if (lane == 0) atomicAdd(P.actr + 1, (uint32_t)more);
    };
    if (p_total && cmin <= n) {
        // ---- lane groups: list j owns lanes [gend_j - gq_j, gend_j), gq_j = 1 + (64 - ng) len_j / P ----
        const uint32_t quota = lane < ng ? 1u + (uint32_t)(((uint64_t)(64u - ng) * glen) / p_total) : 0u;
        const uint32_t qincl = wave_incl_scan(quota);
        uint32_t jl = 0;  // this lane's list: the lists whose groups end at or below it
        for (uint32_t k = 0; k < ng; ++k) jl += lane >= (uint32_t)__builtin_amdgcn_readlane(qincl, k) ? 1u : 0u;
        const bool has = jl < ng;
        const int js = (int)(has ? jl : 0u);
        const uint32_t G = has ? (uint32_t)__shfl(quota, js) : 1u;  // the group's size
        const uint32_t k0 = lane - ((uint32_t)__shfl(qincl, js) - G);  // this lane's slot in it
        const uint64_t lbase = __shfl(gbase, js);
        const uint32_t lrow = (uint32_t)__shfl(grow, js);
        // cmin 2: every colliding pair is a false candidate, so those parts are cut at half the size
        const uint32_t shrink = cmin == 2 ? kLeanShrink2 : 0u;
        // chunks a part may hold of this lane's list: its lanes' three rounds (cut as the sketch part is)
        const uint32_t capc = has ? min(3u * G, max(2u, (3u * G) >> shrink)) : 0u;
        const uint32_t K = X.n_buckets, span = X.bucket_span;
        const uint32_t wmax = (uint32_t)max64(1, min64(K, kMaxPartSpan / max(span, 1u)));
        const uint32_t w = (uint32_t)max64(1, min64(wmax, (uint64_t)K * (kGroupTarget >> shrink) / p_total));
        const uint32_t skrow = lrow * (K + 1);
        constexpr uint32_t b0 = 0;
        const uint32_t Kend = K;
        WSTAMP(1);
        gptr<uint4> post4 = (gptr<uint4>)reinterpret_cast<const uint4*>(X.post);
        asm volatile("" : "+s"(post4));
        const uint32_t a0 = (uint32_t)lbase & 3u;      // list start within its 16-byte chunk
        const uint32_t cb = (uint32_t)(lbase >> 2);    // ... and its chunk (post holds < 2^34 entries)
        // entries [s, e) of this lane's list cover 16-byte chunks [(a0 + s) / 4, (a0 + e + 3) / 4)
        auto chunks = [a0](uint32_t s, uint32_t e) -> uint32_t { return e > s ? ((a0 + e + 3) >> 2) - ((a0 + s) >> 2) : 0u; };
        // end of the next bucket group: skip[row][min(K, bn + w)]; lanes without a list load nothing
        auto next_end = [&](uint32_t bn) -> uint32_t { return X.skip[skrow + min(Kend, bn + w)]; };
        // fill of the fullest list against its cap, in 1/256: sub-part steps aim at 3/4 of it
        auto fill = [&](uint32_t nc) -> uint32_t {
            const uint32_t f = has ? (nc * 256u + capc - 1u) / capc : 0u;
            return max(1u, __builtin_amdgcn_readlane(wave_incl_max_scan(f), 63));
        };
        uint32_t cur = 0, bnext = b0;
        if (b0) cur = has ? X.skip[skrow + b0] : 0u;
        uint32_t e_pre = has ? next_end(b0) : 0u;
        // the first skip-table read waited for here: the loop header then merges only the back
        // edge's pending loads (with this one pending the wait there was vmcnt(0) on every part)
        asm volatile("" ::"v"(e_pre));
        uint32_t in_sub = 0, sub_lo = 0, hi_lim = 0, sub_end = 0, sub_bnext = 0, step = 1;
        unsigned* err = &stats->errors;
        uint32_t guard = 0;
        // ---- the next part: per lane its list's segment [cur, cur + len) of nch chunks ----
        auto plan = [&](uint32_t& nch, uint32_t& len) -> bool {
            bool have_p = false;
            in_sub = __builtin_amdgcn_readfirstlane(in_sub);
            bnext = __builtin_amdgcn_readfirstlane(bnext);
            if (!in_sub && bnext < Kend) {  // common case, straight-line: the next bucket group fits
                const uint32_t e = has ? e_pre : cur;
                nch = chunks(cur, e);
                if (!__ballot(nch > capc) && __ballot(nch != 0)) {
                    len = e - cur;
                    bnext = min(Kend, bnext + w);
                    if (has) e_pre = next_end(bnext);
                    return true;
                }
            }
            for (;;) {
                guard = __builtin_amdgcn_readfirstlane(guard);
                bnext = __builtin_amdgcn_readfirstlane(bnext);
                sub_lo = __builtin_amdgcn_readfirstlane(sub_lo);
                step = __builtin_amdgcn_readfirstlane(step);
                if (++guard > 8u * K + 4096u) {
                    atomicOr(err, 4u);  // every lane (idempotent)
                    break;
                }
                if (!in_sub) {
                    if (bnext >= Kend) break;
                    const uint32_t bhi = min(Kend, bnext + w), e = has ? e_pre : cur;
                    nch = chunks(cur, e);
                    if (!__ballot(nch > capc)) {
                        len = e - cur;
                        bnext = bhi;
                        if (has) e_pre = next_end(bnext);
                        if (__ballot(nch != 0)) { have_p = true; break; }
                        continue;
                    }
                    in_sub = 1;  // the group is over a list's cap: term-id sub-ranges of it
                    sub_lo = bnext * span;
                    hi_lim = (uint32_t)min64((uint64_t)bhi * span, n_long);
                    sub_end = e;
                    sub_bnext = bhi;
                    step = (uint32_t)max64(1, min64((uint64_t)(hi_lim - sub_lo) * 192u / fill(nch), kMaxPartSpan));
                }
                const uint32_t hi = (uint32_t)min64(hi_lim, (uint64_t)sub_lo + step);
                // lower_bound(list, hi) per lane, as a ballot-controlled (uniform) loop
                uint32_t a = cur, b = has ? sub_end : cur;
                while (__ballot(a < b)) {
                    const bool act = a < b;
                    const uint32_t mid = (a + b) >> 1;
                    uint32_t pvv = 0;
                    if (act) pvv = X.post[lbase + mid];
                    const bool below = pvv < hi;
                    a = act && below ? mid + 1 : a;
                    b = act && !below ? mid : b;
                }
                nch = has ? chunks(cur, a) : 0u;
                if (__ballot(nch > capc) && hi - sub_lo > 1) {
                    step = max(1u, (uint32_t)((uint64_t)(hi - sub_lo) * 192u / fill(nch)));
                    continue;
                }
                len = has ? a - cur : 0u;
                sub_lo = hi;
                if (sub_lo >= hi_lim) {
                    in_sub = 0;
                    bnext = sub_bnext;
                    if (has) e_pre = next_end(bnext);
                }
                if (__ballot(nch != 0)) { have_p = true; break; }
                cur = a;
            }
            return __builtin_amdgcn_readfirstlane(have_p ? 1u : 0u) != 0;
        };
        // ---- a planned part's loads (lane k0 of its group: chunks k0, k0 + G, k0 + 2G) ----
        auto stage = [&](uint4 (&v)[kDmaRounds], PartGroups& ps, uint32_t nch, uint32_t len) {
            const uint32_t R = 1u + (__ballot(nch > G) ? 1u : 0u) + (__ballot(nch > 2u * G) ? 1u : 0u);
            const uint32_t head = (a0 + cur) & 3u;
            const uint32_t first = cb + ((a0 + cur) >> 2);
#pragma unroll
            for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) {
                const uint32_t k = k0 + r * G;
                if (r < R && k < nch) v[r] = post4[first + k];  // lanes past their list's segment load nothing
            }
            ps.nch = nch;
            ps.head = head;
            ps.len = len;
            ps.R = R;
            cur += len;
        };
        // ---- count a part; false: the query goes to tier 1b ----
#ifdef NGS_PHASE_STAMPS
        uint32_t last_nc = 0;  // candidates of the last part counted (phase statistics)
#endif
        auto count = [&](const uint4 (&v)[kDmaRounds], const PartGroups& ps) -> bool {
            if (surv_n + 64 > (uint32_t)kWaveSurv) {
                if (!__builtin_amdgcn_readfirstlane(spill() ? 1u : 0u)) {  // (uniform: no exec-masked exit)
                    slot_full();
                    // (DPP sum: a shuffle sum's lane-index vectors would be hoisted out of the part loop)
                    arena_need(wave_sum_u32(has && k0 == 0 ? cur : 0u));
                    return false;
                }
                wave_sync();  // the list is read before it is refilled
            }
            const uint32_t nc = lean_sketch_g(S, v, ps.R, k0, G, ps.nch, ps.head, ps.len, cmin, X.n_short, X.n_terms, surv_n);
#ifdef NGS_PHASE_STAMPS
            last_nc = nc;
#endif
            return __builtin_amdgcn_readfirstlane(nc) <= 64;  // above: a wrapped counter or too many candidates
        };
        // software pipeline in registers: part i+1's loads are in flight while part i is counted
        uint4 pv[kDmaRounds];
        PartGroups ps{};
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) pv[r] = make_uint4(0, 0, 0, 0);
        for (;;) {
            uint4 cv[kDmaRounds];
#pragma unroll
            for (uint32_t r = 0; r < (uint32_t)kDmaRounds; ++r) cv[r] = pv[r];
            const PartGroups cs = ps;
            uint32_t nch = 0, len = 0;
            const bool hp = plan(nch, len);
            WSTAMP(2);
            if (hp) stage(pv, ps, nch, len);
            WSTAMP(4);
            if (cs.R && !count(cv, cs)) { bail(); return; }  // count part i while part i+1 is in flight
            WSTAMP(5);
            WCOUNT(11, cs.R ? 1 : 0);
            WCOUNT(13, cs.R);
            WCOUNT(14, cs.R ? last_nc : 0);
            WCOUNT(15, cs.R && last_nc == 0 ? 1 : 0);
            ps.R = hp ? ps.R : 0u;
            if (!hp) break;
        }
    }
    if (!spill()) {
        slot_full();
        arena_need((uint32_t)p_total);
        bail();
        return;
    }
    WSTAMP(6);
    WPHASE_END(32)
    if (lane == 0) P.esn[q] = spilled | (P.lean_all ? kEmitHeavy : 0u);
    if (lane == 0 && !(P.dbg & 32u)) {
        DevStats* sl = stats + (q & (kStatSlots - 1));
        atomicAdd(&sl->postings, (unsigned long long)p_total);
        atomicAdd(&sl->lists, (unsigned long long)ng);
        atomicAdd(&sl->fast, 1ull);
        atomicAdd(&sl->survivors, (unsigned long long)spilled);
        if (!P.lean_all) {
            atomicAdd(&sl->main_postings, (unsigned long long)p_total);
            atomicAdd(&sl->main_lists, (unsigned long long)ng);
        }
    }
}

// Tier 1b / experiments: the full wave kernel, over every query (qlist == nullptr) or over the
// queries tier 1a handed over (qlist[0 .. *qcount), grid-stride).
__global__ __launch_bounds__(64, kWaveWavesPerSimd) void k_wave(DevIndex X, SearchParams P,
                                                                   const uint8_t* __restrict__ qnorm,
                                                                   const uint64_t* __restrict__ qoff,
                                                                   const uint32_t* __restrict__ qm,
                                                                   uint32_t* __restrict__ out_n,
                                                                   uint32_t* __restrict__ out_k,
                                                                   float* __restrict__ out_s,
                                                                   uint32_t* __restrict__ list2,
                                                                   uint32_t* __restrict__ count2,
                                                                   DevStats* __restrict__ stats,
                                                                   const uint32_t* __restrict__ qlist,
                                                                   const uint32_t* __restrict__ qcount) {
    __shared__ WaveSmem<> S;
    const uint32_t nsl = P.nslices > 1 ? P.nslices : 1u;  // sliced: k_merge follows
    if (!qlist) {  // every query of the batch: a workgroup per (query, slice)
        const uint32_t q = blockIdx.x / nsl;
        wave_query(S, q, X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, stats, nullptr,
                             nullptr, blockIdx.x - q * nsl, nsl);
        return;
    }
    const uint32_t cnt = *qcount;
    if (P.qhead) {
        // a persistent grid of about one workgroup per slot of the GPU pulls (query, slice) items:
        // a near-empty list no longer dispatches B x slices workgroups beside tier 1a, and a long
        // one balances like the hardware dispatcher did. Workgroups beyond the item count leave
        // without touching the counter (thousands of atomics on one address serialise: C2's
        // empty lists cost 80 us that way)
        const uint32_t items = cnt * nsl;
        if (blockIdx.x >= items) return;
        for (uint32_t t = blockIdx.x;;) {
            if (t >= items) break;
            const uint32_t i = t / nsl;
            wave_query(S, qlist[i], X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, stats,
                                 nullptr, nullptr, t - i * nsl, nsl);
            __syncthreads();
            // the first gridDim.x items went one to a workgroup; the rest are pulled in turn
            uint32_t nt = 0;
            if (threadIdx.x == 0) nt = gridDim.x + atomicAdd(P.qhead, 1u);
            t = __builtin_amdgcn_readfirstlane(nt);  // (every lane active: lane 0 holds it)
        }
        return;
    }
    for (uint32_t t = blockIdx.x; t < cnt * nsl; t += gridDim.x) {
        const uint32_t i = t / nsl;
        wave_query(S, qlist[i], X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, stats,
                             nullptr, nullptr, t - i * nsl, nsl);
        __syncthreads();
    }
}



// ngsServe: the persistent low-latency server, one wave per request slot (kServeSlots, so that
// concurrent score() callers are answered side by side). A wave polls its slot's request block
// (coherent pinned host memory) with system-scope loads, answers each request with wave_query
// (the tier-1 wave search, unsliced) writing the results straight into the block, then publishes
// the request's number behind a system-scope release. The waves exit together: on slot 0's stop
// flag, after idle_ms without a request on any slot (`last`: the latest request time, raised by
// every wave) or after life_ms in all (the host relaunches them on the next call), so the server
// can never outlive its process by more than that. s_memrealtime (100 MHz) is read through the
// scalar unit: a read.
__device__ __forceinline__ uint64_t sys_load64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t sys_load32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_serve(DevIndex X, SearchParams P0, ServeBlock* blk0, DevStats* scratch0,
                                              uint32_t* list20, unsigned long long* t_any, uint32_t idle_ms,
                                              uint32_t life_ms) {
    __shared__ WaveSmem<> S;
    const uint32_t lane = lane_id(), slot = blockIdx.x;
    ServeBlock* blk = blk0 + slot;
    DevStats* scratch = scratch0 + (size_t)slot * (kStatSlots + 1);
    uint32_t* list2 = list20 + 4 * slot;
    uint32_t* count2 = reinterpret_cast<uint32_t*>(scratch + kStatSlots);
    if (lane == 0) __hip_atomic_store(&blk->alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t last = sys_load64(&blk->done_seq);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t_req = t0;
    for (;;) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - t_req > (uint64_t)idle_ms * 100000u) {  // this slot idle: any other slot's request?
            const uint64_t ta = __hip_atomic_load(t_any, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            t_req = ta > t_req ? ta : t_req;
        }
        if (sys_load32(&blk0->stop) || now - t_req > (uint64_t)idle_ms * 100000u ||
            now - t0 > (uint64_t)life_ms * 100000u)
            break;
        const uint64_t r = sys_load64(&blk->req_seq);
        const uint64_t seq = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)r) |
                             ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32);
        if (seq == last) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        // the request's fields were stored before req_seq (host release): the wave reads the
        // block's request half in ONE round trip, a system-scope 8-byte load per lane (64 x 8 B
        // covers the header and the query), and keeps it in LDS (S.q holds the query for the
        // search; the header words go through readlane)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        static_assert(offsetof(ServeBlock, q) + kServeMaxQuery <= 64 * 8, "the request half fits one load per lane");
        const uint64_t* req = reinterpret_cast<const uint64_t*>(blk);
        const uint64_t wv = sys_load64(req + lane);
        auto hdr32 = [&](uint32_t byte_off) -> uint32_t {  // 4-byte header field at byte_off (< 512)
            const uint64_t w = (uint64_t)__builtin_amdgcn_readlane((uint32_t)wv, byte_off >> 3) |
                               ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(wv >> 32), byte_off >> 3) << 32);
            return (uint32_t)(w >> (8 * (byte_off & 7)));
        };
        SearchParams P = P0;
        P.thr = __uint_as_float(hdr32(offsetof(ServeBlock, thr)));
        P.limit = hdr32(offsetof(ServeBlock, limit));
        P.out_stride = P.limit;
#pragma unroll
        for (int i = 0; i < 8; ++i) P.valid[i] = hdr32(offsetof(ServeBlock, valid) + 4 * i);
        const uint32_t m = hdr32(offsetof(ServeBlock, m));
        {  // the query's bytes to S.q (one code point per entry), lanes over the 8-byte words
            constexpr uint32_t q0 = offsetof(ServeBlock, q);
            uint8_t* raw = reinterpret_cast<uint8_t*>(S.surv_t);  // scratch: free until the search starts
            reinterpret_cast<uint64_t*>(raw)[lane] = wv;
            wave_sync();
            const uint32_t mq = m == kQueryWildcard ? 0u : min(m, kServeMaxQuery);
            for (uint32_t i = lane; i < mq; i += 64) S.q[i] = raw[q0 + i];
            wave_sync();
        }
        if (lane == 0) __hip_atomic_store(count2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wave_sync();
        wave_query(S, 0u, X, P, blk->q, blk->off, &blk->m, &blk->n, blk->keys, blk->scores, list2, count2,
                             scratch, nullptr, nullptr, 0u, 1u, m);
        const uint32_t routed = __hip_atomic_load(count2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) {
            __hip_atomic_store(&blk->status, routed ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every result store before the number
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&blk->done_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = seq;
        t_req = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) atomicMax(t_any, (unsigned long long)t_req);  // (vector atomic: keeps the others up)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&blk->alive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Tier 1a: the lean wave kernel, survivors spilled to HBM for k_emit. The main launch
// (HEAVY false) takes one query per workgroup; HEAVY: the heavy list's launch, (query, term-id
// slice) items of the list (LOOPED: the overflow launch, grid-stride), and with ONES also its
// cmin-1 queries (part_ones). Each launch compiles its own part loop (with both loops in one
// kernel the main launch carried 76 B of scratch spills and 434 lane reloads; the same speed,
// profiles/r03_s5_ab_lean_one_copy.txt)
template <bool HEAVY, bool ONES = false, bool LOOPED = false>
__global__ __launch_bounds__(64, HEAVY ? kHeavyLeanWavesPerSimd : kLeanWavesPerSimd) void k_wave_lean(DevIndex X, SearchParams P,
                                                                    const uint8_t* __restrict__ qnorm,
                                                                    const uint64_t* __restrict__ qoff,
                                                                    const uint32_t* __restrict__ qm,
                                                                    uint32_t* __restrict__ out_n,
                                                                    uint32_t* __restrict__ out_k,
                                                                    float* __restrict__ out_s,
                                                                    uint32_t* __restrict__ list2,
                                                                    uint32_t* __restrict__ count2,
                                                                    DevStats* __restrict__ stats,
                                                                    uint32_t* __restrict__ fb, uint32_t* __restrict__ fbc,
                                                                    const uint32_t* __restrict__ qlist,
                                                                    const uint32_t* __restrict__ qcount) {
    __shared__ WaveSmem<true> S;
    // lane-group staging (lean_query_g) for the main launch; the heavy list's launch keeps the packed
    // staging (lean_query): its threshold-0 queries' part_ones parts are ~3 chunks per list, where a
    // per-list cap splits most parts
    if constexpr (!HEAVY) {
        lean_query_g(S, blockIdx.x, X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, stats, fb, fbc);
    } else {
        const uint32_t cnt = *qcount;
        // (query, term-id slice) items, one per workgroup (heavy_grid sizes the launch for every
        // item; the rest exit), a query's slices on neighbouring workgroups: enough slices that a
        // short list fills the GPU and no query's wave outlasts the rest by much. No item loop: in one
        // the compiler hoists the arguments' loads out of it and the part loop spills (14-18 VGPRs,
        // whose reloads waited for the next part's loads in the counting: an all-heavy batch of 8,192
        // 8-character queries 0.98 -> 0.75 ms per call). (Lane-group staging here measured slower
        // on C2: 32.0-32.8 against 37.1-37.3 Mq/s, profiles/r05_s12_ab_heavy_staging.txt.)
        // (LOOPED: the overflow launch, items past the first launch's grid, grid-stride; it spills,
        // and runs only when a call has more items than its context's last call)
        const uint32_t nsl = heavy_slices(P, cnt, X);
        if constexpr (LOOPED) {
            for (uint32_t i = P.hbase + blockIdx.x; i < cnt * nsl; i += gridDim.x) {
                const uint32_t k = i / nsl;
                lean_query<ONES>(S, qlist[k], X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, stats, fb, fbc,
                                 i - k * nsl, nsl);
                wave_sync();
            }
        } else {
            const uint32_t i = P.hbase + blockIdx.x;
            if (i >= cnt * nsl) return;
            const uint32_t k = i / nsl;
            lean_query<ONES>(S, qlist[k], X, P, qnorm, qoff, qm, out_n, out_k, out_s, list2, count2, stats, fb, fbc,
                             i - k * nsl, nsl);
        }
    }
}

// Tier 1a's calcScore (nGramSearch.hpp:310-341) and top-L (hpp:397-401), one wave per query
// over the survivor list k_wave_lean left in HBM (DEFER), for every query or the heavy list: the
// fused path's wave_emit (reading the survivors from HBM) and wave_flush, in 2.3 KB of LDS.
struct EmitSmem {
    uint64_t cand_own[kWaveCand];
    __device__ __forceinline__ uint64_t* cand() { return cand_own; }
    uint32_t q[kWaveMaxGrams + 8];
    uint32_t kset[2 * kWaveMaxLimit];  // emit_rank_prefix: the keys of the multi-hit top-L
    uint32_t rstage[8 * 64];            // ... and the ranks of the lists in flight (kRankLoads)
};

// The one-hit records of a threshold-0 query's top-L (DevIndex.rank_post; tier 1a counted the query
// at cmin 2 and its multi-hit records are in the buffer). With one weight, one pair per term and one
// term per key, every one-hit term's record is (enc1 = the score of 1 hit of n, its key rank), and a
// multi-hit record is never worse than that score. A one-hit term in the top-L has all the terms
// before it in its list (smaller key ranks: each a one-hit record that ties and wins on the rank, or a
// multi-hit one at least as good) in the top-L too, so it is among its list's first L entries. Those
// are merged into the buffer (calcScore's records, nGramSearch.hpp:318-336), each list until its
// records pass tau (ascending ranks: the rest are worse). An entry whose term is multi-hit is a
// duplicate of its real record: dropped when that record is among the multi-hit top-L (kset), and
// worse than tau otherwise.
constexpr int kRankLoads = 8;  // lists whose next 64 ranks are in flight at once

// loads of offsets o .. o + 63 of up to kRankLoads lists of `todo` (lowest first, removed from it);
// returns the lists taken
__device__ __forceinline__ unsigned long long rank_issue(const DevIndex& X, uint64_t gbase, uint32_t glen,
                                                         unsigned long long& todo, uint32_t o,
                                                         uint32_t (&r)[kRankLoads]) {
    const uint32_t lane = lane_id();
    unsigned long long taken = 0;
#pragma unroll
    for (int u = 0; u < kRankLoads; ++u) {
        r[u] = 0;
        if (todo) {
            const uint32_t j = (uint32_t)__ffsll((long long)todo) - 1u;
            todo &= todo - 1;
            taken |= 1ull << j;
            const uint32_t len = __builtin_amdgcn_readlane(glen, (int)j);
            const uint64_t b = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(gbase >> 32), (int)j) << 32) |
                               __builtin_amdgcn_readlane((uint32_t)gbase, (int)j);
            if (o + lane < len) r[u] = X.rank_post[b + o + lane];
        }
    }
    return taken;
}

template <bool RADIX>
__device__ __forceinline__ void emit_rank_prefix(EmitSmem& S, const DevIndex& X, uint32_t L, uint32_t enc1,
                                                 uint64_t gbase, uint32_t glen, uint32_t& cand_n, uint64_t& tau) {
    const uint32_t lane = lane_id();
    if (cand_n > L) wave_trim<RADIX>(S, cand_n, tau, L, true);  // the multi-hit top-L, unsorted
    constexpr uint32_t kSet = 2 * kWaveMaxLimit, kEmpty = 0xFFFFFFFFu;
    static_assert(kSet == 256, "8-bit set slots");
    static_assert(sizeof(S.rstage) == sizeof(uint32_t) * 64 * kRankLoads, "staging for kRankLoads lists");
    auto slot = [](uint32_t k) -> uint32_t { return (k * 0x9E3779B1u) >> (32 - 8); };
    auto insert = [&](uint32_t k) {
        for (uint32_t h = slot(k);; h = (h + 1) & (kSet - 1))
            if (atomicCAS(&S.kset[h], kEmpty, k) == kEmpty) break;
    };
    for (uint32_t i = lane; i < kSet; i += 64) S.kset[i] = kEmpty;
    wave_sync();
    if (lane < cand_n) insert((uint32_t)S.cand()[lane]);
    if (lane + 64 < cand_n) insert((uint32_t)S.cand()[lane + 64]);
    wave_sync();
    const uint64_t hi = (uint64_t)(~enc1) << 32;
    unsigned long long alive = __ballot(glen != 0);
    for (uint32_t o = 0; o < L && alive; o += 64) {
        unsigned long long todo = alive & __ballot(glen > o);
        while (todo) {
            // offsets o .. o + 63 of up to kRankLoads lists in flight at once, staged in LDS (no
            // registers live across the buffer trims below)
            unsigned long long taken;
            {
                uint32_t r[kRankLoads];
                taken = rank_issue(X, gbase, glen, todo, o, r);
#pragma unroll
                for (int u = 0; u < kRankLoads; ++u) S.rstage[64 * u + lane] = r[u];
                wave_sync();
            }
#pragma unroll 1
            for (uint32_t u = 0; taken; ++u) {
                const uint32_t j = (uint32_t)__ffsll((long long)taken) - 1u;
                taken &= taken - 1;
                const uint32_t len = __builtin_amdgcn_readlane(glen, (int)j);
                const uint64_t rec = o + lane < len ? hi | S.rstage[64 * u + lane] : kNoCand;
                if (!__ballot(rec < tau)) {  // ascending: the rest of the list is worse too
                    alive &= ~(1ull << j);
                    continue;
                }
                bool want = rec < tau;
                if (want) {
                    const uint32_t k = (uint32_t)rec;
                    for (uint32_t h = slot(k);; h = (h + 1) & (kSet - 1)) {
                        const uint32_t v = S.kset[h];
                        if (v == k) { want = false; break; }
                        if (v == kEmpty) break;
                    }
                }
                if (cand_n + 64 > (uint32_t)kWaveCand) wave_trim<RADIX>(S, cand_n, tau, L, true);
                want = want && rec < tau;
                const unsigned long long bw = __ballot(want);
                if (want) S.cand()[cand_n + rank_below(bw)] = rec;
                cand_n += __popcll(bw);
            }
            wave_sync();  // the staging is read before the next lists' ranks overwrite it
        }
    }
}

// one wave per workgroup: four-wave workgroups wait for four free slots on one CU beside tier 1a
// (the heavy list's k_emit measured 1.8 ms against 0.32 ms)
constexpr uint32_t kEmitWaves = 1;

template <bool RADIX, int D = 1>
__device__ __forceinline__ void emit_query(EmitSmem& S, const uint32_t q, const bool heavy_launch, const DevIndex& X,
                                           const SearchParams& P, const uint8_t* __restrict__ qnorm,
                                           const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qm,
                                           uint32_t* __restrict__ out_n, uint32_t* __restrict__ out_k,
                                           float* __restrict__ out_s, DevStats* __restrict__ stats) {
    const uint32_t lane = lane_id();
    const uint32_t* et = P.est + (size_t)q * P.ecap;
    const uint8_t* ec = P.esc + (size_t)q * P.ecap;
    // the first 64 survivors and the query's length load beside the count (the slots always
    // exist): one round trip for all of them
    uint32_t t = et[lane], code = ec[lane];
    uint32_t sn = P.esn[q];
    const uint32_t m = qm[q];
    // rank lists: the query's lists as tier 1a left them (emit_rank_prefix), in the same round trip
    uint64_t gbase = 0;
    uint32_t glen = 0;
    if (RADIX && X.rank_post) {
        const uint32_t* ri = et + (P.ecap - kRankInfo);
        gbase = ((uint64_t)ri[64 + lane] << 32) | ri[lane];
        glen = ri[128 + lane];
    }
    if (sn == kNoEmit) return;  // tier 1a did not finish this query
    // the main launch leaves the heavy launch's queries to the heavy list's k_emit
    if (!heavy_launch && (sn & kEmitHeavy)) return;
    sn &= ~kEmitHeavy;
    const uint32_t n = m - X.gsz + 1, L = P.limit;
    const float sc_long = lane <= n ? (float)lane / (float)n : 0.0f;  // as wave_query
    const float sc_short = lane <= m ? (float)lane / (float)m : 0.0f;
    // survivors past the query's slots are in the batch's arena (lean_query_g's spill_arena): the
    // slots end where tier 1a's did (the rank-list tail is not theirs)
    const uint32_t ecap_q = P.ecap - (X.rank_post && !(__shfl(sc_long, 1) < P.thr) ? kRankInfo : 0u);
    const uint32_t sn_all = sn;
    sn = min(sn, ecap_q);
    uint32_t cand_n = 0;
    uint64_t tau = kNoCand;
    // the query's characters only for an exact-match test (a survivor scoring > 0.999), rare
    bool have_q = false;
    // threshold 0 with rank lists (emit_rank_prefix; cmin-1 queries are on the heavy list, whose
    // launch is the RADIX one)
    const bool rank_mode = RADIX && X.rank_post && !(__shfl(sc_long, 1) < P.thr);
    // one pair per term (DevIndex.tk_identity): a software pipeline over the batches of 64: while
    // batch b is scored, the pairs of batches b + 1 .. b + D and the survivors of batches up to
    // b + 2D + 1 are in flight (a threshold-0 query has thousands of survivors, and a batch is
    // otherwise two dependent round trips). D = 1 in both launches (2 and 4 for the heavy launch's
    // long queries measured within noise on C2)
    uint32_t base0 = 0;
    if (X.tk_identity && sn > 64) {
        uint32_t T[2 * D + 1], Cc[2 * D + 1];  // survivors of batches b .. b + 2D
        uint2 K[D];                            // pairs of batches b .. b + D - 1
        T[0] = t;
        Cc[0] = code;
#pragma unroll
        for (int j = 1; j <= 2 * D; ++j) {
            T[j] = 0;
            Cc[j] = 0;
            if (64u * j + lane < sn) {
                T[j] = et[64u * j + lane];
                Cc[j] = ec[64u * j + lane];
            }
        }
#pragma unroll
        for (int j = 0; j < D; ++j) K[j] = X.tk[64u * j + lane < sn ? T[j] : 0u];
        for (uint32_t base = 0; base < sn; base += 64) {
            const uint32_t i = base + lane;
            uint32_t tn = 0, cn = 0;
            if (i + 64u * (2 * D + 1) < sn) {
                tn = et[i + 64u * (2 * D + 1)];
                cn = ec[i + 64u * (2 * D + 1)];
            }
            const uint2 kn = X.tk[i + 64u * D < sn ? T[D] : 0u];
            const uint32_t c0 = Cc[0];
            const float s_l = __shfl(sc_long, (int)(c0 & 63u)), s_s = __shfl(sc_short, (int)(c0 & 63u));
            const float s = (c0 & 0x80u) ? s_s : s_l;
            const bool promo = (double)s > 0.999;  // nGramSearch.hpp:328
            if (!have_q && __ballot(i < sn && promo)) {
                const uint8_t* qg = qnorm + qoff[q];
                for (uint32_t k = lane; k < m; k += 64) S.q[k] = char_at(qg, k, X.csize);
                wave_sync();
                have_q = true;
            }
            uint32_t p = 0, pe = 0;
            if (i < sn) term_pairs(X, T[0], s, promo, tau, p, pe);  // p == T[0] unless pruned
            uint64_t rec = kNoCand;
            // (tier 1a leaves long survivors only: it hands every short-search query over)
            if (p < pe) rec = ((uint64_t)(~pair_enc(K[0], s, promo, false, X, S.q, 4u, m, P.valid)) << 32) | K[0].x;
            if (cand_n + 64 > (uint32_t)kWaveCand) wave_trim<RADIX>(S, cand_n, tau, L, X.keys_unique != 0);
            const bool want = rec < tau;
            const unsigned long long bw = __ballot(want);
            if (want) S.cand()[cand_n + rank_below(bw)] = rec;
            cand_n += __popcll(bw);
#pragma unroll
            for (int j = 0; j < 2 * D; ++j) {
                T[j] = T[j + 1];
                Cc[j] = Cc[j + 1];
            }
            T[2 * D] = tn;
            Cc[2 * D] = cn;
#pragma unroll
            for (int j = 0; j + 1 < D; ++j) K[j] = K[j + 1];
            K[D - 1] = kn;
        }
        base0 = sn;
    }
    // wave_emit over the survivors in HBM
    for (uint32_t base = base0; base < sn; base += 64) {
        const uint32_t i = base + lane;
        // the next 64 survivors load while this batch's pairs do (one round trip per batch)
        uint32_t t_next = 0, code_next = 0;
        if (base + 64 < sn && i + 64 < sn) {
            t_next = et[i + 64];
            code_next = ec[i + 64];
        }
        uint32_t p = 0, pe = 0;
        const float s_l = __shfl(sc_long, (int)(code & 63u)), s_s = __shfl(sc_short, (int)(code & 63u));
        const float s = (code & 0x80u) ? s_s : s_l;
        const bool promo = (double)s > 0.999;  // nGramSearch.hpp:328
        if (!have_q && __ballot(i < sn && promo)) {
            const uint8_t* qg = qnorm + qoff[q];
            for (uint32_t k = lane; k < m; k += 64) S.q[k] = char_at(qg, k, X.csize);
            wave_sync();
            have_q = true;
        }
        if (i < sn) term_pairs(X, t, s, promo, tau, p, pe);
        while (__ballot(p < pe)) {
            uint64_t rec = kNoCand;
            if (p < pe) {
                const uint2 kw = X.tk[p++];
                const uint32_t enc = pair_enc(kw, s, promo, false, X, S.q, 4u, m, P.valid);
                rec = ((uint64_t)(~enc) << 32) | kw.x;
            }
            if (cand_n + 64 > (uint32_t)kWaveCand) wave_trim<RADIX>(S, cand_n, tau, L, X.keys_unique != 0);
            const bool want = rec < tau;
            const unsigned long long bw = __ballot(want);
            if (want) S.cand()[cand_n + rank_below(bw)] = rec;
            cand_n += __popcll(bw);
        }
        t = t_next;
        code = code_next;
    }
    // survivors past the slots (rare: a query that outgrew them): its arena blocks in order, 64 at a
    // time, without prefetch (lane 0 walks the chain first: a few dependent loads; the block list goes
    // to rstage, free until emit_rank_prefix)
    if (sn_all > sn) {
        const uint32_t na = sn_all - sn;
        if (lane == 0) {
            uint32_t bnx = P.eovf[q];
            for (uint32_t k = 0; k * kArenaBlock < na && k < kArenaChain && bnx; ++k) {
                S.rstage[k] = bnx - 1u;
                bnx = P.anext[bnx - 1u];
            }
        }
        wave_sync();
        for (uint32_t a = 0; a < na; a += 64) {
            const uint32_t k = a / kArenaBlock, i = a + lane;
            const size_t off = (size_t)__builtin_amdgcn_readfirstlane(S.rstage[k]) * kArenaBlock + (a - k * kArenaBlock);
            const bool live = i < na;
            const uint32_t ta = live ? P.at[off + lane] : 0u, ca = live ? (uint32_t)P.ac[off + lane] : 0u;
            uint32_t p = 0, pe = 0;
            const float s_l = __shfl(sc_long, (int)(ca & 63u)), s_s = __shfl(sc_short, (int)(ca & 63u));
            const float s = (ca & 0x80u) ? s_s : s_l;
            const bool promo = (double)s > 0.999;  // nGramSearch.hpp:328
            if (!have_q && __ballot(live && promo)) {
                const uint8_t* qg = qnorm + qoff[q];
                for (uint32_t c = lane; c < m; c += 64) S.q[c] = char_at(qg, c, X.csize);
                wave_sync();
                have_q = true;
            }
            if (live) term_pairs(X, ta, s, promo, tau, p, pe);
            while (__ballot(p < pe)) {
                uint64_t rec = kNoCand;
                if (p < pe) {
                    const uint2 kw = X.tk[p++];
                    const uint32_t enc = pair_enc(kw, s, promo, false, X, S.q, 4u, m, P.valid);
                    rec = ((uint64_t)(~enc) << 32) | kw.x;
                }
                if (cand_n + 64 > (uint32_t)kWaveCand) wave_trim<RADIX>(S, cand_n, tau, L, X.keys_unique != 0);
                const bool want = rec < tau;
                const unsigned long long bw = __ballot(want);
                if (want) S.cand()[cand_n + rank_below(bw)] = rec;
                cand_n += __popcll(bw);
            }
        }
    }
    // threshold 0 with rank lists: tier 1a counted this query at cmin 2 (its multi-hit terms, above);
    // its one-hit records come from the first L key ranks of each of its lists
    if (rank_mode) {
        const float sc1 = __uint_as_float(X.w_uniform) * __shfl(sc_long, 1);  // pair_enc of one hit
        emit_rank_prefix<RADIX>(S, X, L, sc1 > 0.0f ? __float_as_uint(sc1) + 1u : 1u, gbase, glen, cand_n, tau);
    }
    wave_flush<RADIX>(S, cand_n, tau, L, X.keys_unique != 0);
    const size_t ob = (size_t)q * P.out_stride;
    for (uint32_t i = lane; i < cand_n; i += 64) {
        const uint64_t r = S.cand()[i];
        const uint32_t enc = ~(uint32_t)(r >> 32);
        out_k[ob + i] = (uint32_t)r;
        out_s[ob + i] = __uint_as_float(enc - 1u);
    }
    if (lane == 0) {
        out_n[q] = cand_n;
        if (!(P.dbg & 32u)) atomicAdd(&stats[q & (kStatSlots - 1)].results, (unsigned long long)cand_n);
    }
}

// every query (qlist == nullptr), or the heavy list grid-stride (RADIX: the heavy list's launch,
// whose thousands of survivors per query refill the top-L buffer many times)
template <bool RADIX>
__global__ __launch_bounds__(64 * kEmitWaves) void k_emit(DevIndex X, SearchParams P, const uint8_t* __restrict__ qnorm,
                                                          const uint64_t* __restrict__ qoff,
                                                          const uint32_t* __restrict__ qm, uint32_t* __restrict__ out_n,
                                                          uint32_t* __restrict__ out_k, float* __restrict__ out_s,
                                                          DevStats* __restrict__ stats,
                                                          const uint32_t* __restrict__ qlist,
                                                          const uint32_t* __restrict__ qcount) {
    __shared__ EmitSmem SS[kEmitWaves];
    EmitSmem& S = SS[threadIdx.x >> 6];
    const uint32_t j0 = blockIdx.x * kEmitWaves + (threadIdx.x >> 6);
    if (!qlist) {
        if (j0 < P.n_queries) emit_query<RADIX>(S, j0, false, X, P, qnorm, qoff, qm, out_n, out_k, out_s, stats);
        return;
    }
    const uint32_t cnt = *qcount;
    for (uint32_t j = j0; j < cnt; j += gridDim.x * kEmitWaves) {
        emit_query<RADIX>(S, qlist[j], true, X, P, qnorm, qoff, qm, out_n, out_k, out_s,
                                                      stats);
        wave_sync();
    }
}

// Joins the slices of sliced tier 1b (SearchParams.prec / pcnt): per query of the list, the
// slices' top-L records through the running top-L (key-max dedup, tau pruning), then results.
__global__ __launch_bounds__(64) void k_merge(DevIndex X, SearchParams P, const uint32_t* __restrict__ qlist,
                                              const uint32_t* __restrict__ qcount, uint32_t* __restrict__ out_n,
                                              uint32_t* __restrict__ out_k, float* __restrict__ out_s,
                                              DevStats* __restrict__ stats) {
    __shared__ EmitSmem S;
    const uint32_t lane = lane_id(), nsl = P.nslices, L = P.limit;
    const uint32_t cnt = qlist ? *qcount : P.n_queries;  // no list: every query of the batch
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        const uint32_t q = qlist ? qlist[i] : i;
        const uint32_t* pc = P.pcnt + (size_t)q * nsl;
        if (pc[0] == kNoPart) continue;  // answered by slice 0 directly
        uint32_t cand_n = 0;
        uint64_t tau = kNoCand;
        for (uint32_t j = 0; j < nsl; ++j) {
            const uint32_t nj = pc[j];
            const uint64_t* pr = P.prec + ((size_t)q * nsl + j) * L;
            for (uint32_t b = 0; b < nj; b += 64) {
                const uint64_t rec = b + lane < nj ? pr[b + lane] : kNoCand;
                if (cand_n + 64 > (uint32_t)kWaveCand) wave_trim<true>(S, cand_n, tau, L, X.keys_unique != 0);
                const bool want = rec < tau;
                const unsigned long long bw = __ballot(want);
                if (want) S.cand()[cand_n + rank_below(bw)] = rec;
                cand_n += __popcll(bw);
            }
        }
        wave_flush<true>(S, cand_n, tau, L, X.keys_unique != 0);
        const size_t ob = (size_t)q * P.out_stride;
        for (uint32_t k = lane; k < cand_n; k += 64) {
            const uint64_t r = S.cand()[k];
            const uint32_t enc = ~(uint32_t)(r >> 32);
            out_k[ob + k] = (uint32_t)r;
            out_s[ob + k] = __uint_as_float(enc - 1u);
        }
        if (lane == 0) {
            out_n[q] = cand_n;
            if (!(P.dbg & 32u)) atomicAdd(&stats[q & (kStatSlots - 1)].results, (unsigned long long)cand_n);
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------- general path -------
__device__ __forceinline__ void emit_global(const DevIndex& X, uint32_t t, float s, bool shortg, const uint8_t* q,
                                            uint32_t m, const SearchParams& P, uint32_t* kenc) {
    const bool promo = (double)s > 0.999;
    for (uint32_t p = X.tk_off[t]; p < X.tk_off[t + 1]; ++p) {
        const uint2 kw = X.tk[p];
        const uint32_t enc = pair_enc(kw, s, promo, shortg, X, q, X.csize, m, P.valid);
        if (enc) atomicMax(&kenc[kw.x], enc);
    }
}

__global__ __launch_bounds__(256) void k_gen_long(DevIndex X, SearchParams P, const uint8_t* __restrict__ qnorm,
                                                  const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qm,
                                                  const uint32_t* __restrict__ group, uint32_t* __restrict__ cnt,
                                                  uint32_t* __restrict__ kenc, int phase) {
    const uint32_t gi = blockIdx.y, q = group[gi], m = qm[q];
    if (m == kQueryWildcard || m < X.gsz) return;  // nGramSearch.hpp:281
    const uint32_t n = m - X.gsz + 1, n_long = X.n_terms - X.n_short;
    const uint8_t* qs = qnorm + qoff[q];
    uint32_t* C = cnt + (size_t)gi * n_long;
    uint32_t* K = kenc + (size_t)gi * gen_kstride(X.n_keys);
    const uint64_t me = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    const float fn = (float)n;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t g = gram_at(X, [&](uint32_t j) { return char_at(qs, j, X.csize); }, i);
        if (g == UINT32_MAX) continue;
        const uint64_t a = X.gram_off[g], b = X.gram_off[g + 1];
        for (uint64_t p = a + me; p < b; p += stride) {
            const uint32_t t = X.post[p];
            if (phase == 0) {
                atomicAdd(&C[t], 1u);
            } else {
                const uint32_t c = atomicExch(&C[t], 0u);  // first visitor owns the term
                if (c) {
                    const float s = (float)c / fn;
                    if (!(s < P.thr)) emit_global(X, X.n_short + t, s, false, qs, m, P, K);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_gen_short(DevIndex X, SearchParams P, const uint8_t* __restrict__ qnorm,
                                                   const uint64_t* __restrict__ qoff, const uint32_t* __restrict__ qm,
                                                   const uint32_t* __restrict__ group, uint32_t* __restrict__ kenc) {
    const uint32_t gi = blockIdx.y, q = group[gi], m = qm[q];
    if (m == kQueryWildcard || m == 0 || m >= X.short_query_len) return;
    const uint32_t end = m <= X.full_scan_len ? X.n_terms : X.n_short;  // nGramSearch.hpp:247
    const uint8_t* qs = qnorm + qoff[q];
    uint32_t qc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) qc[i] = (uint32_t)i < m ? char_at(qs, i, X.csize) : 0;
    __shared__ uint8_t peq[256];
    build_peq(peq, [&](uint32_t i) { return char_at(qs, i, X.csize); }, m, threadIdx.x, blockDim.x);
    __syncthreads();
    uint32_t* K = kenc + (size_t)gi * gen_kstride(X.n_keys);
    const float fm = (float)m;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < end; t += gridDim.x * blockDim.x) {
        const float s = (float)string_match(peq, qc, m, X, t) / fm;
        if (!(s < P.thr)) emit_global(X, t, s, true, qs, m, P, K);
    }
}

__global__ __launch_bounds__(256) void k_gen_compact(uint32_t n_keys, uint32_t* __restrict__ kenc,
                                                     uint64_t* __restrict__ list, uint32_t* __restrict__ lcount) {
    const uint32_t gi = blockIdx.y;
    uint32_t* K = kenc + (size_t)gi * gen_kstride(n_keys);
    uint64_t* Lst = list + (size_t)gi * n_keys;
    // (one counter per query: a wave appends its records with one atomic; a full-library scan
    // leaves most keys set, and per-lane atomics on G counters took ~2 ms per group)
    const uint32_t n_it = (n_keys + gridDim.x * blockDim.x - 1) / (gridDim.x * blockDim.x);
    for (uint32_t it = 0, k = blockIdx.x * blockDim.x + threadIdx.x; it < n_it; ++it, k += gridDim.x * blockDim.x) {
        const uint32_t e = k < n_keys ? K[k] : 0u;
        const unsigned long long b = __ballot(e != 0);
        if (!b) continue;
        uint32_t base = 0;
        if (lane_id() == (uint32_t)(__ffsll((long long)b) - 1)) base = atomicAdd(&lcount[gi], (uint32_t)__popcll(b));
        base = __shfl(base, __ffsll((long long)b) - 1);
        if (e) {
            K[k] = 0;
            Lst[base + rank_below(b)] = ((uint64_t)(~e) << 32) | k;
        }
    }
}

__global__ __launch_bounds__(256) void k_gen_write(const uint64_t* __restrict__ sorted, uint32_t n, uint32_t q,
                                                   SearchParams P, uint32_t* __restrict__ out_n,
                                                   uint32_t* __restrict__ out_k, float* __restrict__ out_s) {
    const uint32_t cnt = min(n, P.limit);
    const size_t ob = (size_t)q * P.out_stride;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
        const uint64_t r = sorted[i];
        const uint32_t enc = ~(uint32_t)(r >> 32);
        out_k[ob + i] = (uint32_t)r;
        out_s[ob + i] = __uint_as_float(enc - 1u);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out_n[q] = cnt;
}

// The general path's top-L for limits up to kGenSelCap, one workgroup per query of the group, in
// place of a compaction, a device-wide radix sort per query and k_gen_write (~60 us a query: a
// full-library scan of an m <= 3 query scores most keys). Order as there: score encoding
// descending, key id ascending (hpp:397-401 with the canonical tie order).
// A radix select over the row's encodings (11 + 11 + 10 bits) finds the L-th largest one, T;
// a last pass in key order takes every key above T and the first keys at T, and clears the row;
// the <= L records are sorted in LDS. A thread reads four keys a load (rows are gen_kstride
// apart) with the next load in flight: the passes are latency-bound at one load per round.
__global__ __launch_bounds__(kGenSelThreads) void k_gen_select(uint32_t n_keys, uint32_t* __restrict__ kenc,
                                                              const uint32_t* __restrict__ group, SearchParams P,
                                                              uint32_t* __restrict__ out_n,
                                                              uint32_t* __restrict__ out_k, float* __restrict__ out_s) {
    constexpr uint32_t kBins = 2048, kWaves = kGenSelThreads / 64;
    __shared__ uint32_t hist[kBins];
    __shared__ uint64_t rec[kGenSelCap];
    __shared__ uint32_t wcnt[kWaves];
    __shared__ uint32_t s_pick[3];  // bin, count above it, records taken
    const uint32_t tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
    const uint32_t gi = blockIdx.x, q = group[gi];
    const uint32_t n4 = gen_kstride(n_keys) / 4;
    uint4* K4 = reinterpret_cast<uint4*>(kenc + (size_t)gi * gen_kstride(n_keys));
    const uint32_t L = min(P.limit, kGenSelCap);
    const uint32_t n_it = (n4 + kGenSelThreads - 1) / kGenSelThreads;
    auto ld = [&](uint32_t it) {
        const uint32_t i = it * kGenSelThreads + tid;
        return i < n4 ? K4[i] : make_uint4(0, 0, 0, 0);
    };
    uint32_t prefix = 0, mask = 0, need = L;  // need: rank of T among the keys matching prefix
    bool all = false;                          // fewer than L keys scored: take every one
    for (int pass = 0; pass < 3 && L; ++pass) {
        const uint32_t shift = pass == 0 ? 21u : pass == 1 ? 10u : 0u;
        const uint32_t bmask = pass == 2 ? 0x3FFu : 0x7FFu;
        for (uint32_t i = tid; i < kBins; i += kGenSelThreads) hist[i] = 0;
        __syncthreads();
        uint4 nx = ld(0);
        for (uint32_t it = 0; it < n_it; ++it) {
            const uint4 v = nx;
            if (it + 1 < n_it) nx = ld(it + 1);
            const uint32_t ev[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t e = ev[j];
                const bool in = e != 0 && (e & mask) == prefix;
                const uint32_t bin = (e >> shift) & bmask;
                // equal scores are the rule (m <= 3: a handful of distinct scores): a wave whose
                // counted keys share one bin adds them with one LDS atomic
                const unsigned long long b = __ballot(in);
                if (!b) continue;
                const uint32_t b0 = __shfl(bin, __ffsll((long long)b) - 1);
                if (__ballot(in && bin == b0) == b) {
                    if (lane == (uint32_t)(__ffsll((long long)b) - 1)) atomicAdd(&hist[b0], (uint32_t)__popcll(b));
                } else if (in) {
                    atomicAdd(&hist[bin], 1u);
                }
            }
        }
        __syncthreads();
        if (wid == 0) {  // the bin holding rank `need`, from the top: lane l owns bins kBins-32(l+1) .. kBins-1-32l
            constexpr uint32_t per = kBins / 64;
            uint32_t sum = 0;
            for (uint32_t j = 0; j < per; ++j) sum += hist[kBins - 1 - lane * per - j];
            uint32_t incl = sum;  // inclusive prefix over lanes (lane 0 = the top bins)
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(incl, d);
                if (lane >= d) incl += o;
            }
            const uint32_t total = __shfl(incl, 63);
            const uint32_t excl = incl - sum;
            if (pass == 0 && lane == 0 && total < need) s_pick[0] = 0xFFFFFFFFu;  // fewer than L keys
            if (!(pass == 0 && total < need) && excl < need && need <= incl) {
                uint32_t above = excl, bin = 0;
                for (uint32_t j = 0; j < per; ++j) {
                    const uint32_t bb = kBins - 1 - lane * per - j, c = hist[bb];
                    if (above + c >= need) { bin = bb; break; }
                    above += c;
                }
                s_pick[0] = bin;
                s_pick[1] = above;
            }
        }
        __syncthreads();
        if (s_pick[0] == 0xFFFFFFFFu) { all = true; break; }
        prefix |= s_pick[0] << shift;
        mask |= bmask << shift;
        need -= s_pick[1];
        __syncthreads();  // (s_pick is rewritten by the next pass)
    }
    // T: the L-th largest encoding; take every key above it and the first `need` at it, in key order
    const uint32_t T = all || !L ? 0u : prefix;
    if (tid == 0) s_pick[2] = 0;
    uint32_t eq_base = 0;
    __syncthreads();
    uint4 nx = ld(0);
    for (uint32_t it = 0; it < n_it; ++it) {
        const uint4 v = nx;
        if (it + 1 < n_it) nx = ld(it + 1);
        const uint32_t i4 = it * kGenSelThreads + tid;
        if (v.x | v.y | v.z | v.w) K4[i4] = make_uint4(0, 0, 0, 0);
        const uint32_t ev[4] = {v.x, v.y, v.z, v.w};
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) c += (!all && T != 0 && ev[j] == T) ? 1u : 0u;
        uint32_t incl = c;  // keys at T in this thread and the wave's lanes below it
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
        if (lane == 63) wcnt[wid] = incl;
        __syncthreads();
        uint32_t before = eq_base + incl - c, chunk = 0;
        for (uint32_t w = 0; w < kWaves; ++w) {
            const uint32_t cw = wcnt[w];
            before += w < wid ? cw : 0u;
            chunk += cw;
        }
        eq_base += chunk;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t e = ev[j];
            const bool gt = L && e != 0 && (all || e > T);
            const bool eq = !all && T != 0 && e == T;
            const bool take = gt || (eq && before < need);
            before += eq ? 1u : 0u;
            if (take) {
                const uint32_t at = atomicAdd(&s_pick[2], 1u);
                if (at < kGenSelCap) rec[at] = ((uint64_t)(~e) << 32) | (i4 * 4 + j);
            }
        }
        __syncthreads();  // (wcnt is rewritten by the next chunk)
    }
    const uint32_t n = min(s_pick[2], L);
    const uint32_t P2 = n <= 1 ? 1u : 1u << (32 - __clz(n - 1));
    for (uint32_t i = n + tid; i < P2; i += kGenSelThreads) rec[i] = ~0ull;
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= P2; k2 <<= 1) {
        for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
            for (uint32_t p = tid; p < P2 / 2; p += kGenSelThreads) {
                const uint32_t i = ((p & ~(j - 1u)) << 1) | (p & (j - 1u)), l = i + j;
                const uint64_t x = rec[i], y = rec[l];
                if ((x > y) == ((i & k2) == 0)) { rec[i] = y; rec[l] = x; }
            }
            __syncthreads();
        }
    }
    const size_t ob = (size_t)q * P.out_stride;
    for (uint32_t i = tid; i < n; i += kGenSelThreads) {
        const uint64_t r = rec[i];
        out_k[ob + i] = (uint32_t)r;
        out_s[ob + i] = __uint_as_float(~(uint32_t)(r >> 32) - 1u);
    }
    if (tid == 0) out_n[q] = n;
}

// DevIndex.kt_flag under one validChar set: key k (several pairs) can be promoted by a long term
// and has a short-search pair that the promotion then overwrites (pair_enc). The query that promotes
// k is k's own normalised text nk (escapeBlank + trim, hpp:330-334, upper case already: the query
// is upper-cased), so the flag is a property of the key: nk has at least g characters, no lower
// case, every g-gram of nk has a list (narrow: characters < 0x80) and some long term of k holds
// them all (searchLong counts n of n: s = 1, which passes every threshold that the short pair
// passed); and k has a short term, or nk is short enough (m <= g) for the full-library scan to
// score long terms too.
__global__ void k_key_flags(DevIndex X, ValidSet V, uint8_t* __restrict__ flags) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= X.n_keys) return;
    uint8_t f = 0;
    const uint32_t p0 = X.kt_off[k], p1 = X.kt_off[k + 1], g = X.gsz, cs = X.csize;
    if (p1 - p0 >= 2) {
        uint64_t a = X.key_off[k], e = X.key_off[k + 1] - 1;  // drop the NUL
        while (a < e && dev_space(esc_cs(V.w, char_at(X.key_bytes, a, cs), cs))) ++a;
        while (e > a && dev_space(esc_cs(V.w, char_at(X.key_bytes, e - 1, cs), cs))) --e;
        const uint64_t m = e - a;
        bool ok = m >= g;
        bool has_short = m <= X.full_scan_len;
        for (uint32_t p = p0; p < p1; ++p) has_short |= X.kt_term[p] < X.n_short;
        ok = ok && has_short;
        for (uint64_t i = 0; ok && i < m; ++i) {
            const uint32_t c = esc_cs(V.w, char_at(X.key_bytes, a + i, cs), cs);
            ok = !(c >= 'a' && c <= 'z') && (X.gram_mode ? c <= 0x1FFFFFu : c < 0x80u);
        }
        for (uint32_t p = p0; ok && !f && p < p1; ++p) {
            const uint32_t t = X.kt_term[p];
            if (t < X.n_short) continue;
            const uint64_t ta = X.term_off[t], tl = X.term_off[t + 1] - ta;
            bool all = true;
            for (uint64_t i = 0; all && i + g <= m; ++i) {
                bool hit = false;
                for (uint64_t j = 0; !hit && j + g <= tl; ++j) {
                    bool eq = true;
                    for (uint32_t c = 0; eq && c < g; ++c)
                        eq = char_at(X.term_bytes, ta + j + c, cs) == esc_cs(V.w, char_at(X.key_bytes, a + i + c, cs), cs);
                    hit = eq;
                }
                all = hit;
            }
            f = all ? 1 : 0;
        }
    }
    flags[k] = f;
}

__global__ void k_wild_records(const float* __restrict__ w, uint32_t n, uint64_t* __restrict__ rec) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t b = __float_as_uint(w[k]);
    const uint32_t ord = b ^ ((b >> 31) ? 0xFFFFFFFFu : 0x80000000u);  // ascending with the float
    rec[k] = ((uint64_t)(~ord) << 32) | k;                               // score desc, rank asc
}

__global__ void k_wild_split(const uint64_t* __restrict__ rec, const float* __restrict__ w, uint32_t n,
                             uint32_t* __restrict__ keys, float* __restrict__ scores) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = (uint32_t)rec[i];
    keys[i] = k;
    scores[i] = w[k];
}

__global__ void k_rank_fill(const uint32_t* __restrict__ post, const uint2* __restrict__ tk, uint32_t n_short,
                            uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = tk[n_short + post[i]].x;
}

}  // namespace

hipError_t build_rank_post(const uint64_t* gram_off, uint32_t n_seg, const uint32_t* post, uint64_t n_post,
                           const uint2* tk, uint32_t n_short, uint32_t n_keys, uint32_t* out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out + n_post, 0, 4 * sizeof(uint32_t), s);  // the 16-byte pad
    if (e != hipSuccess || !n_post) return e;
    if (n_post > kRankMaxPostings) return hipErrorNotSupported;  // hipcub's int item count
    uint32_t* a = nullptr;
    void* temp = nullptr;
    size_t bytes = 0;
    const int bits = n_keys > 1 ? 32 - __builtin_clz(n_keys - 1) : 1;
    e = hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, bytes, a, out, (int)n_post, (int)n_seg, gram_off,
                                                    gram_off + 1, 0, bits, s);
    if (e == hipSuccess) e = hipMalloc(&a, sizeof(uint32_t) * n_post);
    if (e == hipSuccess) e = hipMalloc(&temp, std::max<size_t>(bytes, 1));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_rank_fill, dim3((uint32_t)((n_post + 255) / 256)), dim3(256), 0, s, post, tk, n_short,
                           n_post, a);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipcub::DeviceSegmentedRadixSort::SortKeys(temp, bytes, a, out, (int)n_post, (int)n_seg, gram_off,
                                                        gram_off + 1, 0, bits, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(a);
    hipFree(temp);
    return e;
}

hipError_t build_key_flags(const DevIndex& X, const uint32_t valid[8], uint8_t* flags, hipStream_t s) {
    if (!X.n_keys) return hipSuccess;
    ValidSet V;
    for (int i = 0; i < 8; ++i) V.w[i] = valid[i];
    hipLaunchKernelGGL(k_key_flags, dim3((X.n_keys + 255) / 256), dim3(256), 0, s, X, V, flags);
    return hipGetLastError();
}

hipError_t build_wildcard(const float* d_w, uint32_t n_keys, uint32_t* d_keys, float* d_scores, hipStream_t s) {
    if (!n_keys) return hipSuccess;
    uint64_t *a = nullptr, *b = nullptr;
    void* temp = nullptr;
    size_t bytes = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, a, b, (int)n_keys, 0, 64, s);
    if (e == hipSuccess) e = hipMalloc(&a, sizeof(uint64_t) * n_keys);
    if (e == hipSuccess) e = hipMalloc(&b, sizeof(uint64_t) * n_keys);
    if (e == hipSuccess) e = hipMalloc(&temp, bytes);
    if (e == hipSuccess) {
        const uint32_t gx = (n_keys + 255) / 256;
        hipLaunchKernelGGL(k_wild_records, dim3(gx), dim3(256), 0, s, d_w, n_keys, a);
        e = hipcub::DeviceRadixSort::SortKeys(temp, bytes, a, b, (int)n_keys, 0, 64, s);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_wild_split, dim3(gx), dim3(256), 0, s, b, d_w, n_keys, d_keys, d_scores);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    hipFree(a);
    hipFree(b);
    hipFree(temp);
    return e;
}

int phase_stats(unsigned long long* out, int n, bool reset) {
#ifdef NGS_PHASE_STAMPS
    unsigned long long h[48];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < n && i < 48; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[48] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 48;
#else
    (void)out; (void)n; (void)reset;
    return -1;
#endif
}

// The heavy and full lists from k_prep's slot lists: per list, a scan of the 64 slot counts,
// then the slots' entries copied behind each other (slot order: the lists' order does not matter).
// One wave: it runs beside the main tier-1a launch, whose one-wave workgroups refill every wave slot
// as they free up, so a larger workgroup (four free slots on one CU at once) waited ~1.2 ms for
// room at C3 and held back the heavy list's launch behind it.
__global__ __launch_bounds__(64) void k_lists(const uint32_t* __restrict__ slots, uint32_t* __restrict__ ctr,
                                              uint32_t cap, uint32_t* __restrict__ heavy, uint32_t* __restrict__ hcount,
                                              uint32_t* __restrict__ full, uint32_t* __restrict__ fcount) {
    __shared__ uint32_t base[2 * (kListSlots + 1)];
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (uint32_t L = 0; L < 2; ++L) {  // 0: heavy slots, 1: full slots
        const uint32_t c = ctr[16 * (L * kListSlots + lane)];
        ctr[16 * (L * kListSlots + lane)] = 0;  // zero again for the context's next call (kPrepZero)
        const uint32_t incl = wave_incl_scan(c);
        base[L * (kListSlots + 1) + lane + 1] = incl;
        if (lane == 0) base[L * (kListSlots + 1)] = 0;
        if (lane == 63) *(L ? fcount : hcount) = incl;
    }
    __syncthreads();
    // eight slots' copies at once: their loads in flight together (slot by slot, each copy waited for
    // its load: 36 us for C2's 4,096 heavy queries, on the heavy chain's critical path)
    constexpr uint32_t kGroup = 8;
    static_assert((2 * kListSlots) % kGroup == 0, "slot groups");
    for (uint32_t s0 = 0; s0 < 2 * kListSlots; s0 += kGroup) {
        uint32_t b0[kGroup], n[kGroup], nmax = 0;
#pragma unroll
        for (uint32_t j = 0; j < kGroup; ++j) {
            const uint32_t sl = s0 + j, L = sl / kListSlots, k = sl % kListSlots;
            b0[j] = base[L * (kListSlots + 1) + k];
            n[j] = base[L * (kListSlots + 1) + k + 1] - b0[j];
            nmax = max(nmax, n[j]);
        }
        for (uint32_t i = lane; i < nmax; i += 64) {
            uint32_t v[kGroup];
#pragma unroll
            for (uint32_t j = 0; j < kGroup; ++j) v[j] = i < n[j] ? slots[(size_t)(s0 + j) * cap + i] : 0u;
#pragma unroll
            for (uint32_t j = 0; j < kGroup; ++j)
                if (i < n[j]) ((s0 + j) / kListSlots ? full : heavy)[b0[j] + i] = v[j];
        }
    }
}

// NGS_SYNC_DEBUG=1 (diagnostics): every launch of a search is followed by a wait on its stream,
// and the first kernel whose wait fails is named on stderr (a fault is otherwise reported by a
// later, unrelated call)
// workgroups of a persistent grid: one per slot of the GPU at `waves_per_simd` one-wave workgroups
// per SIMD (CUs x 4 SIMDs x waves), for the device current on the calling thread
static uint32_t persistent_slots(uint32_t waves_per_simd) {
    static std::atomic<int> cu_count[64] = {};  // per device, read once
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    int cus = cu_count[dev].load(std::memory_order_relaxed);
    if (cus <= 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        cu_count[dev].store(cus, std::memory_order_relaxed);
    }
    return (uint32_t)cus * 4u * waves_per_simd;
}

static bool sync_debug() {
    static const bool on = [] {
        const char* e = std::getenv("NGS_SYNC_DEBUG");
        return e && std::atoi(e) != 0;
    }();
    return on;
}
static void dbg_check(hipStream_t s, const char* what) {
    if (!sync_debug()) return;
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) std::fprintf(stderr, "ngram_search: NGS_SYNC_DEBUG: %s failed: %s\n", what, hipGetErrorString(e));
}

// A kernel launch queued on s, or with gb, a kernel node appended to gb's graph after its last
// node (the arguments converted to the kernel's parameter types and copied into the node)
template <typename... KArgs, typename... Args>
static void klaunch(GraphBuild* gb, void (*k)(KArgs...), dim3 grid, dim3 block, size_t shm, hipStream_t s,
                    Args... args) {
    if (!gb) {
        hipLaunchKernelGGL(k, grid, block, shm, s, args...);
        return;
    }
    if (gb->err != hipSuccess) return;
    std::tuple<KArgs...> vals(static_cast<KArgs>(args)...);
    void* ptrs[sizeof...(KArgs) > 0 ? sizeof...(KArgs) : 1];
    std::apply([&](auto&... v) {
        size_t i = 0;
        ((ptrs[i++] = static_cast<void*>(&v)), ...);
    }, vals);
    hipKernelNodeParams p{};
    p.func = reinterpret_cast<void*>(k);
    p.gridDim = grid;
    p.blockDim = block;
    p.sharedMemBytes = (unsigned)shm;
    p.kernelParams = ptrs;
    p.extra = nullptr;
    hipGraphNode_t n = nullptr;
    gb->err = hipGraphAddKernelNode(&n, gb->graph, gb->last ? &gb->last : nullptr, gb->last ? 1 : 0, &p);
    if (gb->err == hipSuccess) gb->last = n;
}

hipError_t launch_prep(const uint8_t* raw, const uint64_t* off, uint32_t B, const SearchParams& P, uint8_t* qnorm,
                       uint32_t* qm, uint32_t cs, const DevIndex& X, uint32_t* heavy, uint32_t* hcount,
                       uint32_t* full, uint32_t* fcount, uint32_t* slots, uint32_t* ctr, hipStream_t s,
                       hipStream_t side, hipEvent_t prep_ev, hipEvent_t lists_ev, GraphBuild* gb) {
    if (!B) return hipSuccess;
    if (gb && side != s) return hipErrorInvalidValue;  // (a built graph has no events)
    const uint32_t cap = (B + kListSlots - 1) / kListSlots;
    const bool lists = P.waves == 0;
    klaunch(gb, k_prep, dim3((B + 3) / 4), dim3(64), 0, s, raw, off, B, P, qnorm, qm, cs, X,
                       lists ? slots : nullptr, ctr, cap);
    dbg_check(s, "k_prep");
    if (lists) {  // on the side stream: the main tier-1a launch needs only k_prep's output
        hipError_t e;
        // (one-stream calls, side == s: no cross-stream ordering to queue; a C2 step is ~0.1 ms of
        // GPU time for ~20 host calls, so each one left out counts)
        if (side != s &&
            ((e = hipEventRecord(prep_ev, s)) != hipSuccess || (e = hipStreamWaitEvent(side, prep_ev, 0)) != hipSuccess))
            return e;
        klaunch(gb, k_lists, dim3(1), dim3(64), 0, side, slots, ctr, cap, heavy, hcount, full, fcount);
        dbg_check(side, "k_lists");
        if (side != s && (e = hipEventRecord(lists_ev, side)) != hipSuccess) return e;
    }
    return gb ? gb->err : hipGetLastError();
}

// Workgroups for every (query, slice) item heavy_slices can make from a list of up to n_queries
// queries: automatic slicing keeps cnt x slices within max(kHeavyItems, cnt), so on long-list
// indexes max(kHeavyItems, n_queries), else one per query (C2); NGS_HEAVY_SLICES: n_queries x that
// many. The first heavy launch takes the context's last item count instead (P.hgrid; C3: ~19k
// where this bound is 65,536: the 46k workgroups that only exited cost 2.7 % of a step), and an
// overflow launch the rest.
uint32_t heavy_grid(const DevIndex& X, const SearchParams& P) {
    const uint64_t B = std::max<uint32_t>(P.n_queries, 1);
    uint64_t g = P.hslices ? B * std::min<uint32_t>(P.hslices, kHeavyMaxSlices)
               : X.post_per_row < kHeavySliceList ? B : std::max<uint64_t>(kHeavyItems, B);
    return (uint32_t)std::min<uint64_t>(g, B * kHeavyMaxSlices);
}

hipError_t launch_fast(const DevIndex& X, const SearchParams& P, const uint8_t* qnorm, const uint64_t* off,
                       const uint32_t* qm, uint32_t* out_n, uint32_t* out_k, float* out_s, uint32_t* list2,
                       uint32_t* count2, uint32_t* fb, uint32_t* fbc, uint32_t* fb2, uint32_t* fbc2,
                       const uint32_t* heavy, const uint32_t* hcount, const uint32_t* full,
                       const uint32_t* fcount, uint32_t* glist, uint32_t* gcount, DevStats* stats, hipStream_t s,
                       hipStream_t side, hipStream_t side2, hipEvent_t join, hipEvent_t join2,
                       hipEvent_t lists_ev, bool all_heavy, hipEvent_t main_ev, bool main_wait, GraphBuild* gb) {
    if (!P.n_queries) return hipSuccess;
    if (gb && (side != s || side2 != s || main_ev)) return hipErrorInvalidValue;  // (no events in a built graph)
    hipError_t e = hipSuccess;
    switch (P.waves) {  // SearchParams.waves: 0 = tier 1a + 1b (batches), 1 = tier 1b alone (latency path)
        case 0: {
            // beside tier 1a: the heavy list through the lean kernel, k_emit and tier 1b on its
            // hand-overs (side), and the full list through tier 1b (side2)
            const uint32_t g1b = std::min<uint32_t>(P.n_queries, 1024);  // k_merge: grid-stride over the list
            // tier-1b launches over the hand-over and full lists: persistent grids of one workgroup
            // per slot of the GPU (kWaveWavesPerSimd per SIMD), items from a counter in the
            // path-count line (zeroed per call with it)
            const uint32_t g1s = std::min<uint32_t>(P.n_queries * std::max<uint32_t>(P.nslices, 1u),
                                                    std::min<uint32_t>(persistent_slots(kWaveWavesPerSimd), kTier1bGrid));
            const uint32_t gh = std::min<uint32_t>(P.n_queries, kHeavyGrid);  // (the heavy k_emit's grid)
            // the heavy lean launch: as many workgroups as the context's last call had items (every item
            // heavy_slices can make otherwise), the rest in an overflow launch
            const uint32_t ghb = heavy_grid(X, P);
            const uint32_t ghl = P.hgrid ? std::min(P.hgrid, ghb) : ghb;
            const uint32_t gfull = std::min<uint32_t>(P.n_queries, std::min<uint32_t>(persistent_slots(kWaveWavesPerSimd), kTier1bGrid));
            SearchParams PM = P, PHO = P;  // the main and the heavy hand-over launches
            PM.qhead = gcount + 8;
            PHO.qhead = gcount + 9;
            // (esn[] was reset by k_prep)
            // main_ev (NGS_SERIAL_MAIN): the replica's last main launch, waited for (main_wait) before this
            // one and recorded after it, so that two calls in flight do not run their main launches at once
            auto main_lean = [&]() {
                if (main_ev && main_wait) (void)hipStreamWaitEvent(s, main_ev, 0);
                klaunch(gb, (k_wave_lean<false>), dim3(P.n_queries), dim3(64), 0, s, X,
                                   P, qnorm, off, qm,
                                   out_n, out_k, out_s, list2, count2, stats, fb, fbc, (const uint32_t*)nullptr,
                                   (const uint32_t*)nullptr);
                dbg_check(s, "k_wave_lean");
                if (main_ev) (void)hipEventRecord(main_ev, s);
            };
            // the main launch is queued first: the GPU idled ~35 us while the host queued the side
            // streams' launches ahead of it
            main_lean();
            // then the heavy list's chain on side, which is already ordered after k_prep with k_lists
            // queued on it (launch_prep): queued second, so that it starts soon after k_lists (the
            // host queues ~15 operations per call; at C2 this launch carries every query)
            // (the heavy chain deferred until the main launch ends measured slower at C3, 35.5-35.7
            // against 36.5-36.6 Mq/s; fused with its k_emit into one kernel slower too, C2 18 against
            // 33-35: profiles/r04_s2_ab_defer_heavy.txt, r04_s2_ab_heavy_fuse.txt)
            {
                SearchParams PH = P;
                PH.lean_all = 1;
                {
                    // part_ones is compiled in only where a lean query can have cmin 1: without rank lists,
                    // at a threshold the shortest lean query (n_min grams) passes with one hit
                    const uint32_t n_min = (X.n_short ? X.short_query_len : X.full_scan_len + 1) - X.gsz + 1;
                    const bool ones = !X.rank_post && !(1.0f / (float)n_min < P.thr);
                    PH.hbase = 0;
                    if (ones)
                        klaunch(gb, (k_wave_lean<true, true>), dim3(ghl), dim3(64), 0, side, X, PH,
                                           qnorm, off, qm, out_n, out_k, out_s, list2, count2, stats, fb2, fbc2, heavy,
                                           hcount);
                    else
                        klaunch(gb, (k_wave_lean<true, false>), dim3(ghl), dim3(64), 0, side, X, PH, qnorm,
                                           off, qm, out_n, out_k, out_s, list2, count2, stats, fb2, fbc2, heavy, hcount);
                    dbg_check(side, "k_wave_lean (heavy list)");
                    if (ghl < ghb) {  // items past the first grid, if this call has more than the last
                        PH.hbase = ghl;
                        const uint32_t gov = std::min<uint32_t>(ghb - ghl, kHeavyOverflowGrid);
                        if (ones)
                            klaunch(gb, (k_wave_lean<true, true, true>), dim3(gov), dim3(64), 0,
                                               side, X, PH, qnorm, off, qm, out_n, out_k, out_s, list2, count2, stats,
                                               fb2, fbc2, heavy, hcount);
                        else
                            klaunch(gb, (k_wave_lean<true, false, true>), dim3(gov), dim3(64), 0, side,
                                               X, PH, qnorm, off, qm, out_n, out_k, out_s, list2, count2, stats, fb2,
                                               fbc2, heavy, hcount);
                        dbg_check(side, "k_wave_lean (heavy list overflow)");
                        PH.hbase = 0;
                    }
                    klaunch(gb, k_emit<true>, dim3((gh + kEmitWaves - 1) / kEmitWaves), dim3(64 * kEmitWaves), 0,
                                       side, X, PH, qnorm, off, qm, out_n, out_k, out_s, stats, heavy, hcount);
                    dbg_check(side, "k_emit (heavy list)");
                }
                klaunch(gb, k_wave, dim3(g1s), dim3(64), 0, side, X, PHO, qnorm, off, qm, out_n, out_k,
                                   out_s, list2, count2, stats, (const uint32_t*)fb2, (const uint32_t*)fbc2);
                dbg_check(side, "k_wave (heavy hand-overs)");
                if (P.nslices > 1) {
                    klaunch(gb, k_merge, dim3(g1b), dim3(64), 0, side, X, P, (const uint32_t*)fb2,
                                       (const uint32_t*)fbc2, out_n, out_k, out_s, stats);
                    dbg_check(side, "k_merge (heavy hand-overs)");
                }
            }
            if (side != s && side2 != side && (e = hipEventRecord(join, side)) != hipSuccess) return e;
            // side2 waits for the lists (recorded on side in launch_prep when side != s)
            if (side2 != side && side != s && (e = hipStreamWaitEvent(side2, lists_ev, 0)) != hipSuccess) return e;
            {
                // unsliced: its cmin-1 parts are all counted exactly, and four slices of a C2 query
                // measured 17 % slower than one wave (the hand-over lists below gain from slicing)
                SearchParams PF = P;
                PF.nslices = 1;
                PF.qhead = gcount + 10;
                klaunch(gb, k_wave, dim3(gfull), dim3(64), 0, side2, X, PF, qnorm, off, qm, out_n, out_k,
                                   out_s, list2, count2, stats, full, fcount);
                dbg_check(side2, "k_wave (full list)");
            }
            if (side2 != s && (e = hipEventRecord(join2, side2)) != hipSuccess) return e;
            // all_heavy (every lean query on the heavy list, e.g. threshold 0): the main launch finishes
            // no query and hands none over (it returns before either for a heavy or full one), so its
            // k_emit and hand-over launches would find nothing
            if (!all_heavy) {
                klaunch(gb, k_emit<false>, dim3((P.n_queries + kEmitWaves - 1) / kEmitWaves), dim3(64 * kEmitWaves), 0,
                                   s, X, P, qnorm, off, qm, out_n, out_k, out_s, stats, (const uint32_t*)nullptr,
                                   (const uint32_t*)nullptr);
                dbg_check(s, "k_emit");
            }
            // tier 1b over the queries tier 1a handed over
            if (!all_heavy) {
                klaunch(gb, k_wave, dim3(g1s), dim3(64), 0, s, X, PM, qnorm, off, qm, out_n, out_k, out_s,
                                   list2, count2, stats, (const uint32_t*)fb, (const uint32_t*)fbc);
                dbg_check(s, "k_wave (hand-overs)");
            }
            if (P.nslices > 1 && !all_heavy) {
                klaunch(gb, k_merge, dim3(g1b), dim3(64), 0, s, X, P, (const uint32_t*)fb, (const uint32_t*)fbc,
                                   out_n, out_k, out_s, stats);
                dbg_check(s, "k_merge (hand-overs)");
            }
            // (join2 is recorded after join when side2 is side: then it alone orders s after both)
            if ((side != s && side2 != side && (e = hipStreamWaitEvent(s, join, 0)) != hipSuccess) ||
                (side2 != s && (e = hipStreamWaitEvent(s, join2, 0)) != hipSuccess))
                return e;
            break;
        }
        case 1:
            klaunch(gb, k_wave, dim3(P.n_queries * std::max<uint32_t>(P.nslices, 1u)), dim3(64), 0, s, X, P,
                               qnorm, off, qm, out_n, out_k, out_s, list2, count2, stats, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr);
            dbg_check(s, "k_wave");
            if (P.nslices > 1) {
                klaunch(gb, k_merge, dim3(P.n_queries), dim3(64), 0, s, X, P, (const uint32_t*)nullptr,
                                   (const uint32_t*)nullptr, out_n, out_k, out_s, stats);
                dbg_check(s, "k_merge");
            }
            break;
        default:
            return hipErrorInvalidValue;
    }
    // tier 2 takes every query at a limit past the wave kernels' (1,024 blocks), else only the rare
    // long ones (> 63 grams) and those bound for the general path: 128 blocks, grid-stride (1,024
    // blocks that mostly exit cost ~20 us at C2 and ~50 us at C3 per call)
    const uint32_t grid2 = std::min<uint32_t>(P.n_queries, P.limit > kWaveMaxLimit ? 1024u : 128u);
    klaunch(gb, k_fast, dim3(grid2), dim3(kFastThreads), 0, s, X, P, qnorm, off, qm, out_n, out_k, out_s,
                       (const uint32_t*)list2, (const uint32_t*)count2, glist, gcount, stats);
    dbg_check(s, "k_fast");
    if (gb) return gb->err;
    return hipGetLastError();
}

hipError_t launch_serve(const DevIndex& X, const SearchParams& P, ServeBlock* blk, DevStats* scratch,
                        uint32_t* list2, unsigned long long* t_any, uint32_t idle_ms, uint32_t life_ms, hipStream_t s) {
    hipLaunchKernelGGL(k_serve, dim3(kServeSlots), dim3(64), 0, s, X, P, blk, scratch, list2, t_any, idle_ms, life_ms);
    return hipGetLastError();
}

// one wave per query: its records to the packed arrays. With pp, each key goes out as the
// caller's result pointer instead, pbase + key_off[key] * cs (the host image of the key bytes):
// the random key_off gathers happen here, in HBM, not in the host's marshalling loop
__global__ __launch_bounds__(256) void k_pack(const uint32_t* __restrict__ n, const uint32_t* __restrict__ k,
                                              const float* __restrict__ s, uint32_t B, uint32_t stride,
                                              const uint32_t* __restrict__ pos, uint32_t* __restrict__ pk,
                                              float* __restrict__ ps, const uint64_t* __restrict__ koff,
                                              uint64_t pbase, uint32_t cs, uint64_t* __restrict__ pp) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (q >= B) return;
    const uint32_t c = n[q], o = pos[q];
    const size_t src = (size_t)q * stride;
    for (uint32_t i = lane; i < c; i += 64) {
        if (pp)
            pp[o + i] = pbase + koff[k[src + i]] * cs;
        else
            pk[o + i] = k[src + i];
        ps[o + i] = s[src + i];
    }
}

size_t pack_temp_bytes(uint32_t B) {
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)B + 1);
    return bytes;
}

hipError_t launch_pack(const uint32_t* n, const uint32_t* k, const float* s, uint32_t B, uint32_t stride,
                       uint32_t* pos, uint32_t* pk, float* ps, void* temp, size_t temp_bytes, hipStream_t st,
                       const uint64_t* koff, uint64_t pbase, uint32_t cs, uint64_t* pp) {
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, n, pos, (int)B + 1, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pack, dim3((B + 3) / 4), dim3(256), 0, st, n, k, s, B, stride, pos, pk, ps, koff, pbase, cs,
                       pp);
    return hipGetLastError();
}

// one wave per query, as k_pack: query q's count records to rec[2 pos[q] ..] as {key, score bits}
__global__ __launch_bounds__(256) void k_pack_pairs(const uint32_t* __restrict__ n, const uint32_t* __restrict__ k,
                                                    const float* __restrict__ s, uint32_t B, uint32_t stride,
                                                    const uint32_t* __restrict__ pos, uint2* __restrict__ rec) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (q >= B) return;
    const uint32_t c = min(n[q], stride), o = pos[q];
    const size_t src = (size_t)q * stride;
    for (uint32_t i = lane; i < c; i += 64) rec[o + i] = make_uint2(k[src + i], __float_as_uint(s[src + i]));
}

size_t pack_pairs_temp_bytes(uint32_t B) {
    size_t bytes = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (int)std::max<uint32_t>(B, 1));
    return bytes;
}

// (the caller's counts hold B entries: an inclusive sum into pos + 1 behind pos[0] = 0)
hipError_t launch_pack_pairs(const uint32_t* n, const uint32_t* k, const float* s, uint32_t B, uint32_t stride,
                             uint32_t* pos, uint32_t* rec, void* temp, size_t temp_bytes, hipStream_t st) {
    hipError_t e = hipMemsetAsync(pos, 0, sizeof(uint32_t), st);
    if (e == hipSuccess && B) e = hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, n, pos + 1, (int)B, st);
    if (e != hipSuccess) return e;
    if (B) hipLaunchKernelGGL(k_pack_pairs, dim3((B + 3) / 4), dim3(256), 0, st, n, k, s, B, stride, pos,
                              reinterpret_cast<uint2*>(rec));
    return hipGetLastError();
}

size_t general_sort_temp_bytes(uint32_t n_keys) {
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                      (int)std::max<uint32_t>(n_keys, 1));
    return bytes;
}

hipError_t run_general(const DevIndex& X, const SearchParams& P, const uint8_t* qnorm, const uint64_t* off,
                       const uint32_t* qm, const uint32_t* d_group, const uint32_t* h_group, uint32_t G,
                       GeneralBuffers& W, uint32_t* out_n, uint32_t* out_k, float* out_s, hipStream_t s) {
    const uint32_t n_long = X.n_terms - X.n_short;
    hipError_t e = hipMemsetAsync(W.lcount, 0, sizeof(uint32_t) * G, s);
    if (e != hipSuccess) return e;
    if (n_long) {
        hipLaunchKernelGGL(k_gen_long, dim3(128, G), dim3(256), 0, s, X, P, qnorm, off, qm, d_group, W.cnt, W.kenc, 0);
        hipLaunchKernelGGL(k_gen_long, dim3(128, G), dim3(256), 0, s, X, P, qnorm, off, qm, d_group, W.cnt, W.kenc, 1);
    }
    if (X.n_terms) {
        const uint32_t gx = std::min<uint32_t>((X.n_terms + 255) / 256, 2048);
        hipLaunchKernelGGL(k_gen_short, dim3(gx, G), dim3(256), 0, s, X, P, qnorm, off, qm, d_group, W.kenc);
    }
    if (P.limit <= kGenSelCap) {  // top-L in one kernel, no host round trip
        hipLaunchKernelGGL(k_gen_select, dim3(G), dim3(kGenSelThreads), 0, s, X.n_keys, W.kenc, d_group, P, out_n,
                           out_k, out_s);
        return hipGetLastError();
    }
    if (X.n_keys) {
        const uint32_t gx = std::min<uint32_t>((X.n_keys + 255) / 256, 2048);
        hipLaunchKernelGGL(k_gen_compact, dim3(gx, G), dim3(256), 0, s, X.n_keys, W.kenc, W.list, W.lcount);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t counts[kGeneralMaxGroup];
    if (G > kGeneralMaxGroup) return hipErrorInvalidValue;
    if ((e = hipMemcpyAsync(counts, W.lcount, sizeof(uint32_t) * G, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    for (uint32_t gi = 0; gi < G; ++gi) {
        const uint64_t* src = W.list + (size_t)gi * X.n_keys;
        if (counts[gi] > 1) {
            size_t bytes = W.temp_bytes;
            e = hipcub::DeviceRadixSort::SortKeys(W.temp, bytes, src, W.sorted, (int)counts[gi], 0, 64, s);
            if (e != hipSuccess) return e;
            src = W.sorted;
        }
        const uint32_t cnt = std::min(counts[gi], P.limit);
        const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((cnt + 255) / 256, 1024));
        hipLaunchKernelGGL(k_gen_write, dim3(gx), dim3(256), 0, s, src, counts[gi], h_group[gi], P, out_n, out_k, out_s);
    }
    return hipGetLastError();
}

}  // namespace ngs
