// ngs_intern.hip — the rest of the index build on the GPU: string interning of the normalised
// terms and the trimmed master keys, term ids, key ranks and the term -> (key, weight) CSR.
//
// Reference: the constructor's row loop (nGramSearch.hpp:120-172: trim the key, escapeBlank +
// trim + toUpper every word, skip NULL words / empty aliases / zero weights, wordMap[term] and
// tempWeightMap[term][key] = weight, last write wins) and init's id assignment (hpp:54-108:
// shortLib for terms < 6 characters, longLib for the rest). The host restatement is
// ngs_index.cpp build_impl; this builds the same arrays, bit for bit (ngsIndexDigest compares
// them in tests/test_gpu_build.py):
//   1. k_rows    per row: the trimmed key (bounds, hash); rows whose key is NULL or blank drop out
//   2. k_words   per word: normalised term into a blob at the word's offset, validity of its
//                (term, key) pair, term hash
//   3. terms     valid words sorted by (hash, word): equal-hash runs are one term (every member is
//                compared with the run head: a 64-bit collision falls back to the host build);
//                term ids = runs sorted by (long?, first word), or (long?, best key rank of the
//                term's words, first word) with term_order_by_rank() (after step 4)
//   4. keys      rows with a valid pair sorted by (key hash, row): runs are keys; ranks = runs
//                sorted by (length, first row) — the ScoreComparer tie-break (h:262-269) plus
//                first appearance
//   5. pairs     (term, key) sorted with the word index: runs are distinct pairs; the weight is the
//                run's last word's (last write wins), its position the first word's; pairs sorted
//                by (term, first word) give tk in the host build's order
//   6. layout    term_off / term_bytes, key_off / key_bytes (+ NUL), tk_off / tk, wild_w (max weight
//                of the key's pairs)
// Everything returns to the host index (HostIndex), which keeps the keys for result marshalling
// and uploads the rest to every replica.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "ngs_build.h"
#include "ngs_index.h"

namespace ngs {
namespace {

#define TRY(x)                                \
    do {                                      \
        const hipError_t e_ = (x);            \
        if (e_ != hipSuccess) return e_;      \
    } while (0)

constexpr uint32_t kInternCollision = 1u;  // two different strings with one 64-bit hash
constexpr uint32_t kInternNaN = 2u;        // a NaN weight (host semantics: first-seen NaN sticks)
constexpr uint64_t kKeyLenBit = 1ull << 40;      // key order key: (length << 40) | row
constexpr uint64_t kTermLongBit = 1ull << 63;    // term order key: long? | best key rank << 31 | first word
constexpr uint64_t kTermItemMask = (1ull << 31) - 1;

__device__ __forceinline__ bool d_space(uint32_t c) { return c == 32u || (c >= 9u && c <= 13u); }

// escapeBlank of one character (nGramSearch.h:93-98); wide code points >= 128 are kept, values
// above 0x10FFFF become spaces
template <typename CharT>
__device__ __forceinline__ uint32_t d_esc(const uint32_t* valid, uint32_t c) {
    if (sizeof(CharT) == 1 || c < 128u) return ((valid[c >> 5] >> (c & 31u)) & 1u) ? c : 32u;
    return c > 0x10FFFFu ? 32u : c;
}

template <typename CharT>
__device__ __forceinline__ uint64_t d_hash(const CharT* p, uint64_t n) {
    uint64_t h = 0xCBF29CE484222325ull ^ (n * 0x9E3779B97F4A7C15ull);
    for (uint64_t i = 0; i < n; ++i) h = (h ^ (uint64_t)(uint32_t)p[i]) * 0x100000001B3ull;
    h ^= h >> 31;
    h *= 0xD6E8FEB86659FD93ull;
    return h ^ (h >> 29);
}

struct Valid {
    uint32_t bits[8];
};

// 1. per row: the trimmed master key (hpp:129-134: NULL key or blank key -> the row is skipped)
template <typename CharT>
__global__ __launch_bounds__(256) void k_rows(const CharT* __restrict__ blob, const uint64_t* __restrict__ woff,
                                              const uint8_t* __restrict__ isnull, uint64_t size, uint32_t rowSize,
                                              uint64_t nrows, uint32_t* __restrict__ ka, uint32_t* __restrict__ kl,
                                              uint64_t* __restrict__ kh) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    const uint64_t head = r * rowSize;
    uint32_t a = 0, b = 0;
    if (!isnull[head]) {
        const CharT* p = blob + woff[head];
        b = (uint32_t)(woff[head + 1] - woff[head]);
        while (a < b && (uint32_t)p[a] < 128u && d_space(p[a])) ++a;  // trim(strKey): isspace, no escape
        while (b > a && (uint32_t)p[b - 1] < 128u && d_space(p[b - 1])) --b;
        kh[r] = d_hash(p + a, b - a);
    }
    ka[r] = a;
    kl[r] = b - a;  // 0: no key, the row yields no pair
}

// 2. per word: the normalised term (escapeBlank -> trim -> toUpper, hpp:136-139, :153-156) and
// whether the word makes a (term, key) pair (non-NULL, a key, a non-empty alias term, weight != 0)
template <typename CharT>
__global__ __launch_bounds__(256) void k_words(const CharT* __restrict__ blob, const uint64_t* __restrict__ woff,
                                               const uint8_t* __restrict__ isnull, uint64_t size, uint32_t rowSize,
                                               const float* __restrict__ weight, Valid V,
                                               const uint32_t* __restrict__ kl, CharT* __restrict__ nblob,
                                               uint32_t* __restrict__ tlen, uint64_t* __restrict__ th,
                                               uint32_t* __restrict__ vflag, uint8_t* __restrict__ rowany,
                                               uint32_t* __restrict__ err) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= size) return;
    const uint64_t row = j / rowSize, head = row * rowSize;
    uint32_t ok = 0;
    if (!isnull[j] && kl[row]) {
        const CharT* p = blob + woff[j];
        uint32_t a = 0, b = (uint32_t)(woff[j + 1] - woff[j]);
        while (a < b && d_space(d_esc<CharT>(V.bits, p[a]))) ++a;
        while (b > a && d_space(d_esc<CharT>(V.bits, p[b - 1]))) --b;
        CharT* o = nblob + woff[j];
        for (uint32_t i = a; i < b; ++i) {
            const uint32_t c = d_esc<CharT>(V.bits, p[i]);
            o[i - a] = (CharT)((c >= 'a' && c <= 'z') ? c - 32u : c);
        }
        const uint32_t tl = b - a;
        const float w = weight ? weight[j] : 1.0f;  // hpp:141-143, :159-161
        if (w != w) atomicOr(err, kInternNaN);
        ok = (j == head || tl != 0) && w != 0.0f;   // hpp:157 (aliases only), :144, :162
        if (ok) {
            tlen[j] = tl;
            th[j] = d_hash(o, tl);
            rowany[row] = 1;
        }
    }
    vflag[j] = ok;
}

// scatter of the flagged indices to their exclusive-scan positions
__global__ __launch_bounds__(256) void k_compact(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                                                 uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && flag[i]) out[pos[i]] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_row_flags(const uint8_t* __restrict__ rowany, uint64_t n,
                                                   uint32_t* __restrict__ flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = rowany[i];
}

template <class T>
__global__ __launch_bounds__(256) void k_gather64(const T* __restrict__ src, const uint32_t* __restrict__ idx,
                                                  uint32_t n, T* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[idx[i]];
}

// run heads of a sorted u64 array: head[p] = 1 at the first element of every run
__global__ __launch_bounds__(256) void k_heads(const uint64_t* __restrict__ k, uint32_t n, uint32_t* __restrict__ head) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) head[p] = p == 0 || k[p] != k[p - 1];
}

// seg = inclusive scan of heads - 1: the run of every position; hpos[run] = its first position
__global__ __launch_bounds__(256) void k_runs(const uint32_t* __restrict__ head, uint32_t* __restrict__ seg,
                                              uint32_t n, uint32_t* __restrict__ hpos) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t s = seg[p] - 1;
    seg[p] = s;
    if (head[p]) hpos[s] = p;
}

// every member of a run equals the run's first member (else: a hash collision)
template <typename CharT>
__global__ __launch_bounds__(256) void k_check(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ seg,
                                               const uint32_t* __restrict__ hpos, uint32_t n,
                                               const CharT* __restrict__ base, const uint64_t* __restrict__ off,
                                               const uint32_t* __restrict__ start, const uint32_t* __restrict__ len,
                                               uint32_t* __restrict__ err) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t h = hpos[seg[p]];
    if (h == p) return;
    const uint32_t a = idx[p], b = idx[h];
    const uint32_t la = len[a], lb = len[b];
    if (la != lb) {
        atomicOr(err, kInternCollision);
        return;
    }
    const CharT* x = base + off[a] + (start ? start[a] : 0u);
    const CharT* y = base + off[b] + (start ? start[b] : 0u);
    for (uint32_t i = 0; i < la; ++i)
        if (x[i] != y[i]) {
            atomicOr(err, kInternCollision);
            return;
        }
}

// the best (smallest) key rank among each term run's words
__global__ __launch_bounds__(256) void k_term_minrank(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ seg,
                                                      uint32_t n, uint32_t rowSize,
                                                      const uint32_t* __restrict__ key_of_row,
                                                      uint32_t* __restrict__ minr) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) atomicMin(&minr[seg[p]], key_of_row[idx[p] / rowSize]);
}

// order keys of the runs: terms (long?, best key rank, first word), keys (length, first row)
__global__ __launch_bounds__(256) void k_term_order(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ hpos,
                                                    uint32_t nruns, const uint32_t* __restrict__ tlen, uint32_t long_len,
                                                    const uint32_t* __restrict__ minr, uint64_t* __restrict__ okey,
                                                    uint32_t* __restrict__ oval) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nruns) return;
    const uint32_t j = idx[hpos[s]];  // < 2^31 (larger builds stay on the host)
    okey[s] = (tlen[j] >= long_len ? kTermLongBit : 0ull) | ((uint64_t)minr[s] << 31) | j;
    oval[s] = s;
}

__global__ __launch_bounds__(256) void k_key_order(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ hpos,
                                                   uint32_t nruns, const uint32_t* __restrict__ kl,
                                                   uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nruns) return;
    const uint32_t r = idx[hpos[s]];
    okey[s] = ((uint64_t)kl[r] << 40) | r;
    oval[s] = s;
}

// rank of every run (its position in the order), the head item of every rank, and the number of
// short terms (order keys below long_bit)
__global__ __launch_bounds__(256) void k_ranks(const uint64_t* __restrict__ okey_sorted, const uint32_t* __restrict__ oval_sorted,
                                               uint32_t n, uint64_t long_bit, uint32_t* __restrict__ rank_of_run,
                                               uint32_t* __restrict__ n_short) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    rank_of_run[oval_sorted[r]] = r;
    const bool lng = okey_sorted[r] >= long_bit;
    if (lng && (r == 0 || okey_sorted[r - 1] < long_bit)) *n_short = r;
}

// item -> rank of its run (items: the sorted index list)
__global__ __launch_bounds__(256) void k_item_rank(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ seg,
                                                   const uint32_t* __restrict__ rank_of_run, uint32_t n,
                                                   uint32_t* __restrict__ out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) out[idx[p]] = rank_of_run[seg[p]];
}

// per rank: the head item and its length (+ extra: the key's NUL)
__global__ __launch_bounds__(256) void k_rank_items(const uint64_t* __restrict__ okey_sorted, uint32_t n,
                                                    uint64_t item_mask, const uint32_t* __restrict__ len, uint32_t extra,
                                                    uint32_t* __restrict__ item, uint64_t* __restrict__ rlen) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r > n) return;
    if (r == n) {
        rlen[r] = 0;
        return;
    }
    const uint32_t it = (uint32_t)(okey_sorted[r] & item_mask);
    item[r] = it;
    rlen[r] = (uint64_t)len[it] + extra;
}

// strings of the ranks into the packed layout (offsets in characters)
template <typename CharT>
__global__ __launch_bounds__(256) void k_layout(const uint32_t* __restrict__ item, uint32_t n, const CharT* __restrict__ base,
                                                const uint64_t* __restrict__ off, const uint32_t* __restrict__ start,
                                                const uint32_t* __restrict__ len, const uint64_t* __restrict__ dst_off,
                                                CharT* __restrict__ dst, bool nul) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint32_t it = item[r];
    const CharT* s = base + off[it] + (start ? start[it] : 0u);
    CharT* d = dst + dst_off[r];
    const uint32_t l = len[it];
    for (uint32_t i = 0; i < l; ++i) d[i] = s[i];
    if (nul) d[l] = 0;
}

// 5. the (term, key) key of every valid word, in word order
__global__ __launch_bounds__(256) void k_pair_keys(const uint32_t* __restrict__ vj, uint32_t n, uint32_t rowSize,
                                                   const uint32_t* __restrict__ term_of_word,
                                                   const uint32_t* __restrict__ key_of_row, uint64_t* __restrict__ pk) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t j = vj[p];
    pk[p] = ((uint64_t)term_of_word[j] << 32) | key_of_row[j / rowSize];
}

// per run of equal (term, key): the first word orders it, the last word's weight is its weight
__global__ __launch_bounds__(256) void k_pair_runs(const uint64_t* __restrict__ pk, const uint32_t* __restrict__ pj,
                                                   const uint32_t* __restrict__ head, const uint32_t* __restrict__ seg,
                                                   uint32_t n, const float* __restrict__ weight,
                                                   uint64_t* __restrict__ dkey, uint32_t* __restrict__ dval,
                                                   uint2* __restrict__ dpair) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t s = seg[p];
    if (head[p]) {
        dkey[s] = (pk[p] & 0xFFFFFFFF00000000ull) | pj[p];  // (term, first word)
        dval[s] = s;
    }
    if (p + 1 == n || head[p + 1]) {  // the run's last word: last write wins (tempWeightMap)
        const float w = weight ? weight[pj[p]] : 1.0f;
        uint32_t wb;
        memcpy(&wb, &w, 4);
        dpair[s] = make_uint2((uint32_t)pk[p], wb);
    }
}

__device__ __forceinline__ uint32_t f2ord(float f) {
    uint32_t b;
    memcpy(&b, &f, 4);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o) {
    const uint32_t b = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    float f;
    memcpy(&f, &b, 4);
    return f;
}

// tk in (term, first word) order, tk_off from the term runs, the wildcard weight per key (max)
__global__ __launch_bounds__(256) void k_tk(const uint64_t* __restrict__ dkey_sorted, const uint32_t* __restrict__ dval_sorted,
                                            const uint2* __restrict__ dpair, uint32_t n, uint2* __restrict__ tk,
                                            uint32_t* __restrict__ tk_off, uint32_t* __restrict__ wild_ord) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint2 kw = dpair[dval_sorted[r]];
    tk[r] = kw;
    const uint32_t t = (uint32_t)(dkey_sorted[r] >> 32);
    if (r == 0 || (uint32_t)(dkey_sorted[r - 1] >> 32) != t) tk_off[t] = r;
    float w;
    memcpy(&w, &kw.y, 4);
    atomicMax(&wild_ord[kw.x], f2ord(w));
}

__global__ __launch_bounds__(256) void k_unord(const uint32_t* __restrict__ o, uint32_t n, float* __restrict__ w) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) w[i] = ord2f(o[i]);
}

inline dim3 blocks(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }

// device allocations of one build, freed on exit
struct Arena {
    std::vector<void*> ptrs;
    template <class T>
    hipError_t get(T** p, size_t n) {
        *p = nullptr;
        const hipError_t e = hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
    }
    ~Arena() {
        for (void* p : ptrs) hipFree(p);
    }
};

// growing hipcub scratch
struct Temp {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t b) {
        if (b <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        const hipError_t e = hipMalloc(&p, b);
        if (e == hipSuccess) cap = b;
        return e;
    }
    ~Temp() {
        if (p) hipFree(p);
    }
};

// runs of a sorted u64 key array: head flags, run id per position (seg), first position per run
// (hpos); returns the number of runs
hipError_t runs_of(const uint64_t* keys, uint32_t n, uint32_t* head, uint32_t* seg, uint32_t* hpos, Temp& tmp,
                   uint32_t* d_last, uint32_t& nruns) {
    nruns = 0;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_heads, blocks(n), dim3(256), 0, nullptr, keys, n, head);
    size_t b = 0;
    TRY(hipcub::DeviceScan::InclusiveSum(nullptr, b, head, seg, (int)n));
    TRY(tmp.need(b));
    TRY(hipcub::DeviceScan::InclusiveSum(tmp.p, b, head, seg, (int)n));
    TRY(hipMemcpy(&nruns, seg + n - 1, sizeof(uint32_t), hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(k_runs, blocks(n), dim3(256), 0, nullptr, head, seg, n, hpos);
    (void)d_last;
    return hipGetLastError();
}

template <class K, class V>
hipError_t sort_pairs(const K* kin, K* kout, const V* vin, V* vout, uint32_t n, int bits, Temp& tmp) {
    if (!n) return hipSuccess;
    size_t b = 0;
    TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, b, kin, kout, vin, vout, (int)n, 0, bits));
    TRY(tmp.need(b));
    return hipcub::DeviceRadixSort::SortPairs(tmp.p, b, kin, kout, vin, vout, (int)n, 0, bits);
}

template <class T>
hipError_t excl_scan(const T* in, T* out, uint32_t n, Temp& tmp) {
    size_t b = 0;
    TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, (int)n));
    TRY(tmp.need(b));
    return hipcub::DeviceScan::ExclusiveSum(tmp.p, b, in, out, (int)n);
}

template <class T>
hipError_t download(std::vector<T>& v, const T* d, size_t n) {
    v.resize(n);
    return n ? hipMemcpy(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost) : hipSuccess;
}

template <typename CharT>
hipError_t intern_impl(HostIndex& ix, const CharT* const* words, uint64_t size, uint16_t rowSize,
                       const float* weight, uint32_t g) {
    constexpr uint32_t cs = sizeof(CharT);
    if (size >= (1ull << 31) || !words || rowSize == 0 || size < 2) return hipErrorNotSupported;
    const uint64_t nrows = (size + rowSize - 1) / rowSize;
    // host: word lengths and the packed blob (threads over word ranges)
    std::vector<uint64_t> woff(size + 1);
    std::vector<uint8_t> isnull(size + rowSize, 1);  // padded: a short last row reads no word past size
    const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    auto par = [&](auto&& body) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < T; ++t)
            th.emplace_back([&, t] { body(size * t / T, size * (t + 1) / T); });
        for (auto& x : th) x.join();
    };
    par([&](uint64_t b, uint64_t e) {
        for (uint64_t j = b; j < e; ++j) {
            const CharT* w = words[j];
            uint64_t n = 0;
            if (w)
                while (w[n]) ++n;
            woff[j + 1] = n;
            isnull[j] = w == nullptr;
        }
    });
    woff[0] = 0;
    for (uint64_t j = 0; j < size; ++j) woff[j + 1] += woff[j];
    const uint64_t chars = woff[size];
    std::vector<CharT> blob(std::max<uint64_t>(chars, 1));
    par([&](uint64_t b, uint64_t e) {
        for (uint64_t j = b; j < e; ++j)
            if (words[j]) std::memcpy(blob.data() + woff[j], words[j], (woff[j + 1] - woff[j]) * cs);
    });
    // a row's head word past size cannot exist; woff needs entries up to nrows * rowSize + 1
    woff.resize(nrows * rowSize + 1, chars);
    PhaseTimer pt;

    Arena A;
    Temp tmp;
    CharT *d_blob, *d_nblob;
    uint64_t *d_woff, *d_th, *d_kh;
    uint8_t *d_null, *d_rowany;
    float* d_w = nullptr;
    uint32_t *d_ka, *d_kl, *d_tlen, *d_vflag, *d_err;
    TRY(A.get(&d_blob, std::max<uint64_t>(chars, 1)));
    TRY(A.get(&d_nblob, std::max<uint64_t>(chars, 1)));
    TRY(A.get(&d_woff, woff.size()));
    TRY(A.get(&d_null, isnull.size()));
    TRY(A.get(&d_th, size));
    TRY(A.get(&d_kh, nrows));
    TRY(A.get(&d_rowany, nrows));
    TRY(A.get(&d_ka, nrows));
    TRY(A.get(&d_kl, nrows));
    TRY(A.get(&d_tlen, size));
    TRY(A.get(&d_vflag, size + 1));
    TRY(A.get(&d_err, 2));
    TRY(hipMemcpy(d_blob, blob.data(), std::max<uint64_t>(chars, 1) * cs, hipMemcpyHostToDevice));
    TRY(hipMemcpy(d_woff, woff.data(), woff.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    TRY(hipMemcpy(d_null, isnull.data(), isnull.size(), hipMemcpyHostToDevice));
    if (weight) {
        TRY(A.get(&d_w, size));
        TRY(hipMemcpy(d_w, weight, size * sizeof(float), hipMemcpyHostToDevice));
    }
    pt.mark("intern: blob to HBM");
    std::vector<uint8_t>().swap(isnull);
    std::vector<CharT>().swap(blob);
    TRY(hipMemset(d_rowany, 0, nrows));
    TRY(hipMemset(d_err, 0, 2 * sizeof(uint32_t)));
    TRY(hipMemset(d_vflag + size, 0, sizeof(uint32_t)));
    Valid V{};
    {  // nGramSearch.h:307-313, the index's (default) validChar set
        static const char kValid[] = ".%$ @0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ";
        for (const char* c = kValid; *c; ++c) V.bits[(uint8_t)*c >> 5] |= 1u << ((uint8_t)*c & 31u);
    }
    hipLaunchKernelGGL(k_rows<CharT>, blocks(nrows), dim3(256), 0, nullptr, d_blob, d_woff, d_null, size, rowSize, nrows,
                       d_ka, d_kl, d_kh);
    hipLaunchKernelGGL(k_words<CharT>, blocks(size), dim3(256), 0, nullptr, d_blob, d_woff, d_null, size, rowSize, d_w, V,
                       d_kl, d_nblob, d_tlen, d_th, d_vflag, d_rowany, d_err);
    TRY(hipGetLastError());

    // ---- 3. terms ----
    uint32_t *d_pos, *d_vj;
    TRY(A.get(&d_pos, size + 1));
    TRY(excl_scan(d_vflag, d_pos, (uint32_t)size + 1, tmp));
    uint32_t V_n = 0;
    TRY(hipMemcpy(&V_n, d_pos + size, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (!V_n) return hipErrorNotSupported;  // no pair at all: the host build handles the empty index
    TRY(A.get(&d_vj, V_n));
    hipLaunchKernelGGL(k_compact, blocks(size), dim3(256), 0, nullptr, d_vflag, d_pos, size, d_vj);
    uint64_t *d_hv, *d_hs;
    uint32_t *d_sj, *d_head, *d_seg, *d_hpos;
    TRY(A.get(&d_hv, V_n));
    TRY(A.get(&d_hs, V_n));
    TRY(A.get(&d_sj, V_n));
    TRY(A.get(&d_head, V_n + 1));
    TRY(A.get(&d_seg, V_n + 1));
    TRY(A.get(&d_hpos, V_n + 1));
    hipLaunchKernelGGL(k_gather64<uint64_t>, blocks(V_n), dim3(256), 0, nullptr, d_th, d_vj, V_n, d_hv);
    TRY(sort_pairs(d_hv, d_hs, d_vj, d_sj, V_n, 64, tmp));
    uint32_t n_terms = 0;
    TRY(runs_of(d_hs, V_n, d_head, d_seg, d_hpos, tmp, nullptr, n_terms));
    hipLaunchKernelGGL(k_check<CharT>, blocks(V_n), dim3(256), 0, nullptr, d_sj, d_seg, d_hpos, V_n, d_nblob, d_woff,
                       (const uint32_t*)nullptr, d_tlen, d_err);
    // ---- 4. keys: rows with a valid pair ----
    uint32_t *d_rflag, *d_rpos, *d_vr;
    TRY(A.get(&d_rflag, nrows + 1));
    TRY(A.get(&d_rpos, nrows + 1));
    hipLaunchKernelGGL(k_row_flags, blocks(nrows), dim3(256), 0, nullptr, d_rowany, nrows, d_rflag);
    TRY(hipMemset(d_rflag + nrows, 0, sizeof(uint32_t)));
    TRY(excl_scan(d_rflag, d_rpos, (uint32_t)nrows + 1, tmp));
    uint32_t R_n = 0;
    TRY(hipMemcpy(&R_n, d_rpos + nrows, sizeof(uint32_t), hipMemcpyDeviceToHost));
    TRY(A.get(&d_vr, R_n));
    hipLaunchKernelGGL(k_compact, blocks(nrows), dim3(256), 0, nullptr, d_rflag, d_rpos, nrows, d_vr);
    // row r's key starts at woff[r * rowSize] + ka[r]: an offset array indexed by row
    uint64_t* d_rowoff;
    TRY(A.get(&d_rowoff, nrows));
    {
        std::vector<uint64_t> ro(nrows);
        for (uint64_t r = 0; r < nrows; ++r) ro[r] = woff[r * rowSize];
        TRY(hipMemcpy(d_rowoff, ro.data(), nrows * sizeof(uint64_t), hipMemcpyHostToDevice));
    }
    uint64_t *d_khv, *d_khs;
    uint32_t *d_sr, *d_khead, *d_kseg, *d_khpos;
    TRY(A.get(&d_khv, R_n));
    TRY(A.get(&d_khs, R_n));
    TRY(A.get(&d_sr, R_n));
    TRY(A.get(&d_khead, R_n + 1));
    TRY(A.get(&d_kseg, R_n + 1));
    TRY(A.get(&d_khpos, R_n + 1));
    hipLaunchKernelGGL(k_gather64<uint64_t>, blocks(R_n), dim3(256), 0, nullptr, d_kh, d_vr, R_n, d_khv);
    TRY(sort_pairs(d_khv, d_khs, d_vr, d_sr, R_n, 64, tmp));
    uint32_t n_keys = 0;
    TRY(runs_of(d_khs, R_n, d_khead, d_kseg, d_khpos, tmp, nullptr, n_keys));
    hipLaunchKernelGGL(k_check<CharT>, blocks(R_n), dim3(256), 0, nullptr, d_sr, d_kseg, d_khpos, R_n, d_blob, d_rowoff,
                       d_ka, d_kl, d_err);
    uint64_t *d_kok, *d_koks;
    uint32_t *d_kov, *d_kovs, *d_krank, *d_key_of_row, *d_dummy;
    TRY(A.get(&d_kok, n_keys));
    TRY(A.get(&d_koks, n_keys));
    TRY(A.get(&d_kov, n_keys));
    TRY(A.get(&d_kovs, n_keys));
    TRY(A.get(&d_krank, n_keys));
    TRY(A.get(&d_key_of_row, nrows));
    TRY(A.get(&d_dummy, 1));
    hipLaunchKernelGGL(k_key_order, blocks(n_keys), dim3(256), 0, nullptr, d_sr, d_khpos, n_keys, d_kl, d_kok, d_kov);
    TRY(sort_pairs(d_kok, d_koks, d_kov, d_kovs, n_keys, 64, tmp));
    hipLaunchKernelGGL(k_ranks, blocks(n_keys), dim3(256), 0, nullptr, d_koks, d_kovs, n_keys, kKeyLenBit, d_krank,
                       d_dummy);
    hipLaunchKernelGGL(k_item_rank, blocks(R_n), dim3(256), 0, nullptr, d_sr, d_kseg, d_krank, R_n, d_key_of_row);
    uint32_t* d_kitem;
    uint64_t *d_kl64, *d_koff;
    char* d_kbytes;
    TRY(A.get(&d_kitem, n_keys));
    TRY(A.get(&d_kl64, n_keys + 1));
    TRY(A.get(&d_koff, n_keys + 1));
    // key order key = (length << 40) | row: the item is the row
    hipLaunchKernelGGL(k_rank_items, blocks(n_keys + 1), dim3(256), 0, nullptr, d_koks, n_keys, kKeyLenBit - 1, d_kl, 1u,
                       d_kitem, d_kl64);
    TRY(excl_scan(d_kl64, d_koff, n_keys + 1, tmp));
    uint64_t kchars = 0;
    TRY(hipMemcpy(&kchars, d_koff + n_keys, sizeof(uint64_t), hipMemcpyDeviceToHost));
    TRY(A.get(&d_kbytes, std::max<uint64_t>(kchars, 1) * cs));
    hipLaunchKernelGGL(k_layout<CharT>, blocks(n_keys), dim3(256), 0, nullptr, d_kitem, n_keys, d_blob, d_rowoff, d_ka,
                       d_kl, d_koff, reinterpret_cast<CharT*>(d_kbytes), true);
    TRY(hipGetLastError());

    // ---- 3b. term ids: by (long?, first word) or (long?, best key rank, first word) ----
    uint64_t *d_ok, *d_oks;
    uint32_t *d_ov, *d_ovs, *d_rank, *d_nshort, *d_term_of_word;
    TRY(A.get(&d_ok, n_terms));
    TRY(A.get(&d_oks, n_terms));
    TRY(A.get(&d_ov, n_terms));
    TRY(A.get(&d_ovs, n_terms));
    TRY(A.get(&d_rank, n_terms));
    TRY(A.get(&d_nshort, 1));
    TRY(A.get(&d_term_of_word, size));
    uint32_t* d_minr;
    TRY(A.get(&d_minr, n_terms));
    const bool by_rank = term_order_by_rank();
    TRY(hipMemset(d_minr, by_rank ? 0xFF : 0, n_terms * sizeof(uint32_t)));
    if (by_rank)
        hipLaunchKernelGGL(k_term_minrank, blocks(V_n), dim3(256), 0, nullptr, d_sj, d_seg, V_n, (uint32_t)rowSize,
                           d_key_of_row, d_minr);
    hipLaunchKernelGGL(k_term_order, blocks(n_terms), dim3(256), 0, nullptr, d_sj, d_hpos, n_terms, d_tlen,
                       ix.short_term_len, d_minr, d_ok, d_ov);
    TRY(sort_pairs(d_ok, d_oks, d_ov, d_ovs, n_terms, 64, tmp));
    TRY(hipMemcpy(d_nshort, &n_terms, sizeof(uint32_t), hipMemcpyHostToDevice));  // all short unless a long one is found
    hipLaunchKernelGGL(k_ranks, blocks(n_terms), dim3(256), 0, nullptr, d_oks, d_ovs, n_terms, kTermLongBit, d_rank,
                       d_nshort);
    hipLaunchKernelGGL(k_item_rank, blocks(V_n), dim3(256), 0, nullptr, d_sj, d_seg, d_rank, V_n, d_term_of_word);
    // term layout: lengths by id -> offsets -> characters
    uint32_t* d_titem;
    uint64_t *d_tl64, *d_toff;
    char* d_tbytes;
    TRY(A.get(&d_titem, n_terms));
    TRY(A.get(&d_tl64, n_terms + 1));
    TRY(A.get(&d_toff, n_terms + 1));
    hipLaunchKernelGGL(k_rank_items, blocks(n_terms + 1), dim3(256), 0, nullptr, d_oks, n_terms, kTermItemMask, d_tlen,
                       0u, d_titem, d_tl64);
    TRY(excl_scan(d_tl64, d_toff, n_terms + 1, tmp));
    uint64_t tchars = 0;
    TRY(hipMemcpy(&tchars, d_toff + n_terms, sizeof(uint64_t), hipMemcpyDeviceToHost));
    TRY(A.get(&d_tbytes, std::max<uint64_t>(tchars, 1) * cs));
    hipLaunchKernelGGL(k_layout<CharT>, blocks(n_terms), dim3(256), 0, nullptr, d_titem, n_terms, d_nblob, d_woff,
                       (const uint32_t*)nullptr, d_tlen, d_toff, reinterpret_cast<CharT*>(d_tbytes), false);
    TRY(hipGetLastError());

    // ---- 5. pairs ----
    uint64_t *d_pk, *d_pks;
    uint32_t *d_pj, *d_phead, *d_pseg, *d_phpos;
    TRY(A.get(&d_pk, V_n));
    TRY(A.get(&d_pks, V_n));
    TRY(A.get(&d_pj, V_n));
    TRY(A.get(&d_phead, V_n + 1));
    TRY(A.get(&d_pseg, V_n + 1));
    TRY(A.get(&d_phpos, V_n + 1));
    hipLaunchKernelGGL(k_pair_keys, blocks(V_n), dim3(256), 0, nullptr, d_vj, V_n, (uint32_t)rowSize, d_term_of_word,
                       d_key_of_row, d_pk);
    TRY(sort_pairs(d_pk, d_pks, d_vj, d_pj, V_n, 64, tmp));
    uint32_t n_pairs = 0;
    TRY(runs_of(d_pks, V_n, d_phead, d_pseg, d_phpos, tmp, nullptr, n_pairs));
    uint64_t *d_dk, *d_dks;
    uint32_t *d_dv, *d_dvs, *d_tkoff, *d_word;
    uint2 *d_dp, *d_tk;
    float* d_wild;
    TRY(A.get(&d_dk, n_pairs));
    TRY(A.get(&d_dks, n_pairs));
    TRY(A.get(&d_dv, n_pairs));
    TRY(A.get(&d_dvs, n_pairs));
    TRY(A.get(&d_dp, n_pairs));
    TRY(A.get(&d_tk, n_pairs));
    TRY(A.get(&d_tkoff, n_terms + 1));
    TRY(A.get(&d_word, n_keys));
    TRY(A.get(&d_wild, n_keys));
    hipLaunchKernelGGL(k_pair_runs, blocks(V_n), dim3(256), 0, nullptr, d_pks, d_pj, d_phead, d_pseg, V_n, d_w, d_dk, d_dv,
                       d_dp);
    TRY(sort_pairs(d_dk, d_dks, d_dv, d_dvs, n_pairs, 64, tmp));
    TRY(hipMemset(d_word, 0, n_keys * sizeof(uint32_t)));
    TRY(hipMemcpy(d_tkoff + n_terms, &n_pairs, sizeof(uint32_t), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_tk, blocks(n_pairs), dim3(256), 0, nullptr, d_dks, d_dvs, d_dp, n_pairs, d_tk, d_tkoff, d_word);
    hipLaunchKernelGGL(k_unord, blocks(n_keys), dim3(256), 0, nullptr, d_word, n_keys, d_wild);
    TRY(hipGetLastError());

    uint32_t err = 0, n_short = 0;
    TRY(hipMemcpy(&err, d_err, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (err) return hipErrorNotSupported;  // hash collision or NaN weight: the host build decides
    TRY(hipMemcpy(&n_short, d_nshort, sizeof(uint32_t), hipMemcpyDeviceToHost));

    pt.mark("intern: GPU phases");
    // ---- 6. to the host index ----
    ix.n_terms = n_terms;
    ix.n_short = n_short;
    ix.n_keys = n_keys;
    TRY(download(ix.term_off, d_toff, (size_t)n_terms + 1));
    TRY(download(ix.term_bytes, reinterpret_cast<const uint8_t*>(d_tbytes), tchars * cs));
    TRY(download(ix.tk_off, d_tkoff, (size_t)n_terms + 1));
    TRY(download(ix.tk, d_tk, n_pairs));
    TRY(download(ix.key_off, d_koff, (size_t)n_keys + 1));
    TRY(download(ix.key_bytes, reinterpret_cast<const char*>(d_kbytes), kchars * cs));
    TRY(download(ix.wild_w, d_wild, n_keys));
    pt.mark("intern: arrays to host");
    return hipSuccess;
}

}  // namespace

hipError_t intern_device(HostIndex& ix, const void* const* words, uint64_t size, uint16_t rowSize,
                         const float* weight, uint32_t g) {
    if (ix.csize == 4)
        return intern_impl<uint32_t>(ix, reinterpret_cast<const uint32_t* const*>(words), size, rowSize, weight, g);
    return intern_impl<uint8_t>(ix, reinterpret_cast<const uint8_t* const*>(words), size, rowSize, weight, g);
}

}  // namespace ngs
