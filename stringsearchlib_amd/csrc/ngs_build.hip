// ngs_build.hip — the index's gram CSR, gram dictionary and skip table built on the GPU.
//
// Reference: the gram index of nGramSearch.hpp:13-21 (getGrams(id): ngrams[h].insert(id), a
// per-gram hash SET, so a term is listed once per distinct gram) and :41-46 (buildGrams over
// longLib, terms of >= 6 bytes, hpp:82-85). The host build (ngs_index.cpp) restates it with
// threads; this is the same layout from the normalised terms already in HBM:
//   1. k_gram_count   one thread per long term: its distinct 21-bit gram codes (count)
//   2. scan           exclusive prefix of the counts -> each term's slice of the pair array
//   3. k_gram_emit    pairs (code << 32 | long-term id)
//   4. radix sort     by (code, term): lists come out sorted by term id, as the kernels need
//   5. k_gram_runs    run boundaries per code -> counts -> scan -> gram_off (u64, 2^21 + 1)
//   6. rows           gram -> skip-table row for the non-empty lists (gram_row)
//   7. k_skip         per (row, bucket): lower_bound of the bucket's first term id (skip)
// Dictionary mode (every shape but narrow 3-grams: indexG, indexW): a gram is the key of its g
// characters, 21 bits each (ngs_index.cpp gram_key), and its id the key's rank among the long
// terms' distinct keys. gram_keys_device finds those keys (k_dict_terms emits each term's
// distinct keys, radix sort, unique); the host lays out its lookup table from them
// (set_gram_dict); then steps 1-7 run with ids found by binary search over the keys in place of
// the 21-bit codes, G = the number of keys.
// Everything is bit-identical to the host build (tests/test_gpu_build.py compares digests).
#include <hipcub/hipcub.hpp>

#include "ngs_build.h"

namespace ngs {
namespace {

__device__ __forceinline__ uint32_t code3(const uint8_t* s) { return ((uint32_t)s[0] << 14) | ((uint32_t)s[1] << 7) | s[2]; }
__device__ __forceinline__ bool ascii3(const uint8_t* s) { return !((s[0] | s[1] | s[2]) & 0x80); }

// Distinct grams of long term t (ids n_short + t): the first occurrence of each code counts
// (terms are ASCII; a gram with a byte >= 0x80 is skipped as in term_grams()).
template <bool EMIT>
__global__ __launch_bounds__(256) void k_gram_terms(const uint64_t* __restrict__ term_off,
                                                    const uint8_t* __restrict__ bytes, uint32_t n_short,
                                                    uint32_t n_long, uint64_t* __restrict__ cnt,
                                                    const uint64_t* __restrict__ off, uint64_t* __restrict__ pairs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_long) return;
    const uint64_t a = term_off[n_short + t], L = term_off[n_short + t + 1] - a;
    const uint8_t* s = bytes + a;
    uint32_t n = 0;
    uint64_t o = EMIT ? off[t] : 0;
    for (uint64_t i = 0; i + 2 < L; ++i) {
        if (!ascii3(s + i)) continue;
        const uint32_t c = code3(s + i);
        bool first = true;
        for (uint64_t j = 0; j < i && first; ++j) first = !(ascii3(s + j) && code3(s + j) == c);
        if (!first) continue;
        if (EMIT) pairs[o++] = ((uint64_t)c << 32) | t;
        ++n;
    }
    if (!EMIT) cnt[t] = n;
}

// dictionary mode: the key of the g characters at character a (cs bytes each)
__device__ __forceinline__ uint64_t gram_key_at(const uint8_t* b, uint64_t a, uint32_t g, uint32_t cs) {
    uint64_t k = 0;
    for (uint32_t j = 0; j < g; ++j)
        k = (k << 21) | (cs == 1 ? (uint32_t)b[a + j] : reinterpret_cast<const uint32_t*>(b)[a + j]);
    return k;
}

// Dictionary mode, one thread per long term, over its distinct gram keys (first occurrences):
// MODE 0 counts them, 1 writes the keys at off[t], 2 writes (id << 32 | t) with id the key's rank
// in dict[0 .. nspace).
template <int MODE>
__global__ __launch_bounds__(256) void k_dict_terms(const uint64_t* __restrict__ term_off,
                                                    const uint8_t* __restrict__ bytes, uint32_t n_short,
                                                    uint32_t n_long, uint32_t cs, uint32_t g,
                                                    uint64_t* __restrict__ cnt, const uint64_t* __restrict__ off,
                                                    uint64_t* __restrict__ out, const uint64_t* __restrict__ dict,
                                                    uint32_t nspace) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_long) return;
    const uint64_t a = term_off[n_short + t], L = term_off[n_short + t + 1] - a;
    uint32_t n = 0;
    uint64_t o = MODE ? off[t] : 0;
    for (uint64_t i = 0; i + g <= L; ++i) {
        const uint64_t k = gram_key_at(bytes, a + i, g, cs);
        bool first = true;
        for (uint64_t j = 0; j < i && first; ++j) first = gram_key_at(bytes, a + j, g, cs) != k;
        if (!first) continue;
        if (MODE == 1) out[o++] = k;
        if (MODE == 2) {
            uint32_t lo = 0, hi = nspace;  // lower_bound: the key is present
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (dict[m] < k) lo = m + 1; else hi = m;
            }
            out[o++] = ((uint64_t)lo << 32) | t;
        }
        ++n;
    }
    if (MODE == 0) cnt[t] = n;
}

// Run boundaries of the sorted pairs: first / one-past-last index of every code present.
__global__ __launch_bounds__(256) void k_gram_runs(const uint64_t* __restrict__ pairs, uint64_t P,
                                                   uint64_t* __restrict__ gstart, uint64_t* __restrict__ gend,
                                                   uint32_t* __restrict__ post) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint64_t k = pairs[i];
    const uint32_t g = (uint32_t)(k >> 32);
    post[i] = (uint32_t)k;
    if (i == 0 || (uint32_t)(pairs[i - 1] >> 32) != g) gstart[g] = i;
    if (i + 1 == P || (uint32_t)(pairs[i + 1] >> 32) != g) gend[g] = i + 1;
}

__global__ __launch_bounds__(256) void k_gram_len(const uint64_t* __restrict__ gstart, const uint64_t* __restrict__ gend,
                                                  uint64_t* __restrict__ len, uint32_t* __restrict__ nonempty,
                                                  uint32_t n) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint64_t l = gend[g] - gstart[g];
    len[g] = l;
    nonempty[g] = l != 0;
}

__global__ __launch_bounds__(256) void k_gram_rows(const uint32_t* __restrict__ nonempty,
                                                   const uint32_t* __restrict__ rank, uint32_t n,
                                                   uint32_t* __restrict__ gram_row, uint32_t* __restrict__ row_gram) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    if (nonempty[g]) {
        gram_row[g] = rank[g];
        row_gram[rank[g]] = g;
    } else {
        gram_row[g] = UINT32_MAX;
    }
}

// skip[row][b] = offset in the row's list of the first posting >= b * span (b = K: the length)
__global__ __launch_bounds__(256) void k_skip(const uint64_t* __restrict__ gram_off, const uint32_t* __restrict__ post,
                                              const uint32_t* __restrict__ row_gram, uint32_t rows, uint32_t K,
                                              uint32_t span, uint32_t* __restrict__ skip) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)rows * (K + 1)) return;
    const uint32_t r = (uint32_t)(i / (K + 1)), b = (uint32_t)(i - (uint64_t)r * (K + 1));
    const uint32_t g = row_gram[r];
    const uint32_t* p = post + gram_off[g];
    const uint32_t len = (uint32_t)(gram_off[g + 1] - gram_off[g]);
    uint32_t out = len;
    if (b < K) {
        const uint64_t lo = (uint64_t)b * span;
        uint32_t a = 0, e = len;
        while (a < e) {
            const uint32_t m = (a + e) >> 1;
            if (p[m] < lo) a = m + 1; else e = m;
        }
        out = a;
    }
    skip[i] = out;
}

inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + 255) / 256); }

}  // namespace

#define TRY(x)                                   \
    do {                                         \
        if ((e = (x)) != hipSuccess) goto done;  \
    } while (0)

hipError_t build_grams_device(const uint64_t* term_off, const uint8_t* term_bytes, uint32_t n_short,
                              uint32_t n_terms, DeviceGrams& out, const uint64_t* dict, uint32_t nspace, uint32_t cs,
                              uint32_t g) {
    hipError_t e = hipSuccess;
    const uint32_t n_long = n_terms - n_short, G = dict ? nspace : (uint32_t)kGramSpace;
    // sort width: the gram field above the 32-bit term id
    const int gbits = dict ? (nspace > 1 ? 32 - __builtin_clz(nspace - 1) : 1) : kGramBits;
    uint32_t *nonempty = nullptr, *rank = nullptr, *row_gram = nullptr;
    uint64_t* cnt = nullptr;
    uint64_t *off = nullptr, *pairs = nullptr, *sorted = nullptr, *gstart = nullptr, *gend = nullptr, *len = nullptr;
    uint64_t *d_total = nullptr, *d_max = nullptr;
    uint32_t* d_rows = nullptr;
    void* temp = nullptr;
    size_t tb = 0, need = 0;
    uint64_t P = 0, max_len = 0;
    uint32_t rows = 0;
    hipStream_t s = nullptr;
    out = DeviceGrams{};
    TRY(hipMalloc(&out.gram_off, sizeof(uint64_t) * (G + 1)));
    TRY(hipMalloc(&out.gram_row, sizeof(uint32_t) * (G + 1)));
    TRY(hipMalloc(&cnt, sizeof(uint64_t) * (n_long + 1)));
    TRY(hipMalloc(&off, sizeof(uint64_t) * (n_long + 1)));
    TRY(hipMalloc(&d_total, sizeof(uint64_t) * 2));
    d_max = d_total + 1;
    // 1-2. distinct grams per long term, their slices of the pair array
    if (n_long) {
        if (dict)
            hipLaunchKernelGGL(k_dict_terms<0>, dim3(blocks(n_long)), dim3(256), 0, s, term_off, term_bytes, n_short,
                               n_long, cs, g, cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr, dict, nspace);
        else
            hipLaunchKernelGGL(k_gram_terms<false>, dim3(blocks(n_long)), dim3(256), 0, s, term_off, term_bytes,
                               n_short, n_long, cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr);
        TRY(hipGetLastError());
    }
    TRY(hipMemset(cnt + n_long, 0, sizeof(uint64_t)));
    TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, cnt, off, n_long + 1, s));
    tb = need;
    TRY(hipMalloc(&temp, tb));
    TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb, cnt, off, n_long + 1, s));
    TRY(hipMemcpy(&P, off + n_long, sizeof(uint64_t), hipMemcpyDeviceToHost));
    out.n_post = P;
    TRY(hipMalloc(&out.post, sizeof(uint32_t) * (P + 4)));  // +4: k_wave stages whole 16-byte chunks
    TRY(hipMemset(out.post + P, 0, sizeof(uint32_t) * 4));
    TRY(hipMalloc(&gstart, sizeof(uint64_t) * (G + 1)));
    TRY(hipMalloc(&gend, sizeof(uint64_t) * (G + 1)));
    TRY(hipMemset(gstart, 0, sizeof(uint64_t) * (G + 1)));
    TRY(hipMemset(gend, 0, sizeof(uint64_t) * (G + 1)));
    if (P >= (1ull << 31)) {  // beyond one radix-sort call: the host builds it
        e = hipErrorInvalidValue;
        goto done;
    }
    if (P) {
        // 3-4. pairs, sorted by (code, term): 21 + 32 bits
        TRY(hipMalloc(&pairs, sizeof(uint64_t) * P));
        TRY(hipMalloc(&sorted, sizeof(uint64_t) * P));
        if (dict)
            hipLaunchKernelGGL(k_dict_terms<2>, dim3(blocks(n_long)), dim3(256), 0, s, term_off, term_bytes, n_short,
                               n_long, cs, g, (uint64_t*)nullptr, (const uint64_t*)off, pairs, dict, nspace);
        else
            hipLaunchKernelGGL(k_gram_terms<true>, dim3(blocks(n_long)), dim3(256), 0, s, term_off, term_bytes,
                               n_short, n_long, (uint64_t*)nullptr, (const uint64_t*)off, pairs);
        TRY(hipGetLastError());
        need = 0;
        TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, need, pairs, sorted, (int)P, 0, 32 + gbits, s));
        if (need > tb) {
            TRY(hipFree(temp));
            temp = nullptr;
            tb = need;
            TRY(hipMalloc(&temp, tb));
        }
        TRY(hipcub::DeviceRadixSort::SortKeys(temp, tb, pairs, sorted, (int)P, 0, 32 + gbits, s));
        TRY(hipFree(pairs));
        pairs = nullptr;
        // 5. post and the code -> [start, end) runs
        hipLaunchKernelGGL(k_gram_runs, dim3(blocks(P)), dim3(256), 0, s, sorted, P, gstart, gend, out.post);
        TRY(hipGetLastError());
        TRY(hipFree(sorted));
        sorted = nullptr;
    }
    TRY(hipMalloc(&len, sizeof(uint64_t) * (G + 1)));
    TRY(hipMalloc(&nonempty, sizeof(uint32_t) * (G + 1)));
    TRY(hipMalloc(&rank, sizeof(uint32_t) * (G + 1)));
    if (G) {
        hipLaunchKernelGGL(k_gram_len, dim3(blocks(G)), dim3(256), 0, s, gstart, gend, len, nonempty, G);
        TRY(hipGetLastError());
    }
    TRY(hipMemset(len + G, 0, sizeof(uint64_t)));
    TRY(hipMemset(nonempty + G, 0, sizeof(uint32_t)));
    need = 0;
    TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, len, out.gram_off, G + 1, s));
    {
        size_t n2 = 0, n3 = 0;
        TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, n2, nonempty, rank, G + 1, s));
        TRY(hipcub::DeviceReduce::Max(nullptr, n3, len, d_max, G + 1, s));
        need = std::max(need, std::max(n2, n3));
    }
    if (need > tb) {
        TRY(hipFree(temp));
        temp = nullptr;
        tb = need;
        TRY(hipMalloc(&temp, tb));
    }
    TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb, len, out.gram_off, G + 1, s));
    TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb, nonempty, rank, G + 1, s));
    TRY(hipcub::DeviceReduce::Max(temp, tb, len, d_max, G + 1, s));
    TRY(hipMemcpy(&rows, rank + G, sizeof(uint32_t), hipMemcpyDeviceToHost));
    TRY(hipMemcpy(&max_len, d_max, sizeof(uint64_t), hipMemcpyDeviceToHost));
    out.n_grams = rows;
    // 6. gram -> row
    TRY(hipMalloc(&row_gram, sizeof(uint32_t) * (rows + 1)));
    if (G) {
        hipLaunchKernelGGL(k_gram_rows, dim3(blocks(G)), dim3(256), 0, s, nonempty, rank, G, out.gram_row, row_gram);
        TRY(hipGetLastError());
    }
    // 7. skip table (bucket count: skip_buckets(), the host build's rule)
    skip_buckets(n_long, rows, max_len, out.n_buckets, out.bucket_span);
    TRY(hipMalloc(&out.skip, sizeof(uint32_t) * ((size_t)rows * (out.n_buckets + 1) + 1)));
    if (rows) {
        hipLaunchKernelGGL(k_skip, dim3(blocks((uint64_t)rows * (out.n_buckets + 1))), dim3(256), 0, s, out.gram_off,
                           out.post, row_gram, rows, out.n_buckets, out.bucket_span, out.skip);
        TRY(hipGetLastError());
    }
    TRY(hipDeviceSynchronize());
done:
    for (void* p : {(void*)cnt, (void*)off, (void*)pairs, (void*)sorted, (void*)gstart, (void*)gend, (void*)len,
                    (void*)nonempty, (void*)rank, (void*)row_gram, (void*)d_total, (void*)d_rows, temp})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) {
        for (void* p : {(void*)out.gram_off, (void*)out.gram_row, (void*)out.post, (void*)out.skip})
            if (p) (void)hipFree(p);
        out = DeviceGrams{};
    }
    return e;
}

hipError_t gram_keys_device(const uint64_t* term_off, const uint8_t* term_bytes, uint32_t n_short,
                            uint32_t n_terms, uint32_t cs, uint32_t g, std::vector<uint64_t>& keys) {
    hipError_t e = hipSuccess;
    const uint32_t n_long = n_terms - n_short;
    uint64_t *cnt = nullptr, *off = nullptr, *k = nullptr, *sorted = nullptr;
    int* d_num = nullptr;
    void* temp = nullptr;
    size_t tb = 0, need = 0;
    uint64_t P = 0;
    int num = 0;
    hipStream_t s = nullptr;
    keys.clear();
    TRY(hipMalloc(&cnt, sizeof(uint64_t) * (n_long + 1)));
    TRY(hipMalloc(&off, sizeof(uint64_t) * (n_long + 1)));
    TRY(hipMalloc(&d_num, sizeof(int)));
    if (n_long) {
        hipLaunchKernelGGL(k_dict_terms<0>, dim3(blocks(n_long)), dim3(256), 0, s, term_off, term_bytes, n_short, n_long,
                           cs, g, cnt, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint64_t*)nullptr, 0u);
        TRY(hipGetLastError());
    }
    TRY(hipMemset(cnt + n_long, 0, sizeof(uint64_t)));
    TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, need, cnt, off, n_long + 1, s));
    tb = need;
    TRY(hipMalloc(&temp, std::max<size_t>(tb, 1)));
    TRY(hipcub::DeviceScan::ExclusiveSum(temp, tb, cnt, off, n_long + 1, s));
    TRY(hipMemcpy(&P, off + n_long, sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (P >= (1ull << 31)) {  // beyond one radix-sort call: the host builds it
        e = hipErrorInvalidValue;
        goto done;
    }
    if (P) {
        TRY(hipMalloc(&k, sizeof(uint64_t) * P));
        TRY(hipMalloc(&sorted, sizeof(uint64_t) * P));
        hipLaunchKernelGGL(k_dict_terms<1>, dim3(blocks(n_long)), dim3(256), 0, s, term_off, term_bytes, n_short, n_long,
                           cs, g, (uint64_t*)nullptr, (const uint64_t*)off, k, (const uint64_t*)nullptr, 0u);
        TRY(hipGetLastError());
        need = 0;
        size_t n2 = 0;
        TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, need, k, sorted, (int)P, 0, (int)(21 * g), s));
        TRY(hipcub::DeviceSelect::Unique(nullptr, n2, sorted, k, d_num, (int)P, s));
        need = std::max(need, n2);
        if (need > tb) {
            TRY(hipFree(temp));
            temp = nullptr;
            tb = need;
            TRY(hipMalloc(&temp, tb));
        }
        TRY(hipcub::DeviceRadixSort::SortKeys(temp, tb, k, sorted, (int)P, 0, (int)(21 * g), s));
        TRY(hipcub::DeviceSelect::Unique(temp, tb, sorted, k, d_num, (int)P, s));
        TRY(hipMemcpy(&num, d_num, sizeof(int), hipMemcpyDeviceToHost));
        keys.resize((size_t)num);
        if (num) TRY(hipMemcpy(keys.data(), k, sizeof(uint64_t) * (size_t)num, hipMemcpyDeviceToHost));
    }
done:
    for (void* p : {(void*)cnt, (void*)off, (void*)k, (void*)sorted, (void*)d_num, temp})
        if (p) (void)hipFree(p);
    return e;
}

}  // namespace ngs
