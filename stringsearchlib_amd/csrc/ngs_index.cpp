// ngs_index.cpp — host index build (see ngs_index.h). Paths cited relative to /root/reference.
#include "ngs_index.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace ngs {
namespace {

// NGS_BUILD_TIMING=1 prints the host build phases to stderr
struct PhaseTimer {
    bool on = std::getenv("NGS_BUILD_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngs build] %-22s %8.3f s\n", what, std::chrono::duration<double>(n - t).count());
        t = n;
    }
};

// nGramSearch.h:307-313
constexpr char kDefaultValid[] = ".%$ @0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ";

inline bool is_space(unsigned c) { return c == ' ' || (c >= 9 && c <= 13); }  // C-locale isspace
inline unsigned to_upper(unsigned c) { return (c >= 'a' && c <= 'z') ? c - 32u : c; }

inline uint64_t hash_str(const uint8_t* p, uint32_t n) {
    uint64_t h = 0x243F6A8885A308D3ull ^ n;
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v;
        std::memcpy(&v, p + i, 8);
        h = (h ^ v) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 32;
    }
    uint64_t t = 0;
    for (; i < n; ++i) t = (t << 8) | p[i];
    h = (h ^ t) * 0xD6E8FEB86659FD93ull;
    return h ^ (h >> 29);
}

// String interning in first-insertion order (ids 0..n-1), open addressing.
class Interner {
public:
    Interner() : slots_(1 << 12, 0) {}
    uint32_t intern(const uint8_t* p, uint32_t n) {
        if ((size_t)(len_.size() + 1) * 2 > slots_.size()) grow();
        uint64_t h = hash_str(p, n);
        size_t mask = slots_.size() - 1, i = h & mask;
        for (;;) {
            uint32_t s = slots_[i];
            if (!s) break;
            uint32_t id = s - 1;
            if (hash_[id] == h && len_[id] == n && std::memcmp(blob_.data() + off_[id], p, n) == 0) return id;
            i = (i + 1) & mask;
        }
        uint32_t id = (uint32_t)len_.size();
        off_.push_back(blob_.size());
        len_.push_back(n);
        hash_.push_back(h);
        blob_.insert(blob_.end(), p, p + n);
        slots_[i] = id + 1;
        return id;
    }
    uint32_t size() const { return (uint32_t)len_.size(); }
    const uint8_t* str(uint32_t id) const { return blob_.data() + off_[id]; }
    uint32_t len(uint32_t id) const { return len_[id]; }
    size_t bytes() const { return blob_.size(); }

private:
    void grow() {
        std::vector<uint32_t> s(slots_.size() * 2, 0);
        size_t mask = s.size() - 1;
        for (uint32_t id = 0; id < len_.size(); ++id) {
            size_t i = hash_[id] & mask;
            while (s[i]) i = (i + 1) & mask;
            s[i] = id + 1;
        }
        slots_.swap(s);
    }
    std::vector<uint32_t> slots_;
    std::vector<uint8_t> blob_;
    std::vector<uint64_t> off_, hash_;
    std::vector<uint32_t> len_;
};

struct Pair { uint32_t term, key; float w; };

// escapeBlank (h:93-98) -> trim (h:243-247) -> toUpper (h:72-76); returns the length.
inline uint32_t normalise_term(const bool* valid, const uint8_t* p, uint32_t n, uint8_t* out) {
    uint32_t a = 0, b = n;
    while (a < b && is_space(valid[p[a]] ? p[a] : ' ')) ++a;
    while (b > a && is_space(valid[p[b - 1]] ? p[b - 1] : ' ')) --b;
    for (uint32_t i = a; i < b; ++i) out[i - a] = (uint8_t)to_upper(valid[p[i]] ? p[i] : ' ');
    return b - a;
}

inline uint32_t gram_code(const uint8_t* s) { return ((uint32_t)s[0] << 14) | ((uint32_t)s[1] << 7) | s[2]; }

// Distinct grams of one term (ngrams[h].insert(id) deduplicates per term, hpp:13-21).
inline uint32_t term_grams(const uint8_t* s, uint32_t L, uint32_t* g) {
    uint32_t n = 0;
    for (uint32_t i = 0; i + 2 < L; ++i)
        if (!((s[i] | s[i + 1] | s[i + 2]) & 0x80)) g[n++] = gram_code(s + i);  // terms are ASCII
    std::sort(g, g + n);
    return (uint32_t)(std::unique(g, g + n) - g);
}

}  // namespace

void build_index(HostIndex& ix, char* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                 unsigned threads) {
    ix = HostIndex();
    ix.gram_off.assign((size_t)kGramSpace + 1, 0);
    ix.term_off.assign(1, 0);
    ix.tk_off.assign(1, 0);
    ix.key_off.assign(1, 0);
    // nGramSearch.hpp:122-123: no library -> un-built index (searches answer 0). rowSize 0 would
    // loop forever in the reference (hpp:126); it is refused the same way.
    if (size < 2 || !words || rowSize == 0) return;

    bool valid[256] = {};
    for (const char* c = kDefaultValid; *c; ++c) valid[(uint8_t)*c] = true;
    PhaseTimer pt;

    Interner terms, keys;
    std::vector<Pair> pairs;
    pairs.reserve(size);
    std::vector<uint8_t> scratch(256);
    for (uint64_t i = 0; i < size; i += rowSize) {                        // hpp:126
        if (!words[i]) continue;                                          // hpp:129
        const uint8_t* raw = (const uint8_t*)words[i];
        uint32_t n = (uint32_t)std::strlen(words[i]), a = 0, b = n;
        while (a < b && is_space(raw[a])) ++a;                            // trim(strKey), hpp:132
        while (b > a && is_space(raw[b - 1])) --b;
        if (a == b) continue;                                             // hpp:134
        const uint8_t* key = raw + a;
        const uint32_t klen = b - a;
        uint32_t kid = UINT32_MAX;
        const uint64_t row_end = std::min<uint64_t>(i + rowSize, size);   // hpp:150 (clamped)
        for (uint64_t j = i; j < row_end; ++j) {
            if (!words[j]) continue;
            const uint8_t* src = j == i ? key : (const uint8_t*)words[j];
            uint32_t sl = j == i ? klen : (uint32_t)std::strlen(words[j]);
            if (sl > scratch.size()) scratch.resize(sl * 2);
            uint32_t tl = normalise_term(valid, src, sl, scratch.data()); // hpp:136-139, :153-156
            if (j != i && tl == 0) continue;                              // hpp:157; a key's own term may be ""
            float w = weight ? weight[j] : 1.0f;                          // hpp:141-143, :159-161
            if (w == 0.0f) continue;                                      // hpp:144, :162
            if (kid == UINT32_MAX) kid = keys.intern(key, klen);
            pairs.push_back({terms.intern(scratch.data(), tl), kid, w});  // hpp:146-147, :164-165
        }
    }

    pt.mark("parse+intern");
    // (term, key) -> weight, last write wins (tempWeightMap[term][key] = w)
    {
        size_t hs = 16;
        while (hs < pairs.size() * 2) hs <<= 1;
        std::vector<uint64_t> hk(hs, ~0ull);
        std::vector<uint32_t> hv(hs);
        size_t nu = 0;
        for (size_t p = 0; p < pairs.size(); ++p) {
            uint64_t k = ((uint64_t)pairs[p].term << 32) | pairs[p].key;
            size_t h = (size_t)((k * 0x9E3779B97F4A7C15ull) >> 17) & (hs - 1);
            while (hk[h] != ~0ull && hk[h] != k) h = (h + 1) & (hs - 1);
            if (hk[h] == k) {
                pairs[hv[h]].w = pairs[p].w;
            } else {
                hk[h] = k;
                hv[h] = (uint32_t)nu;
                pairs[nu++] = pairs[p];
            }
        }
        pairs.resize(nu);
    }

    pt.mark("pair dedup");
    // key ranks: stable counting sort by length keeps first appearance within a length
    ix.n_keys = keys.size();
    std::vector<uint32_t> krank(ix.n_keys);
    {
        uint32_t maxlen = 0;
        for (uint32_t k = 0; k < ix.n_keys; ++k) maxlen = std::max(maxlen, keys.len(k));
        std::vector<uint32_t> cnt((size_t)maxlen + 2, 0);
        for (uint32_t k = 0; k < ix.n_keys; ++k) cnt[keys.len(k) + 1]++;
        for (size_t l = 1; l < cnt.size(); ++l) cnt[l] += cnt[l - 1];
        std::vector<uint32_t> order(ix.n_keys);
        for (uint32_t k = 0; k < ix.n_keys; ++k) {
            krank[k] = cnt[keys.len(k)]++;
            order[krank[k]] = k;
        }
        ix.key_off.resize((size_t)ix.n_keys + 1);
        ix.key_bytes.resize(keys.bytes() + ix.n_keys);
        uint64_t o = 0;
        for (uint32_t r = 0; r < ix.n_keys; ++r) {
            uint32_t k = order[r];
            ix.key_off[r] = o;
            std::memcpy(ix.key_bytes.data() + o, keys.str(k), keys.len(k));
            o += keys.len(k);
            ix.key_bytes[o++] = 0;
        }
        ix.key_off[ix.n_keys] = o;
    }

    // term ids: shortLib first (hpp:82-85), each class in first-appearance order
    ix.n_terms = terms.size();
    std::vector<uint32_t> tmap(ix.n_terms);
    {
        uint32_t s = 0;
        for (uint32_t t = 0; t < ix.n_terms; ++t)
            if (terms.len(t) < kShortTermLen) tmap[t] = s++;
        ix.n_short = s;
        for (uint32_t t = 0; t < ix.n_terms; ++t)
            if (terms.len(t) >= kShortTermLen) tmap[t] = s++;
        std::vector<uint32_t> inv(ix.n_terms);
        for (uint32_t t = 0; t < ix.n_terms; ++t) inv[tmap[t]] = t;
        ix.term_off.resize((size_t)ix.n_terms + 1);
        ix.term_bytes.resize(terms.bytes());
        uint64_t o = 0;
        for (uint32_t r = 0; r < ix.n_terms; ++r) {
            uint32_t t = inv[r];
            ix.term_off[r] = o;
            std::memcpy(ix.term_bytes.data() + o, terms.str(t), terms.len(t));
            o += terms.len(t);
        }
        ix.term_off[ix.n_terms] = o;
    }

    pt.mark("keys+terms layout");
    // term -> (key rank, weight) CSR; wildcard weight per key (max of its pairs)
    ix.tk_off.assign((size_t)ix.n_terms + 1, 0);
    for (const Pair& p : pairs) ix.tk_off[tmap[p.term] + 1]++;
    for (uint32_t t = 0; t < ix.n_terms; ++t) ix.tk_off[t + 1] += ix.tk_off[t];
    ix.tk.resize(pairs.size());
    ix.wild_w.assign(ix.n_keys, 0.0f);
    {
        std::vector<uint32_t> fill(ix.tk_off.begin(), ix.tk_off.end() - 1);
        std::vector<uint8_t> seen(ix.n_keys, 0);
        for (const Pair& p : pairs) {
            uint32_t k = krank[p.key];
            uint32_t wb;
            std::memcpy(&wb, &p.w, 4);
            ix.tk[fill[tmap[p.term]]++] = make_uint2(k, wb);
            if (!seen[k] || p.w > ix.wild_w[k]) ix.wild_w[k] = p.w;
            seen[k] = 1;
        }
    }
    std::vector<Pair>().swap(pairs);

    pt.mark("term->key CSR");
    // gram CSR over longLib, two passes, term-range parallel (postings stay sorted by term id)
    const uint32_t n_long = ix.n_terms - ix.n_short;
    if (!threads) threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    threads = std::max(1u, std::min<unsigned>(threads, n_long / 4096 + 1));
    std::vector<std::vector<uint32_t>> counts(threads, std::vector<uint32_t>(kGramSpace, 0));
    auto range = [&](unsigned t, uint32_t& b, uint32_t& e) {
        b = ix.n_short + (uint32_t)((uint64_t)n_long * t / threads);
        e = ix.n_short + (uint32_t)((uint64_t)n_long * (t + 1) / threads);
    };
    auto run = [&](auto&& body) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < threads; ++t) th.emplace_back(body, t);
        for (auto& x : th) x.join();
    };
    run([&](unsigned t) {
        uint32_t b, e;
        range(t, b, e);
        std::vector<uint32_t> g(64);
        uint32_t* c = counts[t].data();
        for (uint32_t id = b; id < e; ++id) {
            uint32_t L = (uint32_t)(ix.term_off[id + 1] - ix.term_off[id]);
            if (L > g.size()) g.resize(L);
            uint32_t n = term_grams(ix.term_bytes.data() + ix.term_off[id], L, g.data());
            for (uint32_t i = 0; i < n; ++i) c[g[i]]++;
        }
    });
    {
        uint64_t o = 0;
        for (uint32_t g = 0; g < kGramSpace; ++g) {
            ix.gram_off[g] = o;
            uint64_t tot = 0;
            for (unsigned t = 0; t < threads; ++t) {
                uint32_t c = counts[t][g];
                counts[t][g] = (uint32_t)(o + tot);  // becomes this thread's write cursor
                tot += c;
            }
            ix.n_grams += tot != 0;
            o += tot;
        }
        ix.gram_off[kGramSpace] = o;
        ix.post.resize(o);
    }
    run([&](unsigned t) {
        uint32_t b, e;
        range(t, b, e);
        std::vector<uint32_t> g(64);
        uint32_t* cur = counts[t].data();
        for (uint32_t id = b; id < e; ++id) {
            uint32_t L = (uint32_t)(ix.term_off[id + 1] - ix.term_off[id]);
            if (L > g.size()) g.resize(L);
            uint32_t n = term_grams(ix.term_bytes.data() + ix.term_off[id], L, g.data());
            for (uint32_t i = 0; i < n; ++i) ix.post[cur[g[i]]++] = id - ix.n_short;
        }
    });
    counts.clear();

    pt.mark("gram CSR");
    // bucket skip table: for every non-empty list, the offset of its first posting in each of
    // K equal term-id buckets. Lets a query cut its lists into term-id parts with one load per
    // (gram, bucket) instead of a binary search (DESIGN.md §Index layout).
    ix.n_buckets = 1;
    while (ix.n_buckets < kMaxBuckets && (uint64_t)ix.n_buckets * kMinBucketTerms < n_long) ix.n_buckets <<= 1;
    ix.bucket_span = n_long ? (n_long + ix.n_buckets - 1) / ix.n_buckets : 1;
    ix.gram_row.assign(kGramSpace, UINT32_MAX);
    std::vector<uint32_t> rows;
    for (uint32_t g = 0; g < kGramSpace; ++g)
        if (ix.gram_off[g + 1] > ix.gram_off[g]) {
            ix.gram_row[g] = (uint32_t)rows.size();
            rows.push_back(g);
        }
    const uint32_t K = ix.n_buckets;
    ix.skip.assign((size_t)rows.size() * (K + 1), 0);
    run([&](unsigned t) {
        for (size_t r = t; r < rows.size(); r += threads) {
            const uint32_t g = rows[r];
            const uint32_t* p = ix.post.data() + ix.gram_off[g];
            const uint32_t len = (uint32_t)(ix.gram_off[g + 1] - ix.gram_off[g]);
            uint32_t* out = ix.skip.data() + r * (K + 1);
            uint32_t i = 0;
            for (uint32_t b = 0; b <= K; ++b) {
                const uint64_t lo = (uint64_t)b * ix.bucket_span;
                while (i < len && p[i] < lo) ++i;
                out[b] = i;
            }
            out[K] = len;
        }
    });
    pt.mark("skip table");
    ix.indexed = true;                                                    // hpp:45
}

void wildcard_order(const HostIndex& ix, std::vector<uint32_t>& keys, std::vector<float>& scores) {
    keys.resize(ix.n_keys);
    for (uint32_t k = 0; k < ix.n_keys; ++k) keys[k] = k;
    std::stable_sort(keys.begin(), keys.end(),
                     [&](uint32_t a, uint32_t b) { return ix.wild_w[a] > ix.wild_w[b]; });
    scores.resize(ix.n_keys);
    for (uint32_t i = 0; i < ix.n_keys; ++i) scores[i] = ix.wild_w[keys[i]];
}

}  // namespace ngs
