// ngs_index.cpp — host index build (see ngs_index.h). Paths cited relative to /root/reference.
#include "ngs_index.h"

#include "ngs_build.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace ngs {
namespace {


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

inline uint32_t gram_code(const uint8_t* s) { return ((uint32_t)s[0] << 14) | ((uint32_t)s[1] << 7) | s[2]; }

// Distinct grams of one term (ngrams[h].insert(id) deduplicates per term, hpp:13-21).
inline uint32_t term_grams(const uint8_t* s, uint32_t L, uint32_t* g) {
    uint32_t n = 0;
    for (uint32_t i = 0; i + 2 < L; ++i)
        if (!((s[i] | s[i + 1] | s[i + 2]) & 0x80)) g[n++] = gram_code(s + i);  // terms are ASCII
    std::sort(g, g + n);
    return (uint32_t)(std::unique(g, g + n) - g);
}

// ---- character-generic helpers (narrow bytes / wide UTF-32 code points) ----------------
// Wide strings (indexW) normalise code points below 128 exactly as narrow bytes; code points
// from 128 are kept as they are (no escaping, no case mapping), except values above 0x10FFFF,
// which are not code points and become spaces.
template <typename CharT>
inline uint32_t str_len(const CharT* p) {
    uint32_t n = 0;
    while (p[n]) ++n;
    return n;
}
template <typename CharT>
inline uint32_t esc_char(const bool* valid, uint32_t c) {
    if (sizeof(CharT) == 1 || c < 128) return valid[c] ? c : ' ';
    return c > 0x10FFFFu ? ' ' : c;
}
template <typename CharT>
inline bool space_char(uint32_t c) { return c < 128 && is_space(c); }

// escapeBlank (h:93-98) -> trim (h:243-247) -> toUpper (h:72-76); returns the length.
template <typename CharT>
inline uint32_t normalise_t(const bool* valid, const CharT* p, uint32_t n, CharT* out) {
    uint32_t a = 0, b = n;
    while (a < b && space_char<CharT>(esc_char<CharT>(valid, p[a]))) ++a;
    while (b > a && space_char<CharT>(esc_char<CharT>(valid, p[b - 1]))) --b;
    for (uint32_t i = a; i < b; ++i) {
        const uint32_t c = esc_char<CharT>(valid, p[i]);
        out[i - a] = (CharT)(c < 128 ? to_upper(c) : c);
    }
    return b - a;
}

// dictionary-mode gram key: g code points (< 2^21 after normalisation), 21 bits each
template <typename CharT>
inline uint64_t gram_key(const CharT* s, uint32_t g) {
    uint64_t k = 0;
    for (uint32_t j = 0; j < g; ++j) k = (k << 21) | (uint64_t)(uint32_t)s[j];
    return k;
}

// open-addressing set / map of u64 keys (~0 = empty)
struct U64Map {
    std::vector<uint64_t> key;
    std::vector<uint32_t> val;
    uint32_t bits = 0;
    size_t n = 0;
    void init(size_t cap) {
        bits = 4;
        while ((size_t(1) << bits) < cap * 2) ++bits;
        key.assign(size_t(1) << bits, ~0ull);
        val.assign(size_t(1) << bits, 0);
        n = 0;
    }
    size_t slot(uint64_t k) const { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - bits)); }
    bool insert(uint64_t k) {  // true if new
        if ((n + 1) * 2 > key.size()) grow();
        size_t i = slot(k), mask = key.size() - 1;
        while (key[i] != ~0ull) {
            if (key[i] == k) return false;
            i = (i + 1) & mask;
        }
        key[i] = k;
        ++n;
        return true;
    }
    uint32_t find(uint64_t k) const {
        size_t i = slot(k), mask = key.size() - 1;
        while (key[i] != ~0ull) {
            if (key[i] == k) return val[i];
            i = (i + 1) & mask;
        }
        return UINT32_MAX;
    }
    void grow() {
        std::vector<uint64_t> old;
        old.swap(key);
        init(n * 2 + 16);
        for (uint64_t k : old)
            if (k != ~0ull) insert(k);
    }
};

}  // namespace

// The gram CSR over longLib and its skip table (nGramSearch.hpp:13-21, 41-46), from the laid-out
// terms: two passes, term-range parallel (postings stay sorted by term id).
template <typename CharT>
static void build_grams_impl(HostIndex& ix, unsigned threads, PhaseTimer& pt) {
    const uint32_t g = ix.gsz;

    // gram CSR over longLib, two passes, term-range parallel (postings stay sorted by term id)
    const uint32_t n_long = ix.n_terms - ix.n_short;
    if (!threads) threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    threads = std::max(1u, std::min<unsigned>(threads, n_long / 4096 + 1));
    auto range = [&](unsigned t, uint32_t& b, uint32_t& e) {
        b = ix.n_short + (uint32_t)((uint64_t)n_long * t / threads);
        e = ix.n_short + (uint32_t)((uint64_t)n_long * (t + 1) / threads);
    };
    auto run = [&](auto&& body) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < threads; ++t) th.emplace_back(body, t);
        for (auto& x : th) x.join();
    };
    const CharT* tchars = reinterpret_cast<const CharT*>(ix.term_bytes.data());
    // dictionary mode: distinct gram keys -> ids in key order; the device looks them up in an
    // open-addressing table (ghash)
    U64Map dict;
    uint32_t nspace = kGramSpace;
    if (ix.gram_mode == 1) {
        std::vector<U64Map> sets(threads);
        run([&](unsigned t) {
            uint32_t b, e;
            range(t, b, e);
            sets[t].init(1024);
            for (uint32_t id = b; id < e; ++id) {
                const uint32_t L = (uint32_t)(ix.term_off[id + 1] - ix.term_off[id]);
                const CharT* p = tchars + ix.term_off[id];
                for (uint32_t i = 0; i + g <= L; ++i) sets[t].insert(gram_key(p + i, g));
            }
        });
        std::vector<uint64_t> all;
        for (auto& st : sets)
            for (uint64_t k : st.key)
                if (k != ~0ull) all.push_back(k);
        sets.clear();
        std::sort(all.begin(), all.end());
        all.erase(std::unique(all.begin(), all.end()), all.end());
        set_gram_dict(ix, std::move(all));
        nspace = (uint32_t)ix.gram_keys.size();
        dict.key = ix.ghash_key;
        dict.val = ix.ghash_val;
        dict.bits = ix.ghash_bits;
        dict.n = nspace;
    }
    // distinct grams of one long term (ngrams[h].insert(id) deduplicates per term, hpp:13-21)
    auto grams_of = [&](uint32_t id, std::vector<uint32_t>& gv) -> uint32_t {
        const uint32_t L = (uint32_t)(ix.term_off[id + 1] - ix.term_off[id]);
        if (L > gv.size()) gv.resize(L);
        if (ix.gram_mode == 0) return term_grams(ix.term_bytes.data() + ix.term_off[id], L, gv.data());
        const CharT* p = tchars + ix.term_off[id];
        uint32_t n = 0;
        for (uint32_t i = 0; i + g <= L; ++i) gv[n++] = dict.find(gram_key(p + i, g));
        std::sort(gv.begin(), gv.begin() + n);
        return (uint32_t)(std::unique(gv.begin(), gv.begin() + n) - gv.begin());
    };
    ix.gram_off.assign((size_t)nspace + 1, 0);
    std::vector<std::vector<uint32_t>> counts(threads, std::vector<uint32_t>(nspace, 0));
    run([&](unsigned t) {
        uint32_t b, e;
        range(t, b, e);
        std::vector<uint32_t> gv(64);
        uint32_t* c = counts[t].data();
        for (uint32_t id = b; id < e; ++id) {
            uint32_t n = grams_of(id, gv);
            for (uint32_t i = 0; i < n; ++i) c[gv[i]]++;
        }
    });
    {
        uint64_t o = 0;
        for (uint32_t gi = 0; gi < nspace; ++gi) {
            ix.gram_off[gi] = o;
            uint64_t tot = 0;
            for (unsigned t = 0; t < threads; ++t) {
                uint32_t c = counts[t][gi];
                counts[t][gi] = (uint32_t)(o + tot);  // becomes this thread's write cursor
                tot += c;
            }
            ix.n_grams += tot != 0;
            o += tot;
        }
        ix.gram_off[nspace] = o;
        ix.post.resize(o);
    }
    run([&](unsigned t) {
        uint32_t b, e;
        range(t, b, e);
        std::vector<uint32_t> gv(64);
        uint32_t* cur = counts[t].data();
        for (uint32_t id = b; id < e; ++id) {
            uint32_t n = grams_of(id, gv);
            for (uint32_t i = 0; i < n; ++i) ix.post[cur[gv[i]]++] = id - ix.n_short;
        }
    });
    counts.clear();
    pt.mark("gram CSR");
    // bucket skip table: for every non-empty list, the offset of its first posting in each of
    // K equal term-id buckets. Lets a query cut its lists into term-id parts with one load per
    // (gram, bucket) instead of a binary search (DESIGN.md §Index layout).
    ix.gram_row.assign(nspace, UINT32_MAX);
    std::vector<uint32_t> rows;
    uint64_t max_len = 0;
    for (uint32_t gi = 0; gi < nspace; ++gi)
        if (ix.gram_off[gi + 1] > ix.gram_off[gi]) {
            ix.gram_row[gi] = (uint32_t)rows.size();
            rows.push_back(gi);
            max_len = std::max<uint64_t>(max_len, ix.gram_off[gi + 1] - ix.gram_off[gi]);
        }
    // K: up to kMaxBuckets buckets of >= kMinBucketTerms terms; more (a power of two) when the
    // lists are dense, so that the longest list has about kDenseBucketLen postings per bucket and
    // a query's parts stay whole buckets (small gram sizes: 1,369 2-grams over 40M terms), as
    // long as the table stays within kSkipBudget bytes
    skip_buckets(n_long, (uint32_t)rows.size(), max_len, ix.n_buckets, ix.bucket_span);
    const uint32_t K = ix.n_buckets;
    ix.skip.assign((size_t)rows.size() * (K + 1), 0);
    run([&](unsigned t) {
        for (size_t r = t; r < rows.size(); r += threads) {
            const uint32_t gi = rows[r];
            const uint32_t* p = ix.post.data() + ix.gram_off[gi];
            const uint32_t len = (uint32_t)(ix.gram_off[gi + 1] - ix.gram_off[gi]);
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
    ix.grams_built = true;
}

template <typename CharT>
static void build_impl(HostIndex& ix, const CharT* const* words, uint64_t size, uint16_t rowSize,
                       const float* weight, uint32_t g, unsigned threads) {
    ix = HostIndex();
    ix.csize = sizeof(CharT);
    ix.gsz = g;
    ix.gram_mode = (sizeof(CharT) == 1 && g == 3) ? 0u : 1u;
    ix.short_term_len = 2 * g;   // nGramSearch.hpp:82 (6 = 2 x 3)
    ix.short_query_len = 3 * g;  // hpp:381 (9 = 3 x 3)
    ix.full_scan_len = g;        // hpp:235,247,266 (3)
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

    // the interning, key ranks and term -> key CSR on the GPU (ngs_intern.hip), unless
    // NGS_HOST_INTERN is set or it defers to the host (collision, NaN weight, size); same arrays
    if (!std::getenv("NGS_HOST_INTERN")) {
        const hipError_t e = intern_device(ix, reinterpret_cast<const void* const*>(words), size, rowSize, weight, g);
        if (e == hipSuccess) {
            pt.mark("intern + CSR (GPU)");
            ix.indexed = true;  // hpp:45
            ix.grams_built = false;
            if (!std::getenv("NGS_HOST_GRAMS")) return;  // the GPU builds them at upload (ngs_build.hip)
            build_grams_impl<CharT>(ix, threads, pt);
            return;
        }
        (void)hipGetLastError();
        if (e != hipErrorNotSupported) std::fprintf(stderr, "ngram_search: GPU index build failed (%s), building on the host\n", hipGetErrorString(e));
    }

    constexpr uint32_t cs = sizeof(CharT);
    Interner terms, keys;  // interned as raw bytes (cs per character)
    std::vector<Pair> pairs;
    pairs.reserve(size);
    std::vector<CharT> scratch(256);
    for (uint64_t i = 0; i < size; i += rowSize) {                        // hpp:126
        if (!words[i]) continue;                                          // hpp:129
        const CharT* raw = words[i];
        uint32_t n = str_len(raw), a = 0, b = n;
        while (a < b && space_char<CharT>(raw[a])) ++a;                   // trim(strKey), hpp:132
        while (b > a && space_char<CharT>(raw[b - 1])) --b;
        if (a == b) continue;                                             // hpp:134
        const CharT* key = raw + a;
        const uint32_t klen = b - a;
        uint32_t kid = UINT32_MAX;
        const uint64_t row_end = std::min<uint64_t>(i + rowSize, size);   // hpp:150 (clamped)
        for (uint64_t j = i; j < row_end; ++j) {
            if (!words[j]) continue;
            const CharT* src = j == i ? key : words[j];
            uint32_t sl = j == i ? klen : str_len(words[j]);
            if (sl > scratch.size()) scratch.resize(sl * 2);
            uint32_t tl = normalise_t<CharT>(valid, src, sl, scratch.data());  // hpp:136-139, :153-156
            if (j != i && tl == 0) continue;                              // hpp:157; a key's own term may be ""
            float w = weight ? weight[j] : 1.0f;                          // hpp:141-143, :159-161
            if (w == 0.0f) continue;                                      // hpp:144, :162
            if (kid == UINT32_MAX) kid = keys.intern((const uint8_t*)key, klen * cs);
            pairs.push_back({terms.intern((const uint8_t*)scratch.data(), tl * cs), kid, w});  // hpp:146-147, :164-165
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
        // offsets in characters; each key ends with one NUL character
        ix.key_off.resize((size_t)ix.n_keys + 1);
        ix.key_bytes.resize(keys.bytes() + (size_t)ix.n_keys * cs);
        uint64_t o = 0;
        for (uint32_t r = 0; r < ix.n_keys; ++r) {
            uint32_t k = order[r];
            ix.key_off[r] = o;
            std::memcpy(ix.key_bytes.data() + o * cs, keys.str(k), keys.len(k));
            o += keys.len(k) / cs;
            std::memset(ix.key_bytes.data() + o * cs, 0, cs);
            ++o;
        }
        ix.key_off[ix.n_keys] = o;
    }

    // term ids: shortLib first (hpp:82-85), each class in first-appearance order, or by the terms'
    // best key rank first (term_order_by_rank(), ngs_build.h; the reference's ids are internal)
    ix.n_terms = terms.size();
    std::vector<uint32_t> tmap(ix.n_terms);
    {
        std::vector<uint32_t> minrank(ix.n_terms, UINT32_MAX);
        if (term_order_by_rank())
            for (const Pair& p : pairs) minrank[p.term] = std::min(minrank[p.term], krank[p.key]);
        std::vector<uint32_t> ord(ix.n_terms);
        for (uint32_t t = 0; t < ix.n_terms; ++t) ord[t] = t;
        auto is_long = [&](uint32_t t) { return terms.len(t) / cs >= ix.short_term_len; };
        std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
            const bool la = is_long(a), lb = is_long(b);
            if (la != lb) return lb;
            if (minrank[a] != minrank[b]) return minrank[a] < minrank[b];
            return a < b;
        });
        uint32_t s = 0;
        for (uint32_t r = 0; r < ix.n_terms; ++r) {
            tmap[ord[r]] = r;
            if (!is_long(ord[r])) s = r + 1;
        }
        ix.n_short = s;
        std::vector<uint32_t> inv(ix.n_terms);
        for (uint32_t t = 0; t < ix.n_terms; ++t) inv[tmap[t]] = t;
        ix.term_off.resize((size_t)ix.n_terms + 1);
        ix.term_bytes.resize(terms.bytes());
        uint64_t o = 0;
        for (uint32_t r = 0; r < ix.n_terms; ++r) {  // offsets in characters
            uint32_t t = inv[r];
            ix.term_off[r] = o;
            std::memcpy(ix.term_bytes.data() + o * cs, terms.str(t), terms.len(t));
            o += terms.len(t) / cs;
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
    ix.indexed = true;                                                    // hpp:45
    // the GPU builds the gram CSR, the gram dictionary and the skip table at upload
    // (ngs_build.hip) unless NGS_HOST_GRAMS is set
    ix.grams_built = false;
    if (!std::getenv("NGS_HOST_GRAMS")) return;
    build_grams_impl<CharT>(ix, threads, pt);
}

void set_gram_dict(HostIndex& ix, std::vector<uint64_t> sorted_keys) {
    U64Map dict;
    dict.init(sorted_keys.size() + 1);
    for (uint64_t k : sorted_keys) dict.insert(k);  // ascending: the table layout is a function of the key set
    for (size_t i = 0; i < dict.key.size(); ++i)
        if (dict.key[i] != ~0ull)
            dict.val[i] = (uint32_t)(std::lower_bound(sorted_keys.begin(), sorted_keys.end(), dict.key[i]) -
                                     sorted_keys.begin());
    ix.ghash_key = std::move(dict.key);
    ix.ghash_val = std::move(dict.val);
    ix.ghash_bits = dict.bits;
    ix.gram_keys = std::move(sorted_keys);
}

void build_grams_host(HostIndex& ix, unsigned threads) {
    PhaseTimer pt;
    if (ix.csize == 1) build_grams_impl<uint8_t>(ix, threads, pt);
    else build_grams_impl<uint32_t>(ix, threads, pt);
}

void build_index(HostIndex& ix, char* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                 unsigned threads) {
    build_impl<uint8_t>(ix, reinterpret_cast<const uint8_t* const*>(words), size, rowSize, weight, 3, threads);
}

void build_index_g(HostIndex& ix, char* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                   uint32_t gsz, unsigned threads) {
    build_impl<uint8_t>(ix, reinterpret_cast<const uint8_t* const*>(words), size, rowSize, weight, gsz, threads);
}

void build_index_w(HostIndex& ix, const uint32_t* const* words, uint64_t size, uint16_t rowSize,
                   const float* weight, uint32_t gsz, unsigned threads) {
    build_impl<uint32_t>(ix, words, size, rowSize, weight, gsz, threads);
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
