/* ngs_oracle.c — CPU restatement of the reference n-gram search path (plain C11).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py. The product (stringsearchlib_amd/csrc) never links it.
 * Pinned against the reference's own answers (tests/golden, see ngs_oracle.h).
 *
 * Each step cites the reference line it restates (paths relative to /root/reference):
 *   normalisation     nGramSearch.h:30-98 (ltrim/rtrim/toUpper/escapeBlank), validChar :307-313
 *   index build       nGramSearch.hpp:120-172 (ctor), :54-108 (init), :13-21/:41-46 (grams)
 *   gram hash         nGramSearch.h:147-150
 *   long search       nGramSearch.hpp:278-301
 *   short search      nGramSearch.hpp:182-222 (stringMatch), :232-254 (getMatchScore)
 *   calcScore         nGramSearch.hpp:310-341
 *   _search / top-k   nGramSearch.hpp:350-404, ScoreComparer nGramSearch.h:249-270
 *
 * Deterministic refinements where the reference's result depends on unordered_map
 * iteration order (documented in DESIGN.md §Parity):
 *   - ties in (score, key length) are broken by the key's first appearance in the input;
 *   - wildcard ("" / "*", hpp:356-369): a key takes the largest weight of its pairs;
 *   - exact-match promotion (hpp:328-335) sets the key's score to 100, an ordinary score in
 *     ScoreComparer (h:262-269): a key with w*s > 100 ranks above a promoted key, and one at
 *     exactly 100 ties with it on the score and is ordered by length. calcScore runs over the
 *     short scores, then the long ones (hpp:393-394), each in unordered_map order, and a
 *     promotion overwrites what the key had so far while a later pair max-merges over it. The
 *     order inside one group is unspecified; this restatement takes a group's promoting pairs
 *     FIRST: a key's score is max(100, w*s of its other long pairs) when a long pair promotes
 *     it (its short pairs came before and are overwritten), else the max over all its pairs
 *     with a promoting pair counting 100. This agrees with the reference whenever its answer
 *     does not depend on the iteration order; ngo_search_amb reports the queries where it does.
 */
#define _GNU_SOURCE
#include "ngs_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define GRAM_SPACE (1u << 21)
#define SHORT_TERM_LEN 6 /* hpp:82 */
#define SHORT_QUERY_LEN 9 /* hpp:381 */

/* nGramSearch.h:307-313 */
static const char DEFAULT_VALID[] =
    ".%$ @0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ";

static int c_isspace(unsigned c) { return c == ' ' || (c >= 9 && c <= 13); } /* C-locale isspace */
static unsigned c_toupper(unsigned c) { return (c >= 'a' && c <= 'z') ? c - 32u : c; }

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "ngs_oracle: out of memory (%zu)\n", n); abort(); }
    return p;
}
static void* xcalloc(size_t n, size_t s) {
    void* p = calloc(n ? n : 1, s ? s : 1);
    if (!p) { fprintf(stderr, "ngs_oracle: out of memory\n"); abort(); }
    return p;
}
static void* xrealloc(void* p, size_t n) {
    p = realloc(p, n ? n : 1);
    if (!p) { fprintf(stderr, "ngs_oracle: out of memory\n"); abort(); }
    return p;
}

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
/* score encoding: enc = bits(max(w*s, +0)) + 1 (0 = key absent); a promoted key is the score 100 */
#define ENC100 (0x42C80000u + 1u)

/* ------------------------------------------------------------------ interning ---------- */
typedef struct {
    uint8_t* blob; uint64_t blob_len, blob_cap;
    uint64_t* off; uint32_t* len; uint32_t n, cap;
    uint32_t* slot; uint64_t nslot; /* id + 1; 0 = empty */
} strtab;

static uint64_t hash_bytes(const uint8_t* p, uint32_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

static void st_init(strtab* t) { memset(t, 0, sizeof(*t)); t->nslot = 1024; t->slot = xcalloc(t->nslot, 4); }
static void st_free(strtab* t) { free(t->blob); free(t->off); free(t->len); free(t->slot); }

static void st_grow(strtab* t) {
    uint64_t ns = t->nslot * 2;
    uint32_t* s = xcalloc(ns, 4);
    for (uint32_t id = 0; id < t->n; ++id) {
        uint64_t h = hash_bytes(t->blob + t->off[id], t->len[id]) & (ns - 1);
        while (s[h]) h = (h + 1) & (ns - 1);
        s[h] = id + 1;
    }
    free(t->slot); t->slot = s; t->nslot = ns;
}

static uint32_t st_intern(strtab* t, const uint8_t* p, uint32_t n) {
    if ((uint64_t)(t->n + 1) * 2 > t->nslot) st_grow(t);
    uint64_t h = hash_bytes(p, n) & (t->nslot - 1);
    while (t->slot[h]) {
        uint32_t id = t->slot[h] - 1;
        if (t->len[id] == n && memcmp(t->blob + t->off[id], p, n) == 0) return id;
        h = (h + 1) & (t->nslot - 1);
    }
    if (t->n == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 1024;
        t->off = xrealloc(t->off, (size_t)t->cap * 8);
        t->len = xrealloc(t->len, (size_t)t->cap * 4);
    }
    if (t->blob_len + n > t->blob_cap) {
        while (t->blob_len + n > t->blob_cap) t->blob_cap = t->blob_cap ? t->blob_cap * 2 : 65536;
        t->blob = xrealloc(t->blob, t->blob_cap);
    }
    memcpy(t->blob + t->blob_len, p, n);
    t->off[t->n] = t->blob_len; t->len[t->n] = n; t->blob_len += n;
    t->slot[h] = ++t->n;
    return t->n - 1;
}

/* ------------------------------------------------------------------ index ------------- */
struct ngo_index {
    int indexed;
    uint8_t valid[256];
    /* terms: ids [0, n_short) have len < 6 (shortLib), [n_short, n_terms) longLib (hpp:82-85) */
    uint32_t n_terms, n_short;
    uint64_t* term_off; uint8_t* term_bytes; /* normalised term strings */
    uint32_t* tk_off; uint32_t* tk_key; float* tk_w; /* wordMap/wordWeight (h:290,293) */
    uint32_t* kt_off; uint32_t* kt_term;             /* key -> its terms (the pairs, transposed) */
    /* keys ordered by (raw trimmed length, first appearance): the tie refinement */
    uint32_t n_keys;
    uint64_t* key_off; uint8_t* key_bytes;
    float* wild_w; uint32_t* wild_order; /* wildcard answer, precomputed */
    /* gram -> long-term postings, CSR over the 21-bit gram space (ngrams, h:296) */
    uint64_t* gram_off; uint32_t* post; uint64_t n_grams;
};

typedef struct { uint32_t term, key; float w; } pair_t;

/* escapeBlank (h:93-98) then trim (h:243-247) then optional toUpper (h:72-76).
 * Returns the length written to out (out must hold n bytes). */
static uint32_t normalise(const uint8_t* valid, const uint8_t* p, uint32_t n, uint8_t* out, int upper) {
    uint32_t a = 0, b = n;
    while (a < b && c_isspace(valid[p[a]] ? p[a] : ' ')) ++a;
    while (b > a && c_isspace(valid[p[b - 1]] ? p[b - 1] : ' ')) --b;
    for (uint32_t i = a; i < b; ++i) {
        unsigned c = valid[p[i]] ? p[i] : ' ';
        out[i - a] = (uint8_t)(upper ? c_toupper(c) : c);
    }
    return b - a;
}

static void trim_raw(const uint8_t* p, uint32_t n, uint32_t* a, uint32_t* b) {
    *a = 0; *b = n;
    while (*a < *b && c_isspace(p[*a])) ++*a;
    while (*b > *a && c_isspace(p[*b - 1])) --*b;
}

static int cmp_key_rank(const void* x, const void* y, void* ctx) {
    const uint32_t* len = ctx;
    uint32_t a = *(const uint32_t*)x, b = *(const uint32_t*)y;
    if (len[a] != len[b]) return len[a] < len[b] ? -1 : 1;
    return a < b ? -1 : a > b;
}

static int cmp_wild(const void* x, const void* y, void* ctx) {
    const float* w = ctx;
    uint32_t a = *(const uint32_t*)x, b = *(const uint32_t*)y;
    if (w[a] > w[b]) return -1;
    if (w[a] < w[b]) return 1;
    return a < b ? -1 : a > b;
}

ngo_index* ngo_build(char* const* words, uint64_t size, uint16_t rowSize, const float* weight) {
    ngo_index* ix = xcalloc(1, sizeof(*ix));
    for (const char* c = DEFAULT_VALID; *c; ++c) ix->valid[(uint8_t)*c] = 1;
    ix->gram_off = xcalloc(GRAM_SPACE + 1, 8);
    /* hpp:122-123: an empty/absent library leaves the index unbuilt (search answers 0).
     * rowSize 0 would loop forever in the reference (hpp:126); treated the same way. */
    if (size < 2 || !words || rowSize == 0) return ix;

    strtab terms, keys;
    st_init(&terms); st_init(&keys);
    uint64_t npair = 0, cap = 1024;
    pair_t* pairs = xmalloc(cap * sizeof(pair_t));
    uint8_t* scratch = NULL; size_t scap = 0;

    for (uint64_t i = 0; i < size; i += rowSize) {                 /* hpp:126 */
        if (!words[i]) continue;                                   /* hpp:129 */
        const uint8_t* raw = (const uint8_t*)words[i];
        uint32_t n = (uint32_t)strlen(words[i]), a, b;
        trim_raw(raw, n, &a, &b);                                  /* hpp:131-132 */
        if (a == b) continue;                                      /* hpp:134 */
        const uint8_t* key = raw + a; uint32_t klen = b - a;
        uint32_t kid = UINT32_MAX;
        for (uint64_t j = i; j < i + rowSize && j < size; ++j) {   /* hpp:150 (clamped) */
            if (!words[j]) continue;
            const uint8_t* src = j == i ? key : (const uint8_t*)words[j];
            uint32_t sl = j == i ? klen : (uint32_t)strlen(words[j]);
            if (sl > scap) { scap = sl * 2 + 16; scratch = xrealloc(scratch, scap); }
            uint32_t tl = normalise(ix->valid, src, sl, scratch, 1); /* hpp:136-139, :153-156 */
            if (j != i && tl == 0) continue;                       /* hpp:157 (key term may be "") */
            float w = weight ? weight[j] : 1.0f;                   /* hpp:141-143, :159-161 */
            if (w == 0.0f) continue;                               /* hpp:144, :162 */
            if (kid == UINT32_MAX) kid = st_intern(&keys, key, klen);
            uint32_t tid = st_intern(&terms, scratch, tl);
            if (npair == cap) { cap *= 2; pairs = xrealloc(pairs, cap * sizeof(pair_t)); }
            pairs[npair++] = (pair_t){tid, kid, w};                /* hpp:146-147, :164-165 */
        }
    }
    free(scratch);

    /* (term,key) -> weight, last write wins (tempWeightMap[t][k] = w). */
    uint64_t hs = 16; while (hs < npair * 2) hs <<= 1;
    uint64_t* hk = xmalloc(hs * 8); uint32_t* hv = xmalloc(hs * 4);
    memset(hk, 0xff, hs * 8);
    uint32_t nuniq = 0;
    for (uint64_t p = 0; p < npair; ++p) {
        uint64_t k = ((uint64_t)pairs[p].term << 32) | pairs[p].key;
        uint64_t h = (k * 0x9E3779B97F4A7C15ull) >> 20;
        for (h &= hs - 1; hk[h] != UINT64_MAX && hk[h] != k; h = (h + 1) & (hs - 1)) {}
        if (hk[h] == k) pairs[hv[h]].w = pairs[p].w;
        else { hk[h] = k; hv[h] = nuniq; pairs[nuniq++] = pairs[p]; }
    }
    free(hk); free(hv);

    /* key ranks: (trimmed raw length asc, first appearance asc) — ScoreComparer h:262-269 */
    ix->n_keys = keys.n;
    uint32_t* korder = xmalloc((size_t)keys.n * 4);
    for (uint32_t k = 0; k < keys.n; ++k) korder[k] = k;
    qsort_r(korder, keys.n, 4, cmp_key_rank, keys.len);
    uint32_t* krank = xmalloc((size_t)keys.n * 4);
    ix->key_off = xmalloc(((size_t)keys.n + 1) * 8);
    ix->key_bytes = xmalloc(keys.blob_len + 1);
    uint64_t ko = 0;
    for (uint32_t r = 0; r < keys.n; ++r) {
        uint32_t k = korder[r]; krank[k] = r;
        ix->key_off[r] = ko;
        memcpy(ix->key_bytes + ko, keys.blob + keys.off[k], keys.len[k]);
        ko += keys.len[k];
    }
    ix->key_off[keys.n] = ko;

    /* term ids: shortLib (len < 6) first, then longLib, each in first-appearance order */
    ix->n_terms = terms.n;
    uint32_t* tmap = xmalloc((size_t)terms.n * 4);
    uint32_t ns = 0;
    for (uint32_t t = 0; t < terms.n; ++t) if (terms.len[t] < SHORT_TERM_LEN) tmap[t] = ns++;
    ix->n_short = ns;
    uint32_t nl = ns;
    for (uint32_t t = 0; t < terms.n; ++t) if (terms.len[t] >= SHORT_TERM_LEN) tmap[t] = nl++;
    ix->term_off = xmalloc(((size_t)terms.n + 1) * 8);
    ix->term_bytes = xmalloc(terms.blob_len + 1);
    {
        uint32_t* inv = xmalloc((size_t)terms.n * 4);
        for (uint32_t t = 0; t < terms.n; ++t) inv[tmap[t]] = t;
        uint64_t o = 0;
        for (uint32_t r = 0; r < terms.n; ++r) {
            uint32_t t = inv[r];
            ix->term_off[r] = o;
            memcpy(ix->term_bytes + o, terms.blob + terms.off[t], terms.len[t]);
            o += terms.len[t];
        }
        ix->term_off[terms.n] = o;
        free(inv);
    }

    /* term -> (key, weight) CSR */
    ix->tk_off = xcalloc((size_t)terms.n + 1, 4);
    for (uint32_t p = 0; p < nuniq; ++p) ix->tk_off[tmap[pairs[p].term] + 1]++;
    for (uint32_t t = 0; t < terms.n; ++t) ix->tk_off[t + 1] += ix->tk_off[t];
    ix->tk_key = xmalloc((size_t)nuniq * 4); ix->tk_w = xmalloc((size_t)nuniq * 4);
    {
        uint32_t* fill = xmalloc((size_t)terms.n * 4);
        memcpy(fill, ix->tk_off, (size_t)terms.n * 4);
        for (uint32_t p = 0; p < nuniq; ++p) {
            uint32_t t = tmap[pairs[p].term], d = fill[t]++;
            ix->tk_key[d] = krank[pairs[p].key]; ix->tk_w[d] = pairs[p].w;
        }
        free(fill);
    }
    /* key -> terms: which pairs a promotable key has (emit_term's short-group rule) */
    ix->kt_off = xcalloc((size_t)keys.n + 1, 4);
    ix->kt_term = xmalloc((size_t)nuniq * 4 + 4);
    for (uint32_t p = 0; p < nuniq; ++p) ix->kt_off[krank[pairs[p].key] + 1]++;
    for (uint32_t k = 0; k < keys.n; ++k) ix->kt_off[k + 1] += ix->kt_off[k];
    {
        uint32_t* fill = xmalloc((size_t)keys.n * 4 + 4);
        memcpy(fill, ix->kt_off, (size_t)keys.n * 4);
        for (uint32_t p = 0; p < nuniq; ++p) ix->kt_term[fill[krank[pairs[p].key]]++] = tmap[pairs[p].term];
        free(fill);
    }

    /* wildcard answer (hpp:356-369): every key with a weight of one of its pairs */
    ix->wild_w = xmalloc((size_t)keys.n * 4);
    {
        uint8_t* seen = xcalloc(keys.n, 1);
        for (uint32_t p = 0; p < nuniq; ++p) {
            uint32_t k = krank[pairs[p].key];
            if (!seen[k] || pairs[p].w > ix->wild_w[k]) ix->wild_w[k] = pairs[p].w;
            seen[k] = 1;
        }
        free(seen);
        ix->wild_order = xmalloc((size_t)keys.n * 4);
        for (uint32_t k = 0; k < keys.n; ++k) ix->wild_order[k] = k;
        qsort_r(ix->wild_order, keys.n, 4, cmp_wild, ix->wild_w);
    }

    /* grams of long terms, deduplicated per term (ngrams[h].insert(id), hpp:13-21) */
    {
        uint32_t* stamp = xcalloc(GRAM_SPACE, 4);
        uint64_t* cnt = ix->gram_off + 1;
        for (uint32_t t = ns; t < terms.n; ++t) {
            const uint8_t* s = ix->term_bytes + ix->term_off[t];
            uint32_t L = (uint32_t)(ix->term_off[t + 1] - ix->term_off[t]);
            for (uint32_t i = 0; i + 2 < L; ++i) {
                uint32_t g = ((uint32_t)s[i] << 14) | ((uint32_t)s[i + 1] << 7) | s[i + 2];
                if (stamp[g] != t + 1) { stamp[g] = t + 1; cnt[g]++; }
            }
        }
        for (uint32_t g = 0; g < GRAM_SPACE; ++g) {
            ix->n_grams += ix->gram_off[g + 1] != 0;
            ix->gram_off[g + 1] += ix->gram_off[g];
        }
        ix->post = xmalloc(ix->gram_off[GRAM_SPACE] * 4 + 4);
        uint64_t* pos = xmalloc((size_t)GRAM_SPACE * 8);
        memcpy(pos, ix->gram_off, (size_t)GRAM_SPACE * 8);
        memset(stamp, 0, (size_t)GRAM_SPACE * 4);
        for (uint32_t t = ns; t < terms.n; ++t) {
            const uint8_t* s = ix->term_bytes + ix->term_off[t];
            uint32_t L = (uint32_t)(ix->term_off[t + 1] - ix->term_off[t]);
            for (uint32_t i = 0; i + 2 < L; ++i) {
                uint32_t g = ((uint32_t)s[i] << 14) | ((uint32_t)s[i + 1] << 7) | s[i + 2];
                if (stamp[g] != t + 1) { stamp[g] = t + 1; ix->post[pos[g]++] = t - ns; }
            }
        }
        free(pos); free(stamp);
    }

    free(korder); free(krank); free(tmap); free(pairs);
    st_free(&terms); st_free(&keys);
    ix->indexed = 1;                                               /* hpp:45 */
    return ix;
}

void ngo_free(ngo_index* ix) {
    if (!ix) return;
    free(ix->term_off); free(ix->term_bytes); free(ix->tk_off); free(ix->tk_key); free(ix->tk_w);
    free(ix->kt_off); free(ix->kt_term);
    free(ix->key_off); free(ix->key_bytes); free(ix->wild_w); free(ix->wild_order);
    free(ix->gram_off); free(ix->post); free(ix);
}

int ngo_indexed(const ngo_index* ix) { return ix && ix->indexed; }
uint64_t ngo_size(const ngo_index* ix) { return ix ? ix->n_terms : 0; }
uint64_t ngo_libsize(const ngo_index* ix) { return ix ? ix->n_grams : 0; }
uint32_t ngo_nkeys(const ngo_index* ix) { return ix ? ix->n_keys : 0; }

const char* ngo_key(const ngo_index* ix, uint32_t key, uint32_t* len) {
    if (len) *len = (uint32_t)(ix->key_off[key + 1] - ix->key_off[key]);
    return (const char*)ix->key_bytes + ix->key_off[key];
}

void ngo_set_valid(ngo_index* ix, const char* chars, int n) {
    memset(ix->valid, 0, sizeof(ix->valid));
    for (int i = 0; i < n; ++i) ix->valid[(uint8_t)chars[i]] = 1;
}

/* ------------------------------------------------------------------ search ------------ */
typedef struct {
    uint32_t* cnt; uint32_t* touched; /* long-term counters + touched list */
    uint32_t* kenc; uint32_t* ktouch; uint32_t nkt;
    /* per key, for ngo_search_amb: bit 0 a long pair promotes, bit 1 a short pair promotes;
     * the best non-promoting long / short encodings */
    uint8_t* kfl; uint32_t* knl; uint32_t* kns;
    uint64_t* sortbuf;
    uint8_t* q; size_t qcap;
} workspace;

static void ws_init(workspace* w, const ngo_index* ix) {
    memset(w, 0, sizeof(*w));
    uint32_t nl = ix->n_terms - ix->n_short;
    w->cnt = xcalloc(nl + 1, 4); w->touched = xmalloc(((size_t)nl + 1) * 4);
    w->kenc = xcalloc((size_t)ix->n_keys + 1, 4); w->ktouch = xmalloc(((size_t)ix->n_keys + 1) * 4);
    w->sortbuf = xmalloc(((size_t)ix->n_keys + 1) * 8);
    w->kfl = xcalloc((size_t)ix->n_keys + 1, 1);
    w->knl = xcalloc((size_t)ix->n_keys + 1, 4); w->kns = xcalloc((size_t)ix->n_keys + 1, 4);
}
static void ws_free(workspace* w) {
    free(w->cnt); free(w->touched); free(w->kenc); free(w->ktouch); free(w->sortbuf); free(w->q);
    free(w->kfl); free(w->knl); free(w->kns);
}

/* libStr = escapeBlank(stringLib[key]); trim; libStr == query  (hpp:330-334; no toUpper) */
static int key_matches_query(const ngo_index* ix, uint32_t k, const uint8_t* q, uint32_t m) {
    const uint8_t* p = ix->key_bytes + ix->key_off[k];
    uint32_t n = (uint32_t)(ix->key_off[k + 1] - ix->key_off[k]), a = 0, b = n;
    while (a < b && c_isspace(ix->valid[p[a]] ? p[a] : ' ')) ++a;
    while (b > a && c_isspace(ix->valid[p[b - 1]] ? p[b - 1] : ' ')) --b;
    if (b - a != m) return 0;
    for (uint32_t i = 0; i < m; ++i)
        if ((ix->valid[p[a + i]] ? p[a + i] : ' ') != q[i]) return 0;
    return 1;
}

/* Does key k have a long term that every gram of the query hits (searchLong scores it
 * count/n = 1 > 0.999, hpp:300,328) and that passes the threshold? Then calcScore's long pass
 * promotes k (hpp:335) after every short pair of k (hpp:393-394). */
static int key_promoted_long(const ngo_index* ix, uint32_t k, const uint8_t* q, uint32_t m, float thr) {
    if (m < 3 || 1.0f < thr) return 0;                             /* hpp:281, :315 */
    for (uint32_t p = ix->kt_off[k]; p < ix->kt_off[k + 1]; ++p) {
        uint32_t t = ix->kt_term[p];
        if (t < ix->n_short) continue;
        const uint8_t* s = ix->term_bytes + ix->term_off[t];
        uint32_t L = (uint32_t)(ix->term_off[t + 1] - ix->term_off[t]), all = 1;
        for (uint32_t i = 0; all && i + 2 < m; ++i) {
            if ((q[i] | q[i + 1] | q[i + 2]) & 0x80) { all = 0; break; } /* never counted (search_ws) */
            uint32_t hit = 0;
            for (uint32_t j = 0; !hit && j + 2 < L; ++j)
                hit = s[j] == q[i] && s[j + 1] == q[i + 1] && s[j + 2] == q[i + 2];
            all = hit;
        }
        if (all) return 1;
    }
    return 0;
}

/* calcScore (hpp:310-341) for one scored term: threshold, weight, max-merge, promotion.
 * grp: 1 = a short score (searchShort), 0 = a long one (searchLong). */
static void emit_term(const ngo_index* ix, workspace* w, uint32_t t, float s, float thr,
                      const uint8_t* q, uint32_t m, int grp) {
    if (s < thr) return;                                           /* hpp:315 */
    int exact_possible = (double)s > 0.999;                        /* hpp:328 */
    for (uint32_t p = ix->tk_off[t]; p < ix->tk_off[t + 1]; ++p) {
        uint32_t k = ix->tk_key[p];
        float sc = ix->tk_w[p] * s;                                /* hpp:326 */
        uint32_t enc = sc > 0.0f ? f2u(sc) + 1u : 1u;              /* max(w*s, 0.0f) */
        int promo = exact_possible && key_matches_query(ix, k, q, m);
        if (promo) enc = ENC100;                                   /* hpp:335: score = 100 */
        /* a short pair above 100 of a key that the long pass promotes later is overwritten */
        if (grp && !promo && enc > ENC100 && key_matches_query(ix, k, q, m) && key_promoted_long(ix, k, q, m, thr))
            continue;
        if (!w->kenc[k]) w->ktouch[w->nkt++] = k;
        if (enc > w->kenc[k]) w->kenc[k] = enc;
        if (promo) w->kfl[k] |= grp ? 2 : 1;
        else if (grp) { if (enc > w->kns[k]) w->kns[k] = enc; }
        else if (enc > w->knl[k]) w->knl[k] = enc;
    }
}

/* stringMatch (hpp:182-222): semi-global edit distance, free start/end in the source */
static uint32_t string_match(const uint8_t* q, uint32_t m, const uint8_t* s, uint32_t n) {
    uint32_t col[SHORT_QUERY_LEN + 1];
    for (uint32_t i = 0; i <= m; ++i) col[i] = i;                  /* column j = 0 */
    uint32_t best = m;
    for (uint32_t j = 0; j < n; ++j) {
        uint32_t diag = col[0], cur = 0;                           /* D[0][j] = 0: free start */
        for (uint32_t i = 1; i <= m; ++i) {
            uint32_t up = col[i];
            uint32_t v = diag + (q[i - 1] != s[j]);
            if (up + 1 < v) v = up + 1;
            if (cur + 1 < v) v = cur + 1;
            diag = up; col[i] = v; cur = v;
        }
        col[0] = 0;
        if (col[m] < best) best = col[m];                          /* hpp:217-220 */
    }
    return m - best;
}

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

static uint32_t search_ws(const ngo_index* ix, workspace* w, const char* query, float thr, uint32_t limit,
                          uint32_t* out_keys, float* out_scores, uint32_t cap, int* amb) {
    if (amb) *amb = 0;
    if (!ix->indexed) return 0;                                    /* hpp:417-418 */
    if (limit == 0) limit = 2147483647u;                           /* hpp:420-421 */
    if (cap < limit) limit = cap;
    size_t qn = strlen(query);
    if (qn == 0 || (qn == 1 && query[0] == '*')) {                 /* hpp:356 wildcard */
        uint32_t n = ix->n_keys < limit ? ix->n_keys : limit;
        for (uint32_t i = 0; i < n; ++i) {
            out_keys[i] = ix->wild_order[i];
            out_scores[i] = ix->wild_w[ix->wild_order[i]];
        }
        return n;
    }
    if (qn > w->qcap) { w->qcap = qn * 2; w->q = xrealloc(w->q, w->qcap); }
    uint32_t m = normalise(ix->valid, (const uint8_t*)query, (uint32_t)qn, w->q, 1); /* hpp:372-376 */
    if (m == 0) return 0;
    const uint8_t* q = w->q;
    w->nkt = 0;

    if (m < SHORT_QUERY_LEN) {                                     /* hpp:381 searchShort */
        uint32_t end = m <= 3 ? ix->n_terms : ix->n_short;         /* hpp:247 */
        for (uint32_t t = 0; t < end; ++t) {
            const uint8_t* s = ix->term_bytes + ix->term_off[t];
            uint32_t L = (uint32_t)(ix->term_off[t + 1] - ix->term_off[t]);
            emit_term(ix, w, t, (float)string_match(q, m, s, L) / (float)m, thr, q, m, 1); /* hpp:244 */
        }
    }
    if (m >= 3) {                                                  /* hpp:281 searchLong */
        uint32_t ng = m - 2, nt = 0;
        for (uint32_t i = 0; i < ng; ++i) {
            if ((q[i] | q[i + 1] | q[i + 2]) & 0x80) continue;     /* negative hash: never indexed */
            uint32_t g = ((uint32_t)q[i] << 14) | ((uint32_t)q[i + 1] << 7) | q[i + 2];
            for (uint64_t p = ix->gram_off[g]; p < ix->gram_off[g + 1]; ++p) { /* hpp:289-298 */
                uint32_t t = ix->post[p];
                if (w->cnt[t]++ == 0) w->touched[nt++] = t;
            }
        }
        for (uint32_t i = 0; i < nt; ++i) {
            uint32_t t = w->touched[i];
            emit_term(ix, w, ix->n_short + t, (float)w->cnt[t] / (float)ng, thr, q, m, 0); /* hpp:300 */
            w->cnt[t] = 0;
        }
    }

    /* partial_sort by ScoreComparer (hpp:397-401): score desc, then key rank asc */
    for (uint32_t i = 0; i < w->nkt; ++i) {
        uint32_t k = w->ktouch[i];
        w->sortbuf[i] = ((uint64_t)(~w->kenc[k]) << 32) | k;
        /* the reference's score of k depends on unordered_map order: a long promotion with a
         * long pair above 100 beside it, or (no long promotion) a short promotion with a short
         * pair above both 100 and every long pair */
        if (amb && ((w->kfl[k] & 1) ? w->knl[k] > ENC100
                                     : (w->kfl[k] & 2) && w->kns[k] > ENC100 && w->kns[k] > w->knl[k]))
            *amb = 1;
        w->kenc[k] = 0; w->kfl[k] = 0; w->knl[k] = 0; w->kns[k] = 0;
    }
    qsort(w->sortbuf, w->nkt, 8, cmp_u64);
    uint32_t n = w->nkt < limit ? w->nkt : limit;                  /* hpp:425 */
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t enc = ~(uint32_t)(w->sortbuf[i] >> 32);
        out_keys[i] = (uint32_t)w->sortbuf[i];
        out_scores[i] = u2f(enc - 1u);
    }
    return n;
}

uint32_t ngo_search(const ngo_index* ix, const char* query, float threshold, uint32_t limit,
                    uint32_t* out_keys, float* out_scores, uint32_t cap) {
    workspace w;
    ws_init(&w, ix);
    uint32_t n = search_ws(ix, &w, query, threshold, limit, out_keys, out_scores, cap, NULL);
    ws_free(&w);
    return n;
}

uint32_t ngo_search_amb(const ngo_index* ix, const char* query, float threshold, uint32_t limit,
                        uint32_t* out_keys, float* out_scores, uint32_t cap, int* ambiguous) {
    workspace w;
    ws_init(&w, ix);
    uint32_t n = search_ws(ix, &w, query, threshold, limit, out_keys, out_scores, cap, ambiguous);
    ws_free(&w);
    return n;
}

typedef struct {
    const ngo_index* ix; const char* const* qs; uint32_t n; float thr; uint32_t limit;
    uint32_t* counts; uint32_t* keys; float* scores; uint32_t cap;
    uint32_t* next; pthread_mutex_t* mu;
} batch_arg;

static void* batch_worker(void* p) {
    batch_arg* a = p;
    workspace w;
    ws_init(&w, a->ix);
    for (;;) {
        pthread_mutex_lock(a->mu);
        uint32_t i = *a->next; *a->next += 16;
        pthread_mutex_unlock(a->mu);
        if (i >= a->n) break;
        uint32_t e = i + 16 < a->n ? i + 16 : a->n;
        for (; i < e; ++i)
            a->counts[i] = search_ws(a->ix, &w, a->qs[i], a->thr, a->limit, a->keys + (size_t)i * a->cap,
                                     a->scores + (size_t)i * a->cap, a->cap, NULL);
    }
    ws_free(&w);
    return NULL;
}

void ngo_search_batch(const ngo_index* ix, const char* const* queries, uint32_t n, float threshold,
                      uint32_t limit, uint32_t* out_counts, uint32_t* out_keys, float* out_scores,
                      uint32_t cap, int threads) {
    if (threads < 1) threads = 1;
    uint32_t next = 0;
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    batch_arg a = {ix, queries, n, threshold, limit, out_counts, out_keys, out_scores, cap, &next, &mu};
    pthread_t* th = xmalloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &a);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
}
