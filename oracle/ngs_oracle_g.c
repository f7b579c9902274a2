/* ngs_oracle_g.c — CPU restatement of the search path generalised to a gram size g and to
 * UTF-32 strings (the indexG / indexW extensions; plain C11).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for tests/ and the cpu_baseline leg of bench.py.
 * The product (stringsearchlib_amd/csrc) never links it.
 *
 * PARITY UNPINNED beyond g = 3 narrow: the reference has no gram-size parameter and no wide
 * path (Readme.md:47,91,135 only documents them). This restatement follows
 * the same reference lines as ngs_oracle.c with every literal scaled by g:
 *   long/short term split  len >= 2g                (nGramSearch.hpp:82, 6 = 2 x 3)
 *   short search           |q| < 3g                 (hpp:381, 9 = 3 x 3)
 *   full-library scan      |q| <= g                 (hpp:235,247, 3)
 *   long search            |q| >= g, n = |q| - g + 1 (hpp:281,286)
 *   grams                  g consecutive characters (nGramSearch.h:147-150 for g = 3)
 * Wide normalisation: code points < 128 follow the byte rules (validChar h:307-313,
 * toUpper h:72-76, isspace trim h:30-52); code points >= 128 are kept unchanged; values
 * above 0x10FFFF (not code points) become spaces.
 * Its pin is self-consistency: with g = 3 on byte strings it must answer exactly like
 * ngs_oracle.c (tests/test_oracle_generic.py), which is pinned to the reference.
 * It is written independently of ngs_oracle.c (hash maps instead of the 21-bit gram table)
 * so that the cross-check is not a check of shared code.
 * Promotion (hpp:328-335) follows ngs_oracle.c: a promoted key scores 100, an ordinary score;
 * a group's promoting pairs are taken first (a long promotion overwrites the key's short pairs).
 */
#define _GNU_SOURCE
#include "ngs_oracle_g.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ENC100 (0x42C80000u + 1u) /* enc of the score 100: a promoted key */
#define MAX_G 3

static const char DEFAULT_VALID[] =
    ".%$ @0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"; /* h:307-313 */

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "ngs_oracle_g: out of memory (%zu)\n", n); abort(); }
    return p;
}
static void* xcalloc(size_t n, size_t s) {
    void* p = calloc(n ? n : 1, s ? s : 1);
    if (!p) { fprintf(stderr, "ngs_oracle_g: out of memory\n"); abort(); }
    return p;
}
static void* xrealloc(void* p, size_t n) {
    p = realloc(p, n ? n : 1);
    if (!p) { fprintf(stderr, "ngs_oracle_g: out of memory\n"); abort(); }
    return p;
}
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static int is_space(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13); }
static uint32_t to_upper(uint32_t c) { return (c >= 'a' && c <= 'z') ? c - 32u : c; }

/* ------------------------------------------------------------------ u32 strings ------- */
typedef struct { uint32_t* p; uint32_t n; } ustr;

static uint64_t hash_u32s(const uint32_t* p, uint32_t n) {
    uint64_t h = 0xcbf29ce484222325ull ^ n;
    for (uint32_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ull; }
    return h ^ (h >> 31);
}

/* interning table of u32 strings in first-insertion order */
typedef struct {
    ustr* s; uint32_t n, cap;
    uint32_t* slot; uint64_t nslot;
} stab;

static void stab_init(stab* t) { memset(t, 0, sizeof(*t)); t->nslot = 256; t->slot = xcalloc(t->nslot, 4); }
static uint32_t stab_intern(stab* t, const uint32_t* p, uint32_t n) {
    if ((uint64_t)(t->n + 1) * 2 > t->nslot) {
        uint64_t ns = t->nslot * 2;
        uint32_t* s = xcalloc(ns, 4);
        for (uint32_t id = 0; id < t->n; ++id) {
            uint64_t h = hash_u32s(t->s[id].p, t->s[id].n) & (ns - 1);
            while (s[h]) h = (h + 1) & (ns - 1);
            s[h] = id + 1;
        }
        free(t->slot); t->slot = s; t->nslot = ns;
    }
    uint64_t h = hash_u32s(p, n) & (t->nslot - 1);
    while (t->slot[h]) {
        uint32_t id = t->slot[h] - 1;
        if (t->s[id].n == n && memcmp(t->s[id].p, p, (size_t)n * 4) == 0) return id;
        h = (h + 1) & (t->nslot - 1);
    }
    if (t->n == t->cap) { t->cap = t->cap ? t->cap * 2 : 256; t->s = xrealloc(t->s, t->cap * sizeof(ustr)); }
    ustr u = {xmalloc((size_t)n * 4 + 4), n};
    memcpy(u.p, p, (size_t)n * 4);
    u.p[n] = 0;
    t->s[t->n] = u;
    t->slot[h] = ++t->n;
    return t->n - 1;
}

/* ------------------------------------------------------------------ index ------------- */
typedef struct { uint32_t key; float w; } kw;
typedef struct { uint64_t gram; uint32_t* post; uint32_t n, cap; } glist;

struct ngog_index {
    int indexed, wide;
    uint32_t g;
    uint8_t valid[256];
    uint32_t n_terms;            /* terms in first-appearance order (ids are not reordered) */
    ustr* terms;
    kw** tkeys; uint32_t* ntk;   /* term -> (key rank, weight) in insertion order */
    uint32_t* kt_off; uint32_t* kt_term; /* key rank -> its terms */
    uint32_t n_keys;
    ustr* keys;                  /* by rank: (trimmed raw length, first appearance) */
    float* wild_w; uint32_t* wild_order;
    glist* gl; uint64_t nglist;  /* open addressing on the packed gram (gram ~0 = empty) */
    uint64_t n_grams;
};

static uint32_t esc(const ngog_index* ix, uint32_t c) {
    if (!ix->wide || c < 128) return c < 256 && ix->valid[c] ? c : ' ';
    return c > 0x10FFFFu ? ' ' : c;
}

/* escapeBlank (h:93-98) -> trim (h:243-247) -> optional toUpper (h:72-76) */
static uint32_t normalise(const ngog_index* ix, const uint32_t* p, uint32_t n, uint32_t* out, int upper) {
    uint32_t a = 0, b = n;
    while (a < b && is_space(esc(ix, p[a]))) ++a;
    while (b > a && is_space(esc(ix, p[b - 1]))) --b;
    for (uint32_t i = a; i < b; ++i) {
        uint32_t c = esc(ix, p[i]);
        out[i - a] = upper ? to_upper(c) : c;
    }
    return b - a;
}

static uint64_t gram_of(const uint32_t* s, uint32_t g) {
    uint64_t k = 0;
    for (uint32_t j = 0; j < g; ++j) k = (k << 21) | s[j];
    return k;
}

static glist* gl_find(const ngog_index* ix, uint64_t gram) {
    if (!ix->nglist) return NULL;
    uint64_t h = (gram * 0x9E3779B97F4A7C15ull) >> 17;
    for (h &= ix->nglist - 1; ix->gl[h].gram != ~0ull; h = (h + 1) & (ix->nglist - 1))
        if (ix->gl[h].gram == gram) return &ix->gl[h];
    return NULL;
}

static glist* gl_insert(ngog_index* ix, uint64_t gram) {
    if ((ix->n_grams + 1) * 2 > ix->nglist) {
        glist* old = ix->gl; uint64_t on = ix->nglist;
        ix->nglist = on ? on * 2 : 1024;
        ix->gl = xmalloc(ix->nglist * sizeof(glist));
        for (uint64_t i = 0; i < ix->nglist; ++i) ix->gl[i].gram = ~0ull;
        for (uint64_t i = 0; i < on; ++i) {
            if (old[i].gram == ~0ull) continue;
            uint64_t h = ((old[i].gram * 0x9E3779B97F4A7C15ull) >> 17) & (ix->nglist - 1);
            while (ix->gl[h].gram != ~0ull) h = (h + 1) & (ix->nglist - 1);
            ix->gl[h] = old[i];
        }
        free(old);
    }
    uint64_t h = ((gram * 0x9E3779B97F4A7C15ull) >> 17) & (ix->nglist - 1);
    while (ix->gl[h].gram != ~0ull) {
        if (ix->gl[h].gram == gram) return &ix->gl[h];
        h = (h + 1) & (ix->nglist - 1);
    }
    ix->gl[h] = (glist){gram, NULL, 0, 0};
    ix->n_grams++;
    return &ix->gl[h];
}

static uint32_t ulen(const uint32_t* p) { uint32_t n = 0; while (p[n]) ++n; return n; }

static int cmp_rank(const void* x, const void* y, void* ctx) {
    const ustr* k = ctx;
    uint32_t a = *(const uint32_t*)x, b = *(const uint32_t*)y;
    if (k[a].n != k[b].n) return k[a].n < k[b].n ? -1 : 1;
    return a < b ? -1 : a > b;
}
static int cmp_wild(const void* x, const void* y, void* ctx) {
    const float* w = ctx;
    uint32_t a = *(const uint32_t*)x, b = *(const uint32_t*)y;
    if (w[a] != w[b]) return w[a] > w[b] ? -1 : 1;
    return a < b ? -1 : a > b;
}

ngog_index* ngog_build(const uint32_t* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                       uint32_t g, int wide) {
    ngog_index* ix = xcalloc(1, sizeof(*ix));
    ix->g = g; ix->wide = wide;
    for (const char* c = DEFAULT_VALID; *c; ++c) ix->valid[(uint8_t)*c] = 1;
    if (g < 1 || g > MAX_G || size < 2 || !words || rowSize == 0) return ix; /* hpp:122-123 */

    stab terms, keys;
    stab_init(&terms); stab_init(&keys);
    uint32_t tcap = 0;
    uint32_t* scratch = NULL; uint32_t scap = 0;
    for (uint64_t i = 0; i < size; i += rowSize) {                          /* hpp:126 */
        if (!words[i]) continue;                                            /* hpp:129 */
        const uint32_t* raw = words[i];
        uint32_t n = ulen(raw), a = 0, b = n;
        while (a < b && raw[a] < 128 && is_space(raw[a])) ++a;              /* hpp:131-132 */
        while (b > a && raw[b - 1] < 128 && is_space(raw[b - 1])) --b;
        if (a == b) continue;                                               /* hpp:134 */
        int64_t kid = -1;
        uint64_t end = i + rowSize < size ? i + rowSize : size;             /* hpp:150 (clamped) */
        for (uint64_t j = i; j < end; ++j) {
            if (!words[j]) continue;
            const uint32_t* src = j == i ? raw + a : words[j];
            uint32_t sl = j == i ? b - a : ulen(words[j]);
            if (sl + 1 > scap) { scap = sl * 2 + 16; scratch = xrealloc(scratch, (size_t)scap * 4); }
            uint32_t tl = normalise(ix, src, sl, scratch, 1);               /* hpp:136-139, :153-156 */
            if (j != i && tl == 0) continue;                                /* hpp:157 */
            float w = weight ? weight[j] : 1.0f;                            /* hpp:141-143, :159-161 */
            if (w == 0.0f) continue;                                        /* hpp:144, :162 */
            if (kid < 0) kid = stab_intern(&keys, raw + a, b - a);
            uint32_t t = stab_intern(&terms, scratch, tl);
            if (terms.n > tcap) {
                uint32_t nc = terms.n * 2;
                ix->tkeys = xrealloc(ix->tkeys, (size_t)nc * sizeof(kw*));
                ix->ntk = xrealloc(ix->ntk, (size_t)nc * 4);
                for (uint32_t x = tcap; x < nc; ++x) { ix->tkeys[x] = NULL; ix->ntk[x] = 0; }
                tcap = nc;
            }
            /* tempWeightMap[term][key] = w: last write wins */
            uint32_t e = 0;
            while (e < ix->ntk[t] && ix->tkeys[t][e].key != (uint32_t)kid) ++e;
            if (e == ix->ntk[t]) {
                ix->tkeys[t] = xrealloc(ix->tkeys[t], (size_t)(e + 1) * sizeof(kw));
                ix->ntk[t]++;
            }
            ix->tkeys[t][e] = (kw){(uint32_t)kid, w};
        }
    }
    free(scratch);

    /* key ranks (ScoreComparer h:262-269 plus first appearance) */
    ix->n_keys = keys.n;
    uint32_t* order = xmalloc((size_t)keys.n * 4);
    for (uint32_t k = 0; k < keys.n; ++k) order[k] = k;
    qsort_r(order, keys.n, 4, cmp_rank, keys.s);
    uint32_t* rank = xmalloc((size_t)keys.n * 4);
    ix->keys = xmalloc((size_t)keys.n * sizeof(ustr) + sizeof(ustr));
    for (uint32_t r = 0; r < keys.n; ++r) { rank[order[r]] = r; ix->keys[r] = keys.s[order[r]]; }
    free(keys.s); free(keys.slot); /* strings now owned by ix->keys */

    ix->n_terms = terms.n;
    ix->terms = terms.s; terms.s = NULL;
    free(terms.slot);
    ix->wild_w = xcalloc(ix->n_keys, 4);
    uint8_t* seen = xcalloc(ix->n_keys, 1);
    for (uint32_t t = 0; t < ix->n_terms; ++t)
        for (uint32_t e = 0; e < ix->ntk[t]; ++e) {
            kw* p = &ix->tkeys[t][e];
            p->key = rank[p->key];
            if (!seen[p->key] || p->w > ix->wild_w[p->key]) ix->wild_w[p->key] = p->w;
            seen[p->key] = 1;
        }
    free(seen); free(order); free(rank);
    {
        uint64_t np = 0;
        ix->kt_off = xcalloc((size_t)ix->n_keys + 1, 4);
        for (uint32_t t = 0; t < ix->n_terms; ++t)
            for (uint32_t e = 0; e < ix->ntk[t]; ++e) { ix->kt_off[ix->tkeys[t][e].key + 1]++; ++np; }
        for (uint32_t k = 0; k < ix->n_keys; ++k) ix->kt_off[k + 1] += ix->kt_off[k];
        ix->kt_term = xmalloc((size_t)np * 4 + 4);
        uint32_t* fill = xmalloc((size_t)ix->n_keys * 4 + 4);
        memcpy(fill, ix->kt_off, (size_t)ix->n_keys * 4);
        for (uint32_t t = 0; t < ix->n_terms; ++t)
            for (uint32_t e = 0; e < ix->ntk[t]; ++e) ix->kt_term[fill[ix->tkeys[t][e].key]++] = t;
        free(fill);
    }
    ix->wild_order = xmalloc((size_t)ix->n_keys * 4);
    for (uint32_t k = 0; k < ix->n_keys; ++k) ix->wild_order[k] = k;
    qsort_r(ix->wild_order, ix->n_keys, 4, cmp_wild, ix->wild_w);

    /* grams of long terms (len >= 2g), one posting per (gram, term): ngrams[h].insert(id) */
    for (uint32_t t = 0; t < ix->n_terms; ++t) {
        const ustr* s = &ix->terms[t];
        if (s->n < 2 * g) continue;
        for (uint32_t i = 0; i + g <= s->n; ++i) {
            glist* l = gl_insert(ix, gram_of(s->p + i, g));
            if (l->n && l->post[l->n - 1] == t) continue;
            if (l->n == l->cap) { l->cap = l->cap ? l->cap * 2 : 4; l->post = xrealloc(l->post, (size_t)l->cap * 4); }
            l->post[l->n++] = t;
        }
    }
    ix->indexed = 1;                                                         /* hpp:45 */
    return ix;
}

void ngog_free(ngog_index* ix) {
    if (!ix) return;
    for (uint32_t t = 0; t < ix->n_terms; ++t) { free(ix->terms[t].p); free(ix->tkeys[t]); }
    for (uint32_t k = 0; k < ix->n_keys; ++k) free(ix->keys[k].p);
    for (uint64_t i = 0; i < ix->nglist; ++i) if (ix->gl[i].gram != ~0ull) free(ix->gl[i].post);
    free(ix->terms); free(ix->tkeys); free(ix->ntk); free(ix->keys);
    free(ix->wild_w); free(ix->wild_order); free(ix->gl); free(ix->kt_off); free(ix->kt_term); free(ix);
}

int ngog_indexed(const ngog_index* ix) { return ix && ix->indexed; }
uint64_t ngog_size(const ngog_index* ix) { return ix ? ix->n_terms : 0; }
uint64_t ngog_libsize(const ngog_index* ix) { return ix ? ix->n_grams : 0; }
uint32_t ngog_nkeys(const ngog_index* ix) { return ix ? ix->n_keys : 0; }

const uint32_t* ngog_key(const ngog_index* ix, uint32_t key, uint32_t* len) {
    if (len) *len = ix->keys[key].n;
    return ix->keys[key].p;
}

void ngog_set_valid(ngog_index* ix, const char* chars, int n) {             /* dllmain.cpp:142-151 */
    memset(ix->valid, 0, sizeof(ix->valid));
    for (int i = 0; i < n; ++i) ix->valid[(uint8_t)chars[i]] = 1;
}

/* ------------------------------------------------------------------ search ------------ */
typedef struct {
    uint32_t* cnt; uint32_t* touched;
    uint32_t* kenc; uint32_t* ktouch; uint32_t nkt;
    uint64_t* sortbuf;
    uint32_t* q; size_t qcap;
    uint32_t* k; size_t kcap;
} ws;

static void ws_init(ws* w, const ngog_index* ix) {
    memset(w, 0, sizeof(*w));
    w->cnt = xcalloc((size_t)ix->n_terms + 1, 4); w->touched = xmalloc(((size_t)ix->n_terms + 1) * 4);
    w->kenc = xcalloc((size_t)ix->n_keys + 1, 4); w->ktouch = xmalloc(((size_t)ix->n_keys + 1) * 4);
    w->sortbuf = xmalloc(((size_t)ix->n_keys + 1) * 8);
}
static void ws_free(ws* w) {
    free(w->cnt); free(w->touched); free(w->kenc); free(w->ktouch); free(w->sortbuf); free(w->q); free(w->k);
}

/* hpp:330-334: escapeBlank(key), trim, == normalised query (no toUpper on the key) */
static int key_is_query(const ngog_index* ix, ws* w, uint32_t k, const uint32_t* q, uint32_t m) {
    const ustr* s = &ix->keys[k];
    if (s->n + 1 > w->kcap) { w->kcap = s->n * 2 + 2; w->k = xrealloc(w->k, w->kcap * 4); }
    uint32_t n = normalise(ix, s->p, s->n, w->k, 0);
    return n == m && memcmp(w->k, q, (size_t)m * 4) == 0;
}

/* key k has a long term holding every gram of the query (searchLong: s = 1) at this threshold */
static int key_long_full(const ngog_index* ix, uint32_t k, const uint32_t* q, uint32_t m, float thr) {
    const uint32_t g = ix->g;
    if (m < g || 1.0f < thr) return 0;                                       /* hpp:281, :315 */
    for (uint32_t p = ix->kt_off[k]; p < ix->kt_off[k + 1]; ++p) {
        const ustr* s = &ix->terms[ix->kt_term[p]];
        if (s->n < 2 * g) continue;
        int all = 1;
        for (uint32_t i = 0; all && i + g <= m; ++i) {
            const uint64_t gr = gram_of(q + i, g);
            int hit = 0;
            for (uint32_t j = 0; !hit && j + g <= s->n; ++j) hit = gram_of(s->p + j, g) == gr;
            all = hit;
        }
        if (all) return 1;
    }
    return 0;
}

/* calcScore (hpp:310-341); grp 1 = a short score (calcScore's first pass, hpp:393) */
static void emit(const ngog_index* ix, ws* w, uint32_t t, float s, float thr, const uint32_t* q, uint32_t m,
                 int grp) {
    if (s < thr) return;                                                     /* hpp:315 */
    int exact = (double)s > 0.999;                                           /* hpp:328 */
    for (uint32_t e = 0; e < ix->ntk[t]; ++e) {
        uint32_t k = ix->tkeys[t][e].key;
        float sc = ix->tkeys[t][e].w * s;                                    /* hpp:326 */
        uint32_t enc = sc > 0.0f ? f2u(sc) + 1u : 1u;
        const int promo = exact && key_is_query(ix, w, k, q, m);
        if (promo) enc = ENC100;                                             /* hpp:335: score = 100 */
        if (grp && !promo && enc > ENC100 && key_is_query(ix, w, k, q, m) && key_long_full(ix, k, q, m, thr))
            continue;  /* overwritten by the long pass's promotion */
        if (!w->kenc[k]) w->ktouch[w->nkt++] = k;
        if (enc > w->kenc[k]) w->kenc[k] = enc;
    }
}

/* stringMatch (hpp:182-222): edit distance with free start and end in the term */
static uint32_t string_match(const uint32_t* q, uint32_t m, const uint32_t* s, uint32_t n) {
    uint32_t col[3 * MAX_G + 1];
    for (uint32_t i = 0; i <= m; ++i) col[i] = i;
    uint32_t best = m;
    for (uint32_t j = 0; j < n; ++j) {
        uint32_t diag = 0, cur = 0;
        for (uint32_t i = 1; i <= m; ++i) {
            uint32_t up = col[i], v = diag + (q[i - 1] != s[j]);
            if (up + 1 < v) v = up + 1;
            if (cur + 1 < v) v = cur + 1;
            diag = up; col[i] = v; cur = v;
        }
        if (col[m] < best) best = col[m];
    }
    return m - best;
}

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

static uint32_t search_ws(const ngog_index* ix, ws* w, const uint32_t* query, float thr, uint32_t limit,
                          uint32_t* out_keys, float* out_scores, uint32_t cap) {
    if (!ix->indexed) return 0;                                              /* hpp:417-418 */
    if (limit == 0) limit = 2147483647u;                                     /* hpp:420-421 */
    if (cap < limit) limit = cap;
    uint32_t qn = ulen(query);
    if (qn == 0 || (qn == 1 && query[0] == '*')) {                           /* hpp:356 */
        uint32_t n = ix->n_keys < limit ? ix->n_keys : limit;
        for (uint32_t i = 0; i < n; ++i) {
            out_keys[i] = ix->wild_order[i];
            out_scores[i] = ix->wild_w[ix->wild_order[i]];
        }
        return n;
    }
    if (qn + 1 > w->qcap) {
        w->qcap = qn * 2 + 2;
        w->q = xrealloc(w->q, w->qcap * 4);
    }
    uint32_t m = normalise(ix, query, qn, w->q, 1);                          /* hpp:372-376 */
    if (m == 0) return 0;
    const uint32_t* q = w->q;
    const uint32_t g = ix->g;
    w->nkt = 0;
    if (m < 3 * g) {                                                         /* hpp:381 */
        for (uint32_t t = 0; t < ix->n_terms; ++t) {
            const ustr* s = &ix->terms[t];
            if (m > g && s->n >= 2 * g) continue;                            /* hpp:247: shortLib only */
            emit(ix, w, t, (float)string_match(q, m, s->p, s->n) / (float)m, thr, q, m, 1); /* hpp:244 */
        }
    }
    if (m >= g) {                                                            /* hpp:281 */
        uint32_t ng = m - g + 1, nt = 0;
        for (uint32_t i = 0; i < ng; ++i) {
            const glist* l = gl_find(ix, gram_of(q + i, g));
            if (!l) continue;
            for (uint32_t p = 0; p < l->n; ++p)                              /* hpp:289-298 */
                if (w->cnt[l->post[p]]++ == 0) w->touched[nt++] = l->post[p];
        }
        for (uint32_t i = 0; i < nt; ++i) {
            uint32_t t = w->touched[i];
            emit(ix, w, t, (float)w->cnt[t] / (float)ng, thr, q, m, 0);       /* hpp:300 */
            w->cnt[t] = 0;
        }
    }
    for (uint32_t i = 0; i < w->nkt; ++i) {                                 /* hpp:397-401 */
        uint32_t k = w->ktouch[i];
        w->sortbuf[i] = ((uint64_t)(~w->kenc[k]) << 32) | k;
        w->kenc[k] = 0;
    }
    qsort(w->sortbuf, w->nkt, 8, cmp_u64);
    uint32_t n = w->nkt < limit ? w->nkt : limit;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t enc = ~(uint32_t)(w->sortbuf[i] >> 32);
        out_keys[i] = (uint32_t)w->sortbuf[i];
        out_scores[i] = u2f(enc - 1u);
    }
    return n;
}

uint32_t ngog_search(const ngog_index* ix, const uint32_t* query, float threshold, uint32_t limit,
                     uint32_t* out_keys, float* out_scores, uint32_t cap) {
    ws w;
    ws_init(&w, ix);
    uint32_t n = search_ws(ix, &w, query, threshold, limit, out_keys, out_scores, cap);
    ws_free(&w);
    return n;
}

typedef struct {
    const ngog_index* ix; const uint32_t* const* qs; uint32_t n; float thr; uint32_t limit;
    uint32_t* counts; uint32_t* keys; float* scores; uint32_t cap;
    uint32_t* next; pthread_mutex_t* mu;
} barg;

static void* worker(void* p) {
    barg* a = p;
    ws w;
    ws_init(&w, a->ix);
    for (;;) {
        pthread_mutex_lock(a->mu);
        uint32_t i = *a->next; *a->next += 16;
        pthread_mutex_unlock(a->mu);
        if (i >= a->n) break;
        for (uint32_t e = i + 16 < a->n ? i + 16 : a->n; i < e; ++i)
            a->counts[i] = search_ws(a->ix, &w, a->qs[i], a->thr, a->limit, a->keys + (size_t)i * a->cap,
                                     a->scores + (size_t)i * a->cap, a->cap);
    }
    ws_free(&w);
    return NULL;
}

void ngog_search_batch(const ngog_index* ix, const uint32_t* const* queries, uint32_t n, float threshold,
                       uint32_t limit, uint32_t* out_counts, uint32_t* out_keys, float* out_scores,
                       uint32_t cap, int threads) {
    if (threads < 1) threads = 1;
    uint32_t next = 0;
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    barg a = {ix, queries, n, threshold, limit, out_counts, out_keys, out_scores, cap, &next, &mu};
    pthread_t* th = xmalloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &a);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
}
