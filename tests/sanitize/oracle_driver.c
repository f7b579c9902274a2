/* oracle_driver.c — TEST INFRASTRUCTURE: drives the CPU restatement (oracle/ngs_oracle.c,
 * oracle/ngs_oracle_g.c) and the synthetic generator (stringsearchlib_amd/csrc/synth.c) under
 * the compiler's sanitizers (tests/test_sanitizers.py builds it with ASan+UBSan, and with TSan
 * for the pthread batch). Exercises: the synthetic corpus and queries (rowSize 1 and 3, wide
 * copies), index builds with weights (zero, negative, large), NULL words, an empty library,
 * single searches at several thresholds and limits (0 = unlimited, the wildcard, short queries,
 * the full-library scan), setValidChar, the ambiguity report, and ngo_search_batch /
 * ngog_search_batch on 4 threads. Prints "ok" and a checksum of every answer. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ngs_oracle.h"
#include "ngs_oracle_g.h"

int ngs_synth_corpus(uint64_t rows, uint64_t seed, uint32_t min_len, uint32_t span, uint32_t row_size,
                     char** blob_out, char*** words_out, float** weights_out, uint64_t* state_out);
int ngs_synth_queries(char* const* words, uint64_t nwords, uint32_t row_size, uint64_t nq, uint64_t* state,
                      uint32_t qlen, char** blob_out, uint64_t** off_out);
int ngs_synth_widen(char* const* words, uint64_t n, uint32_t** blob_out, uint32_t*** words_out);
void ngs_synth_free(void* p);

static uint64_t mix(uint64_t h, uint64_t v) { return (h ^ v) * 0x100000001b3ull; }

static uint64_t run(uint64_t rows, uint32_t row_size, uint32_t min_len, uint32_t span, int threads) {
    char* blob; char** words; float* wts; uint64_t st;
    if (ngs_synth_corpus(rows, 42 + rows, min_len, span, row_size, &blob, &words, &wts, &st)) abort();
    const uint64_t n = rows * row_size;
    for (uint64_t i = 0; i < n; i += 17) wts[i] = 0.0f;      /* dropped pairs */
    for (uint64_t i = 5; i < n; i += 13) wts[i] = -1.0f;     /* score 0 */
    for (uint64_t i = 7; i < n; i += 11) wts[i] = 150.0f;    /* above the promotion score */
    for (uint64_t i = 3; i < n; i += 29) words[i] = NULL;    /* holes */
    char* qb; uint64_t* qo;
    const uint32_t nq = 300;
    char** live = malloc(sizeof(char*) * n);
    uint64_t nl = 0;
    for (uint64_t i = 0; i < n; ++i) live[nl++] = words[i] ? words[i] : (char*)"ABCDEFGH";
    if (ngs_synth_queries(live, nl - nl % row_size, row_size, nq, &st, 12, &qb, &qo)) abort();
    char** qs = malloc(sizeof(char*) * (nq + 8));
    for (uint32_t i = 0; i < nq; ++i) {
        const uint64_t l = qo[i + 1] - qo[i];
        qs[i] = malloc(l + 1);
        memcpy(qs[i], qb + qo[i], l);
        qs[i][l] = 0;
    }
    const char* extra[8] = {"", "*", "AB", "A", "  x y  ", "###", live[0], live[row_size]};
    for (int i = 0; i < 8; ++i) qs[nq + i] = strdup(extra[i]);
    const uint32_t tq = nq + 8;

    ngo_index* ix = ngo_build(words, n, (uint16_t)row_size, wts);
    uint64_t h = mix(ngo_size(ix), ngo_libsize(ix));
    const uint32_t cap = ngo_nkeys(ix) ? ngo_nkeys(ix) : 1;
    uint32_t* keys = malloc(sizeof(uint32_t) * cap);
    float* sc = malloc(sizeof(float) * cap);
    const float thr[3] = {0.0f, 0.3f, 0.6f};
    const uint32_t lim[3] = {0, 7, 100};
    for (uint32_t i = 0; i < tq; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                int amb = 0;
                const uint32_t k = ngo_search_amb(ix, qs[i], thr[a], lim[b], keys, sc, cap, &amb);
                h = mix(h, k + 31u * (uint32_t)amb);
                for (uint32_t j = 0; j < k; ++j) {
                    uint32_t u; memcpy(&u, &sc[j], 4);
                    uint32_t kl; (void)ngo_key(ix, keys[j], &kl);
                    h = mix(mix(h, keys[j]), u ^ kl);
                }
            }
    ngo_set_valid(ix, "ABCDE ", 6);
    for (uint32_t i = 0; i < tq; i += 7) h = mix(h, ngo_search(ix, qs[i], 0.2f, 50, keys, sc, cap));
    ngo_set_valid(ix, ".%$ @0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ", 66);
    /* the pthread batch (TSan: the workers share the index and the counter) */
    const uint32_t bcap = 100;
    uint32_t* bc = malloc(sizeof(uint32_t) * tq);
    uint32_t* bk = malloc(sizeof(uint32_t) * tq * bcap);
    float* bs = malloc(sizeof(float) * tq * bcap);
    ngo_search_batch(ix, (const char* const*)qs, tq, 0.3f, 100, bc, bk, bs, bcap, threads);
    for (uint32_t i = 0; i < tq; ++i) {
        const uint32_t k = ngo_search(ix, qs[i], 0.3f, 100, keys, sc, cap);
        if (k != bc[i] || memcmp(keys, bk + (size_t)i * bcap, k * 4) || memcmp(sc, bs + (size_t)i * bcap, k * 4)) {
            fprintf(stderr, "batch answer %u differs\n", i);
            abort();
        }
    }
    ngo_free(ix);

    /* the generic restatement over UTF-32 copies, gram sizes 1..3, and its batch */
    uint32_t* wb; uint32_t** ww;
    char** nn = malloc(sizeof(char*) * n);
    for (uint64_t i = 0; i < n; ++i) nn[i] = words[i] ? words[i] : (char*)"";
    if (ngs_synth_widen(nn, n, &wb, &ww)) abort();
    uint32_t** wq = malloc(sizeof(uint32_t*) * tq);
    for (uint32_t i = 0; i < tq; ++i) {
        const size_t l = strlen(qs[i]);
        wq[i] = malloc(4 * (l + 1));
        for (size_t j = 0; j <= l; ++j) wq[i][j] = (unsigned char)qs[i][j];
    }
    for (uint32_t g = 1; g <= 3; ++g) {
        ngog_index* gx = ngog_build((const uint32_t* const*)ww, n, (uint16_t)row_size, wts, g, 1);
        const uint32_t gc = ngog_nkeys(gx) ? ngog_nkeys(gx) : 1;
        uint32_t* gk = malloc(sizeof(uint32_t) * gc);
        float* gs = malloc(sizeof(float) * gc);
        for (uint32_t i = 0; i < tq; i += 3) h = mix(h, ngog_search(gx, wq[i], 0.3f, 0, gk, gs, gc));
        ngog_search_batch(gx, (const uint32_t* const*)wq, tq, 0.3f, 100, bc, bk, bs, bcap, threads);
        for (uint32_t i = 0; i < tq; ++i) h = mix(h, bc[i]);
        ngog_free(gx);
        free(gk); free(gs);
    }
    for (uint32_t i = 0; i < tq; ++i) { free(qs[i]); free(wq[i]); }
    free(qs); free(wq); free(nn); free(live); free(keys); free(sc); free(bc); free(bk); free(bs);
    ngs_synth_free(wb); ngs_synth_free(ww);
    ngs_synth_free(qb); ngs_synth_free(qo);
    ngs_synth_free(blob); ngs_synth_free(words); ngs_synth_free(wts);
    return h;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 4;
    uint64_t h = run(2000, 1, 8, 17, threads);
    h = mix(h, run(600, 3, 3, 12, threads));
    h = mix(h, run(400, 1, 1, 6, threads));
    /* an empty library and a NULL word list: unbuilt indexes answer nothing */
    ngo_index* e = ngo_build(NULL, 0, 1, NULL);
    uint32_t k; float s;
    h = mix(h, ngo_search(e, "ABC", 0.0f, 10, &k, &s, 1));
    ngo_free(e);
    printf("ok %016llx\n", (unsigned long long)h);
    return 0;
}
