/* synth.c — synthetic corpus / query generator for bench.py.
 *
 * Byte-identical to stringsearchlib_amd/synth.py (tests/test_synth.py checks it); C because
 * the bench corpus has 10M rows. Words are NUL-terminated strings in one malloc'd blob;
 * `words` points into it, so the arrays can go straight to indexN(). Free with ngs_synth_free.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 ";

static uint64_t next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__attribute__((visibility("default"))) int ngs_synth_corpus(uint64_t rows, uint64_t seed, uint32_t min_len,
                                                            uint32_t span, uint32_t row_size, char** blob_out,
                                                            char*** words_out, float** weights_out,
                                                            uint64_t* state_out) {
    const uint64_t n = rows * row_size;
    char* blob = malloc(n * (min_len + span) + 1);
    char** words = malloc(sizeof(char*) * (n ? n : 1));
    float* weights = malloc(sizeof(float) * (n ? n : 1));
    if (!blob || !words || !weights) { free(blob); free(words); free(weights); return -1; }
    uint64_t s = seed, o = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t L = min_len + (uint32_t)(next(&s) % span);
        char* w = blob + o;
        for (uint32_t j = 0; j < L; ++j) w[j] = A[next(&s) % 37];
        w[0] = A[next(&s) % 26];
        w[L - 1] = A[next(&s) % 26];
        w[L] = 0;
        words[i] = w;
        weights[i] = 0.5f + (float)(next(&s) >> 40) / 16777216.0f;
        o += L + 1;
    }
    *blob_out = blob;
    *words_out = words;
    *weights_out = weights;
    *state_out = s;
    return 0;
}

__attribute__((visibility("default"))) int ngs_synth_queries(char* const* words, uint64_t nwords, uint32_t row_size,
                                                             uint64_t nq, uint64_t* state, uint32_t qlen,
                                                             char** blob_out, uint64_t** off_out) {
    const uint64_t nkeys = nwords / row_size;
    char* blob = malloc(nq * qlen + 1);
    uint64_t* off = malloc(sizeof(uint64_t) * (nq + 1));
    if (!blob || !off || !nkeys) { free(blob); free(off); return -1; }
    uint64_t o = 0;
    off[0] = 0;
    for (uint64_t i = 0; i < nq; ++i) {
        const char* src = words[(next(state) % nkeys) * row_size];
        const uint64_t len = strlen(src);
        const uint64_t l = len < qlen ? len : qlen;
        const uint64_t st = next(state) % (len - l + 1);
        memcpy(blob + o, src + st, l);
        const uint64_t p = next(state) % l;
        blob[o + p] = A[next(state) % 26];
        o += l;
        off[i + 1] = o;
    }
    *blob_out = blob;
    *off_out = off;
    return 0;
}

__attribute__((visibility("default"))) void ngs_synth_free(void* p) { free(p); }

/* UTF-32 copies of n NUL-terminated byte strings (the C4 wide corpus: every byte becomes one
 * code point), for indexW. Free both outputs with ngs_synth_free. */
__attribute__((visibility("default"))) int ngs_synth_widen(char* const* words, uint64_t n, uint32_t** blob_out,
                                                           uint32_t*** words_out) {
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += strlen(words[i]) + 1;
    uint32_t* blob = malloc(sizeof(uint32_t) * (total ? total : 1));
    uint32_t** w = malloc(sizeof(uint32_t*) * (n ? n : 1));
    if (!blob || !w) { free(blob); free(w); return -1; }
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; ++i) {
        w[i] = blob + o;
        for (const unsigned char* p = (const unsigned char*)words[i]; *p; ++p) blob[o++] = *p;
        blob[o++] = 0;
    }
    *blob_out = blob;
    *words_out = w;
    return 0;
}
