/* ngs_oracle.h — CPU restatement of the reference search path.
 *
 * TEST INFRASTRUCTURE ONLY. Imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py — never by the product library, which must run on the GPU.
 *
 * Parity pinning: checked against the reference's answers in tests/golden/ fixtures (made by
 * tests/golden/make_golden.py from the reference compiled in place, oracle/_ref) with the
 * tie-aware checker of tests/tiecheck.py. Ties inside a (score, key length) group are
 * unspecified in the reference (partial_sort over unordered_map order, nGramSearch.hpp:397-401);
 * this restatement refines them by first appearance of the key in the input,
 * which is the order the GPU path produces too, so GPU-vs-oracle comparisons are exact.
 */
#ifndef NGS_ORACLE_H
#define NGS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ngo_index ngo_index;

/* nGramSearch.hpp:120-172 (ctor) + init :54-108 + buildGrams :41-46. */
ngo_index* ngo_build(char* const* words, uint64_t size, uint16_t rowSize, const float* weight);
void ngo_free(ngo_index* ix);

int ngo_indexed(const ngo_index* ix);        /* nGramSearch.h:301 */
uint64_t ngo_size(const ngo_index* ix);      /* nGramSearch.hpp:488-491, wordMap.size() */
uint64_t ngo_libsize(const ngo_index* ix);   /* nGramSearch.hpp:496-499, ngrams.size() */
uint32_t ngo_nkeys(const ngo_index* ix);
const char* ngo_key(const ngo_index* ix, uint32_t key, uint32_t* len);

/* dllmain.cpp:142-151 / nGramSearch.hpp:505-508 */
void ngo_set_valid(ngo_index* ix, const char* chars, int n);

/* nGramSearch.hpp:415-438 (score) over _search :350-404. Writes at most `cap` results
 * (key ids into out_keys, scores into out_scores) and returns how many; limit 0 = unlimited. */
uint32_t ngo_search(const ngo_index* ix, const char* query, float threshold, uint32_t limit,
                    uint32_t* out_keys, float* out_scores, uint32_t cap);

/* ngo_search, and *ambiguous = 1 when the reference's answer to this query depends on its
 * unordered_map iteration order beyond ties (a promoted key with another pair scoring above 100
 * in the same calcScore pass, see ngs_oracle.c); 0 otherwise. Test infrastructure (the fuzz). */
uint32_t ngo_search_amb(const ngo_index* ix, const char* query, float threshold, uint32_t limit,
                        uint32_t* out_keys, float* out_scores, uint32_t cap, int* ambiguous);

/* Batch over `threads` pthreads (cpu_baseline). Query i gets slots [i*cap, i*cap+cap). */
void ngo_search_batch(const ngo_index* ix, const char* const* queries, uint32_t n, float threshold,
                      uint32_t limit, uint32_t* out_counts, uint32_t* out_keys, float* out_scores,
                      uint32_t cap, int threads);

#ifdef __cplusplus
}
#endif
#endif
