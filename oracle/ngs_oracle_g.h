/* ngs_oracle_g.h — CPU restatement of the search path for a gram size g (1..3) and for
 * UTF-32 strings: the checker of the indexG / indexW extensions.
 *
 * TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline). PARITY UNPINNED beyond g = 3 on
 * byte strings: the reference has no such path. Pinned by self-consistency with ngs_oracle.c
 * (g = 3, bytes), see ngs_oracle_g.c.
 *
 * Strings are arrays of uint32_t characters ending with 0. `wide` = 0: characters are bytes
 * (0..255) normalised as narrow strings; `wide` = 1: UTF-32 code points (indexW rules).
 */
#ifndef NGS_ORACLE_G_H
#define NGS_ORACLE_G_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ngog_index ngog_index;

ngog_index* ngog_build(const uint32_t* const* words, uint64_t size, uint16_t rowSize, const float* weight,
                       uint32_t g, int wide);
void ngog_free(ngog_index* ix);
int ngog_indexed(const ngog_index* ix);
uint64_t ngog_size(const ngog_index* ix);
uint64_t ngog_libsize(const ngog_index* ix);
uint32_t ngog_nkeys(const ngog_index* ix);
const uint32_t* ngog_key(const ngog_index* ix, uint32_t key, uint32_t* len);
void ngog_set_valid(ngog_index* ix, const char* chars, int n);
uint32_t ngog_search(const ngog_index* ix, const uint32_t* query, float threshold, uint32_t limit,
                     uint32_t* out_keys, float* out_scores, uint32_t cap);
void ngog_search_batch(const ngog_index* ix, const uint32_t* const* queries, uint32_t n, float threshold,
                       uint32_t limit, uint32_t* out_counts, uint32_t* out_keys, float* out_scores,
                       uint32_t cap, int threads);

#ifdef __cplusplus
}
#endif
#endif
