/* ngram_search.h — C ABI of libngram_search.so, the MI355X-native n-gram fuzzy search engine.
 *
 * Drop-in boundary: the first eight entry points have exactly the signatures, argument
 * meaning, ownership rules and error behaviour of the reference DLL's exports
 * (serena-yu17/StringSearchLib, nGramSearch/dllmain.cpp; line numbers below). A host that
 * binds the reference through its C ABI binds this library unchanged.
 *
 * The search path runs on the GPU: queries are normalised, hashed into 3-grams, matched
 * against gram -> term posting lists kept as CSR in HBM, counted in a u4 count-sketch in LDS
 * (candidates resolved exactly; exact LDS hash counting where the sketch cannot decide),
 * weighted, merged per key and cut to `limit` by HIP kernels for gfx950. indexN interns the
 * strings and builds the CSR on the GPU (ngs_intern.hip, ngs_build.hip; for gram dictionaries of
 * other gram sizes the GPU also finds the distinct gram keys and the host lays out only their
 * lookup table) and keeps it resident. There is no CPU search fallback: if no
 * GPU is usable, indexN prints the HIP error and returns 0.
 *
 * Threading: one global reader/writer lock, as the reference (dllmain.cpp:22). indexN and
 * dispose are exclusive; everything else may run concurrently (each call takes its own
 * stream and scratch from the handle's pool).
 */
#ifndef NGRAM_SEARCH_H
#define NGRAM_SEARCH_H

#include <stddef.h>
#include <stdint.h>
#include <wchar.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGS_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------
 * Reference exports (nGramSearch/dllmain.cpp), identical signatures.
 * ------------------------------------------------------------------------------------ */

/* dllmain.cpp:37. Index `size` words laid out as rows of `rowSize` (first word of a row =
 * master key, the rest aliases). `weight` (may be NULL) is indexed by FLAT word index;
 * weight 0 drops the pair. Returns the smallest free handle >= 1; 0 on failure. A
 * library with size < 2 or words == NULL yields a handle whose searches return 0. */
NGS_API uint32_t indexN(char** words, uint64_t size, uint16_t rowSize, float* weight);

/* dllmain.cpp:61. Like score() without the scores array. */
NGS_API uint32_t search(uint32_t handle, const char* query, char*** results, float threshold,
                        uint32_t limit);

/* dllmain.cpp:82. Top-`limit` master keys for `query` (limit 0 = unlimited) whose match
 * ratio passes `threshold`, sorted by score desc then key length asc. *results receives a
 * new[]'d array of pointers to index-owned key strings (valid until dispose), *scores a
 * new[]'d float array; free both with release(). Returns the count. Unknown handle or
 * un-built index: returns 0 and leaves *results / *scores untouched. */
NGS_API uint32_t score(uint32_t handle, const char* query, char*** results, float** scores,
                       float threshold, uint32_t limit);

/* dllmain.cpp:98. delete[]s arrays returned by search/score/searchBatch/scoreBatch. */
NGS_API void release(uint32_t handle, char** results, float* scores);

/* dllmain.cpp:110. Frees the index (host and device). Unknown handles are ignored. */
NGS_API void dispose(uint32_t handle);

/* dllmain.cpp:120. Number of distinct normalised terms (wordMap.size()). */
NGS_API uint64_t getSize(uint32_t handle);

/* dllmain.cpp:133. Number of distinct 3-grams over the long terms (ngrams.size()). */
NGS_API uint64_t getLibSize(uint32_t handle);

/* dllmain.cpp:142. Replaces the set of bytes kept by query normalisation (others become
 * spaces) for later searches. The index itself keeps the default set it was built with. */
NGS_API void setValidChar(uint32_t handle, char* characters, int n);

/* ------------------------------------------------------------------------------------
 * Batch extensions (BASELINE.json north_star: "the batched search() scoring loop").
 * Same semantics as score()/search() for each query; one GPU pass for the whole batch.
 * counts[i] = results of query i; *results / *scores are ONE flat new[]'d array each,
 * query i's results starting at sum(counts[0..i)). Returns the total; free with release().
 * Unknown handle / un-built index: returns 0, counts zeroed, outputs untouched.
 * ------------------------------------------------------------------------------------ */
NGS_API uint32_t scoreBatch(uint32_t handle, const char* const* queries, uint32_t nQueries,
                            float threshold, uint32_t limit, uint32_t* counts, char*** results,
                            float** scores);
NGS_API uint32_t searchBatch(uint32_t handle, const char* const* queries, uint32_t nQueries,
                             float threshold, uint32_t limit, uint32_t* counts, char*** results);

/* ------------------------------------------------------------------------------------
 * Gram-size and wide-string extensions (BASELINE config 4; Readme.md:47,91,135,170,190,208
 * documents indexW/searchW/releaseW/disposeW/getSizeW/getLibSizeW with a gSize parameter,
 * but the reference code has neither — parity self-consistent only).
 * Handles are shared with the narrow API; wchar_t is 4 bytes (UTF-32) on Linux.
 * Every threshold of the reference scales with g: terms of length >= 2g are gram-indexed,
 * queries shorter than 3g also run the edit-distance search, queries of <= g characters
 * scan the whole library, a query of m characters has m - g + 1 grams.
 * Wide normalisation: code points < 128 follow the byte rules (validChar, toupper);
 * code points >= 128 are kept as they are; values > 0x10FFFF become spaces.
 * ------------------------------------------------------------------------------------ */

/* indexN with grams of gSize (1..3) bytes; gSize 3 is indexN. Returns 0 for other gSize. */
NGS_API uint32_t indexG(char** words, uint64_t size, uint16_t rowSize, float* weight, uint16_t gSize);
/* Wide index (Readme.md:91): words are NUL-terminated UTF-32 strings; gSize 1..3. */
NGS_API uint32_t indexW(wchar_t** words, uint64_t size, uint16_t rowSize, float* weight, uint16_t gSize);
/* Wide search/score (Readme.md:135) on an indexW handle; result strings are index-owned
 * wchar_t keys. Return 0 on a narrow handle (and the narrow calls return 0 on a wide one). */
NGS_API uint32_t searchW(uint32_t handle, const wchar_t* query, wchar_t*** results, float threshold,
                         uint32_t limit);
NGS_API uint32_t scoreW(uint32_t handle, const wchar_t* query, wchar_t*** results, float** scores,
                        float threshold, uint32_t limit);
NGS_API uint32_t scoreBatchW(uint32_t handle, const wchar_t* const* queries, uint32_t nQueries,
                             float threshold, uint32_t limit, uint32_t* counts, wchar_t*** results,
                             float** scores);
NGS_API uint32_t searchBatchW(uint32_t handle, const wchar_t* const* queries, uint32_t nQueries,
                              float threshold, uint32_t limit, uint32_t* counts, wchar_t*** results);
/* Readme.md:170,190,208,226 — same meaning as release/dispose/getSize/getLibSize. */
NGS_API void releaseW(uint32_t handle, wchar_t** results, float* scores);
NGS_API void disposeW(uint32_t handle);
NGS_API uint64_t getSizeW(uint32_t handle);
NGS_API uint64_t getLibSizeW(uint32_t handle);

/* ------------------------------------------------------------------------------------
 * Device-level extensions: inputs and outputs stay in HBM (bench, multi-GPU sharding,
 * host frameworks that already hold device buffers). Not in the reference.
 * ------------------------------------------------------------------------------------ */

/* Selects the HIP device that the calling thread's next indexN builds on (default: the
 * current HIP device). Same as ngsSetDevices(&device, 1). Returns 0, or a negative HIP error code. */
NGS_API int ngsSetDevice(int device);
/* Multi-GPU (BASELINE north_star: "one-shard-per-GPU across the node"): the calling thread's next
 * indexN / indexG / indexW places one replica of the index on each of the n devices (repeats
 * allowed; n = 0 restores the default). score/search/scoreBatch/searchBatch on such a handle
 * split a batch of at least 4,096 queries per replica into contiguous slices, one per replica,
 * scored concurrently (one host thread and stream each) and joined in query order: the results
 * are those of one device. ngsSearchDevice uses the replica on the caller's current device
 * (-3 if the index has none there).
 * Returns 0, or a negative HIP error code (nothing changed). */
NGS_API int ngsSetDevices(const int* devices, int n);
/* Replicas of the index (devices it was placed on); -1 for an unknown handle. */
NGS_API int ngsReplicaCount(uint32_t handle);
NGS_API int ngsDeviceCount(void);

/* Number of master keys; key ids used by ngsSearchDevice are 0..n-1. */
NGS_API uint32_t ngsNumKeys(uint32_t handle);
/* NUL-terminated, index-owned string of key `keyId` (NULL if out of range or if the
 * index's character width differs: ngsKey for narrow indexes, ngsKeyW for indexW). */
NGS_API const char* ngsKey(uint32_t handle, uint32_t keyId);
NGS_API const wchar_t* ngsKeyW(uint32_t handle, uint32_t keyId);
/* Character width in bytes (1 or 4) and gram size of the index; 0 for an unknown handle. */
NGS_API uint32_t ngsCharSize(uint32_t handle);
NGS_API uint32_t ngsGramSize(uint32_t handle);

/* Scores nQueries queries held on the handle's device: query i is the raw bytes
 * dQueryBytes[dQueryOffsets[i] .. dQueryOffsets[i+1]) (no NUL needed; for an indexW handle
 * the bytes are UTF-32 characters and the offsets multiples of 4). Writes, for query i,
 * dCounts[i] results to dKeys/dScores[i*outStride ...]; outStride must be >=
 * min(limit ? limit : 2^31-1, ngsNumKeys). `stream` is the caller's hipStream_t (NULL = the
 * null stream): the call's kernels are ordered after the work already queued on it, and the
 * call returns when the results are complete.
 * Returns 0, or a negative error (-1 bad handle, -2 un-built index, -3 bad argument,
 * -4 HIP failure, -5 internal error flagged by a kernel, e.g. an exhausted LDS table). */
NGS_API int ngsSearchDevice(uint32_t handle, const uint8_t* dQueryBytes, const uint64_t* dQueryOffsets,
                            uint32_t nQueries, float threshold, uint32_t limit, uint32_t outStride,
                            uint32_t* dCounts, uint32_t* dKeys, float* dScores, void* stream);

/* Asynchronous ngsSearchDevice: the call is ordered after the work already queued on `stream`,
 * runs on streams of its own and returns once it is queued, with a ticket. The results are
 * complete when ngsSearchDeviceWait(handle, ticket) returns 0 (it waits, runs the library-wide
 * path for the rare queries that need it and records the statistics); every ticket must be
 * waited for once, and the output buffers must not be read or reused before. Calls in flight
 * together overlap on the GPU (a batch's tail beside the next batch's counting). Return codes
 * as ngsSearchDevice; Wait answers -3 for an unknown ticket. dispose() waits for calls in flight. */
NGS_API int ngsSearchDeviceAsync(uint32_t handle, const uint8_t* dQueryBytes, const uint64_t* dQueryOffsets,
                                 uint32_t nQueries, float threshold, uint32_t limit, uint32_t outStride,
                                 uint32_t* dCounts, uint32_t* dKeys, float* dScores, void* stream,
                                 uint64_t* ticket);
NGS_API int ngsSearchDeviceWait(uint32_t handle, uint64_t ticket);

/* Low-latency score()/search() (narrow indexes): a persistent one-wave server kernel answers
 * single queries from a request block in pinned host memory, with no kernel launch, copy or
 * stream wait per call. It serves libraries small enough that one wave searches a query (fewer
 * than 16 skip buckets; large libraries keep the sliced latency path) and limits up to 128; other
 * calls take the regular path. It starts by itself on such a library after the 4th score()/
 * search() call; ngsServe(h, 1) starts it at once, ngsServe(h, 0) stops it and turns the automatic
 * start off. The kernel leaves after 200 ms without a request (or 10 s of life) and is relaunched
 * on the next call; a batch call (scoreBatch/searchBatch of more than 16 queries, the device entry
 * points) stops it first and keeps it stopped until the batch is done, so no batch kernel queues
 * behind it; dispose() stops it. Answers are the regular path's, bit for bit. One request at a
 * time per handle: a call that finds the server busy takes the regular path. Returns 0, -1 (bad
 * handle), -2 (unbuilt index), -3 (wide index), -4 (HIP error). */
NGS_API int ngsServe(uint32_t handle, int enable);
/* Packs a device result block in ngsSearchDevice's layout (counts[n], query i's records at
 * i * stride) on `stream`: dOffsets[n + 1] = exclusive prefix sum of the counts (dOffsets[n] = total
 * records) and dRecords[2 * total] = {key id, fp32 score bits} per record in query order. Used by the
 * multi-GPU gather (stringsearchlib_amd/shard.py) so that the bytes sent to rank 0 follow the
 * results, not n x stride. Returns 0, -3 (bad argument), -4 (HIP error). */
NGS_API int ngsPackResults(const uint32_t* dCounts, const uint32_t* dKeys, const float* dScores, uint32_t n,
                           uint32_t stride, uint32_t* dOffsets, uint32_t* dRecords, void* stream);

/* The server of `handle`: 0 none, 1 set up but its kernel not running, 2 its kernel running; -1
 * bad handle (tests). */
NGS_API int ngsServeState(uint32_t handle);

/* Per-call statistics of the last search on `handle` (enable timing first). */
typedef struct {
    uint64_t queries;          /* queries in the call */
    uint64_t fast_queries;     /* handled by the fused LDS kernel */
    uint64_t general_queries;  /* handled by the dense library-wide kernels */
    uint64_t postings;         /* posting ids read by the LDS kernels (k_wave: per gram occurrence) */
    uint64_t lists;            /* posting lists opened */
    uint64_t results;          /* results written by the fused kernel */
    uint64_t survivors;        /* terms whose match ratio passed the threshold (fused kernel) */
    double fast_kernel_ms;     /* fused kernel time from HIP events on the call's stream */
    double prep_kernel_ms;     /* normalisation kernel time */
    double general_ms;         /* general path time (all its kernels) */
    uint64_t handover_queries; /* queries the lean tier-1a kernel handed to the full tier-1b kernel */
    uint64_t tier2_queries;    /* queries routed to the block-per-query tier-2 kernel */
    uint64_t heavy_queries;    /* listed by the prep kernel as heavy (cmin 2: lean kernel on a side stream) */
    uint64_t full_queries;     /* listed by the prep kernel for tier 1b from the start (cmin 1, short search) */
    uint64_t slot_full_queries; /* handed to tier 1b because their survivor slots were full (the
                                   context's slots grow for later calls) */
    uint64_t survivor_slots;   /* survivor slots per query the call ran with */
    uint64_t survivor_slot_bytes; /* bytes of survivor slots and arena the call's context held (rows x
                                     slots x 5 + arena blocks x 1,024 x 5; the slots at most 16 GiB,
                                     and grown slots go back after 16 calls in a row that fill none) */
    uint64_t main_postings;    /* postings and lists of the queries the main tier-1a launch finished */
    uint64_t main_lists;
    uint64_t arena_blocks;     /* survivor arena: blocks (1,024 survivors each) the call's context holds
                                  (queries whose survivors outgrow their slots go on there) */
    uint64_t arena_used;       /* ... blocks the call took (past arena_blocks: it ran out, those
                                  queries went to tier 1b, and later calls get a larger arena) */
} ngs_stats;
NGS_API int ngsSetTiming(uint32_t handle, int enable);
/* The last failure of a call on this thread (0: none); clear != 0 resets it. A HIP error code, or
 * NGS_ERR_INTERNAL (a kernel reported an internal error, the -5 of the device entry points) or
 * NGS_ERR_QUERY_BUFFER (a batch outgrew the normalised-query buffer on its rerun). A batch split
 * across replicas hands a replica thread's failure to the calling thread. The reference entry
 * points answer 0 on failure, indistinguishable from "no results": a caller that must tell them
 * apart asks here afterwards. */
#define NGS_ERR_INTERNAL 0x10001
#define NGS_ERR_QUERY_BUFFER 0x10002
NGS_API int ngsLastError(int clear);
NGS_API int ngsLastStats(uint32_t handle, ngs_stats* out);

/* Test support: digests of the index as the kernels read it, for comparing the GPU index build
 * (default) with the host build (environment NGS_HOST_GRAMS=1 / NGS_HOST_INTERN=1 at build time).
 * out[0..7] = postings, lists, skip buckets, FNV-1a of gram_off, post, gram_row, skip, bucket span
 * (zeros for dictionary indexes: gram sizes other than narrow 3); out[8..15] = FNV-1a of term_off,
 * term_bytes, tk_off, tk, key_off, key_bytes, wildcard keys, wildcard scores; out[16] = shape flags
 * (1 keys unique, 2 one pair per term, 4 term ids in key-rank order, 8 rank lists: the threshold-0
 * shortcut of indexes with one weight, DevIndex.rank_post). Returns min(n, 17),
 * -1 (bad handle), -4 (HIP error). */
NGS_API int ngsIndexDigest(uint32_t handle, uint64_t* out, int n);
/* The same digests of replica `replica` (0 .. ngsReplicaCount - 1): every replica of an index
 * placed on several devices holds the same arrays. -1 for a bad handle or replica. */
NGS_API int ngsReplicaDigest(uint32_t handle, int replica, uint64_t* out, int n);

/* Index files (an extension; the reference rebuilds on every indexN): ngsSaveIndex writes the
 * interned library of `handle` (terms, term -> (key, weight) pairs, keys, wildcard weights,
 * the validChar set) to `path`: 0, or -1 (bad handle), -2 (unbuilt index), -3 (I/O), -4 (HIP
 * error). ngsLoadIndex builds an index from such a file like indexN builds one from words (the
 * gram CSR is rebuilt; the devices of ngsSetDevices apply): its handle, or 0 if the file cannot
 * be read, is not an index file or is inconsistent. A loaded index answers exactly like the
 * saved one. */
NGS_API int ngsSaveIndex(uint32_t handle, const char* path);
NGS_API uint32_t ngsLoadIndex(const char* path);

/* Library build identification: "ngram_search <version> gfx950 src=<hash>", where <hash> is the
 * first 16 hex digits of the SHA-256 of the sources the library was compiled from. */
NGS_API const char* ngsVersion(void);

/* Diagnostics: the host batch path's phases (scoreBatch / searchBatch / batch score paths of more
 * than 16 queries), nanoseconds summed over the calls since the last reset: [0] query packing,
 * [1] copies in + kernels queued, [2] kernels waited for, [3] device pack + offsets back,
 * [4] records back + marshalling, [5] whole calls, [6] number of calls; [7] the number of
 * one-stream batch calls (all queries heavy, at most 16,384) replayed from a captured graph,
 * any entry point. Writes min(n, 8) values, resets them all if `reset`, returns 8. */
NGS_API int ngsHostPhases(uint64_t* out, int n, int reset);

/* Diagnostics: per-phase time of the LDS kernels (s_memtime shader-clock ticks, summed over
 * waves / blocks) in the instrumented build libngram_search_prof.so; -1 in the regular build. */
NGS_API int ngsPhaseStats(uint64_t* out, int n, int reset);

#ifdef __cplusplus
}
#endif
#endif /* NGRAM_SEARCH_H */
