/*
 * vectorscan_amd_hs.h — the pure-literal database API over the GPU literal
 * matcher: hs_compile_lit_multi / hs_scan / hs_scan_vector / streams, as
 * the reference runs them when a database holds only pure literals
 * (ROSE_RUNTIME_PURE_LITERAL, src/rose/rose_build_bytecode.cpp:258-303).
 *
 * Each entry point mirrors the reference function named beside it (same
 * arguments, return codes and callback contract); a maintainer binds the
 * reference's names to these.  Matches are found by the
 * HWLM scan of vectorscan_amd.h (one GPU launch per call: per write for a
 * stream, all pieces of a vector at once) and delivered in the reference
 * order: increasing `to`; at one `to`, literal fragments in HWLM confirm
 * order, then patterns in compile order.
 *
 * Host buffers are copied to the GPU on every call; for device-resident
 * corpora use vsa_scan_blocks* directly.
 */
#ifndef VECTORSCAN_AMD_HS_H
#define VECTORSCAN_AMD_HS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* hs_common.h:478-584 */
#define VSA_HS_SUCCESS 0
#define VSA_HS_INVALID (-1)
#define VSA_HS_NOMEM (-2)
#define VSA_HS_SCAN_TERMINATED (-3)
#define VSA_HS_COMPILER_ERROR (-4)
#define VSA_HS_DB_VERSION_ERROR (-5)
#define VSA_HS_DB_PLATFORM_ERROR (-6)
#define VSA_HS_DB_MODE_ERROR (-7)
#define VSA_HS_SCRATCH_IN_USE (-10)
#define VSA_HS_UNKNOWN_ERROR (-13)

/* hs_compile.h:869-1005, 1156-1171 */
#define VSA_HS_FLAG_CASELESS 1u
#define VSA_HS_FLAG_DOTALL 2u
#define VSA_HS_FLAG_MULTILINE 4u
#define VSA_HS_FLAG_SINGLEMATCH 8u
#define VSA_HS_FLAG_ALLOWEMPTY 16u
#define VSA_HS_FLAG_UTF8 32u
#define VSA_HS_FLAG_UCP 64u
#define VSA_HS_FLAG_PREFILTER 128u
#define VSA_HS_FLAG_SOM_LEFTMOST 256u
#define VSA_HS_FLAG_COMBINATION 512u
#define VSA_HS_FLAG_QUIET 1024u
#define VSA_HS_MODE_BLOCK 1u
#define VSA_HS_MODE_STREAM 2u
#define VSA_HS_MODE_VECTORED 4u
#define VSA_HS_MODE_SOM_HORIZON_LARGE (1u << 24)
#define VSA_HS_MODE_SOM_HORIZON_MEDIUM (1u << 25)
#define VSA_HS_MODE_SOM_HORIZON_SMALL (1u << 26)

typedef struct vsa_hs_database vsa_hs_database_t;
typedef struct vsa_hs_scratch vsa_hs_scratch_t;
typedef struct vsa_hs_stream vsa_hs_stream_t;

/* hs_compile_error_t, hs_compile.h:112-130 */
typedef struct {
    char *message;
    int expression;
} vsa_hs_compile_error_t;

/* match_event_handler, hs_runtime.h:125-128: nonzero stops matching */
typedef int (*vsa_hs_match_event_handler)(unsigned int id, unsigned long long from,
                                          unsigned long long to, unsigned int flags,
                                          void *context);

/* hs_compile_lit_multi, hs_compile.h:690-697 (checks of hs.cpp:290-400 and
 * compiler.cpp:391-433).  `platform` is accepted for signature parity and
 * ignored. */
int vsa_hs_compile_lit_multi(const char *const *expressions, const unsigned *flags,
                             const unsigned *ids, const size_t *lens, unsigned elements,
                             unsigned mode, const void *platform, vsa_hs_database_t **db,
                             vsa_hs_compile_error_t **error);
/* hs_compile_lit, hs_compile.h:608-611 */
int vsa_hs_compile_lit(const char *expression, unsigned flags, size_t len, unsigned mode,
                       const void *platform, vsa_hs_database_t **db,
                       vsa_hs_compile_error_t **error);
int vsa_hs_free_compile_error(vsa_hs_compile_error_t *error); /* hs_compile.h:710 */
int vsa_hs_free_database(vsa_hs_database_t *db);              /* hs_common.h:80 */

/* hs_alloc_scratch / hs_free_scratch, hs_runtime.h:555 / :609: one scratch per
 * thread; it holds a GPU context and the device copies of the databases it
 * was allocated for. */
int vsa_hs_alloc_scratch(const vsa_hs_database_t *db, vsa_hs_scratch_t **scratch);
int vsa_hs_free_scratch(vsa_hs_scratch_t *scratch);

/* hs_scan, hs_runtime.h:479-482 (runtime.c:316-470; pureLiteralBlockExec
 * runtime.c:204-230) */
int vsa_hs_scan(const vsa_hs_database_t *db, const char *data, unsigned int length,
                unsigned int flags, vsa_hs_scratch_t *scratch,
                vsa_hs_match_event_handler onEvent, void *context);
/* hs_scan_vector, hs_runtime.h:522-527 (runtime.c:1106-1180): all pieces
 * in one GPU launch, each a stream write with the previous pieces as
 * history */
int vsa_hs_scan_vector(const vsa_hs_database_t *db, const char *const *data,
                       const unsigned int *length, unsigned int count, unsigned int flags,
                       vsa_hs_scratch_t *scratch, vsa_hs_match_event_handler onEvent,
                       void *context);

/* streams: hs_open_stream / hs_scan_stream / hs_close_stream /
 * hs_reset_stream, hs_runtime.h:148, :188, :232, :273 (runtime.c:560-1000, pureLiteralStreamExec
 * runtime.c:802-831) */
int vsa_hs_open_stream(const vsa_hs_database_t *db, unsigned int flags,
                       vsa_hs_stream_t **stream);
int vsa_hs_scan_stream(vsa_hs_stream_t *id, const char *data, unsigned int length,
                       unsigned int flags, vsa_hs_scratch_t *scratch,
                       vsa_hs_match_event_handler onEvent, void *ctxt);
int vsa_hs_close_stream(vsa_hs_stream_t *id, vsa_hs_scratch_t *scratch,
                        vsa_hs_match_event_handler onEvent, void *ctxt);
int vsa_hs_reset_stream(vsa_hs_stream_t *id, unsigned int flags, vsa_hs_scratch_t *scratch,
                        vsa_hs_match_event_handler onEvent, void *context);

/* hsbench's corpus loop (tools/hsbench/main.cpp:487-511 block mode,
 * :520-600 streaming / vectored) in ONE launch over device-resident blocks
 * (d_data on the scratch's device).  Block database: each block is one
 * hs_scan.  Stream / vectored database: blocks sharing a stream_ids value
 * are, in array order, the writes of one stream and lie back to back in
 * d_data.  counts[nblocks] (optional) gets each block's match count, *total
 * their sum (matches as delivered to a callback: after long-literal checks,
 * exhaustion and dedupe).  h_data = host copy of the same bytes, required
 * only when some literal is longer than 8 bytes; `threads` host threads
 * replay the records where one record is not exactly one match. */
int vsa_hs_scan_corpus(const vsa_hs_database_t *db, vsa_hs_scratch_t *scratch,
                       const uint8_t *d_data, const uint8_t *h_data, const uint64_t *offsets,
                       const uint64_t *lens, const uint32_t *stream_ids, uint32_t nblocks,
                       uint64_t *counts, uint64_t *total, unsigned threads);

/* The same corpus prepared once (launch plan on the device, stream
 * grouping on the host) and scanned many times, as hsbench's repeats do.
 * The scratch must stay allocated (and not be used concurrently) for the
 * corpus's life. */
typedef struct vsa_hs_corpus vsa_hs_corpus_t;
int vsa_hs_corpus_prepare(const vsa_hs_database_t *db, vsa_hs_scratch_t *scratch,
                          const uint8_t *d_data, const uint8_t *h_data,
                          const uint64_t *offsets, const uint64_t *lens,
                          const uint32_t *stream_ids, uint32_t nblocks,
                          vsa_hs_corpus_t **corpus);
int vsa_hs_corpus_scan(vsa_hs_corpus_t *corpus, uint64_t *counts, uint64_t *total,
                       unsigned threads);
/* As vsa_hs_corpus_scan, plus digests[nblocks] (optional): per block, the
 * fold of vsa_hs_seq_digest_step over its callback sequence (id, from, to)
 * in delivery order, from 0 -- an order-dependent fingerprint of exactly
 * what hs_scan / hs_scan_stream would have delivered for that block. */
int vsa_hs_corpus_scan_ex(vsa_hs_corpus_t *corpus, uint64_t *counts, uint64_t *digests,
                          uint64_t *total, unsigned threads);
/* hsbench's repeat loop: `repeats` scans of the corpus, pass k + 1 on the
 * GPU while the host replays pass k (the report program of the records
 * that do not map one to one onto matches).  totals[repeats] = the matches
 * of each pass; counts / digests (optional, as vsa_hs_corpus_scan_ex) are
 * those of the last pass. */
int vsa_hs_corpus_scan_repeats(vsa_hs_corpus_t *corpus, uint32_t repeats, uint64_t *totals,
                               uint64_t *counts, uint64_t *digests, unsigned threads);
static inline uint64_t vsa_hs_seq_digest_step(uint64_t h, unsigned id, unsigned long long from,
                                              unsigned long long to) {
    uint64_t x = h ^ ((uint64_t)id * 0x9E3779B97F4A7C15ULL) ^
                 ((uint64_t)from * 0xC2B2AE3D27D4EB4FULL) ^ ((uint64_t)to * 0x165667B19E3779F9ULL);
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ULL;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
int vsa_hs_corpus_free(vsa_hs_corpus_t *corpus);

/* Streams, continued: hs_copy_stream / hs_reset_and_copy_stream
 * (hs_runtime.h:291 / :324, runtime.c:713-779) and hs_stream_size
 * (hs_common.h:183). */
int vsa_hs_copy_stream(vsa_hs_stream_t **to_id, const vsa_hs_stream_t *from_id);
int vsa_hs_reset_and_copy_stream(vsa_hs_stream_t *to_id, const vsa_hs_stream_t *from_id,
                                 vsa_hs_scratch_t *scratch, vsa_hs_match_event_handler onEvent,
                                 void *context);
int vsa_hs_stream_size(const vsa_hs_database_t *db, size_t *stream_size);

/* Scratch, continued: hs_clone_scratch / hs_scratch_size (hs_runtime.h:576
 * / :593).  A clone has its own GPU context and database copies. */
int vsa_hs_clone_scratch(const vsa_hs_scratch_t *src, vsa_hs_scratch_t **dest);
int vsa_hs_scratch_size(const vsa_hs_scratch_t *scratch, size_t *scratch_size);

/* hs_valid_platform / hs_version (hs_common.h:463 / :446) */
int vsa_hs_valid_platform(void);
const char *vsa_hs_version(void);

/* Serialized databases in the reference's envelope (database.c:61-455):
 * 32 header bytes (magic 0xdbdbdbdb, HS_VERSION_32BIT of 5.4.11, bytecode
 * length, platform, CRC-32C), the bytecode, zero padding to 104 + length
 * bytes.  The bytecode opens with the RoseEngine fields the reference reads
 * without running it (pureLiteral, runtimeImpl = PURE_LITERAL, mode at
 * byte 12), then this engine's pattern list, which deserializing compiles
 * again.  A reference-serialized database (a full RoseEngine) is refused
 * with VSA_HS_DB_PLATFORM_ERROR; hs_serialized_database_info reads either.
 * `bytes` / `info` are malloc'ed (the reference's default allocator). */
int vsa_hs_serialize_database(const vsa_hs_database_t *db, char **bytes, size_t *length);
int vsa_hs_deserialize_database(const char *bytes, size_t length, vsa_hs_database_t **db);
int vsa_hs_serialized_database_size(const char *bytes, size_t length, size_t *deserialized_size);
int vsa_hs_database_size(const vsa_hs_database_t *db, size_t *database_size);
int vsa_hs_serialized_database_info(const char *bytes, size_t length, char **info);
int vsa_hs_database_info(const vsa_hs_database_t *db, char **info);

/* Introspection for tests: the database's HWLM blob (fragment id = HWLM
 * literal id) and the number of literal fragments. */
int vsa_hs_database_hwlm(const vsa_hs_database_t *db, const void **hwlm, size_t *size,
                         unsigned *fragments);

#ifdef __cplusplus
}
#endif

#endif
