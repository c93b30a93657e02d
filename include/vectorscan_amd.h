/*
 * vectorscan_amd.h — C ABI of libvectorscan_amd.so, the MI355X engine for
 * Vectorscan's literal / char-class prefilter hot path.
 *
 * Part 1 is the drop-in boundary: the same names, signatures and semantics
 * as the reference entry points it replaces, so Rose (or the reference's
 * own unit tests) link against it unchanged.  Part 2 is the new device-batch
 * API (64-bit lengths, device-resident buffers, many blocks per launch)
 * that hsbench-style drivers and multi-GPU striping use.  Part 3 builds HWLM
 * bytecode in the reference layout.
 *
 * No torch or HIP types appear in any signature; streams are void*.
 */
#ifndef VECTORSCAN_AMD_H
#define VECTORSCAN_AMD_H

#include <stddef.h>
#include <stdint.h>

#if defined(__x86_64__) || defined(__i386__)
#include <emmintrin.h>
typedef __m128i vsa_m128_t; /* passed in XMM registers, as the reference's m128 */
#else
typedef struct { uint8_t b[16]; } __attribute__((aligned(16))) vsa_m128_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ *
 * Part 1 — drop-in entry points (reference file:line of the interface)
 * ------------------------------------------------------------------ */

struct HWLM;
struct FDR;
struct noodTable;
struct hs_scratch;
union AccelAux;

typedef int hwlm_error_t;             /* hwlm.h:57 */
typedef uint64_t hwlm_group_t;        /* hwlm.h:60 */
typedef hwlm_group_t hwlmcb_rv_t;     /* hwlm.h:63 */
/* hwlm.h:98 */
typedef hwlmcb_rv_t (*HWLMCallback)(size_t end, uint32_t id,
                                    struct hs_scratch *scratch);

/* The GPU entry points under their own names (same arguments and results
 * as hwlmExec, hwlmExecStreaming, fdrExec, noodExec above), for a build
 * that keeps the reference's definitions and routes each call by its
 * length. */
hwlm_error_t vsa_gpu_hwlmExec(const struct HWLM *tab, const uint8_t *buf, size_t len,
                              size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                              hwlm_group_t groups);
hwlm_error_t vsa_gpu_hwlmExecStreaming(const struct HWLM *tab, size_t len, size_t start,
                                       HWLMCallback cb, struct hs_scratch *scratch,
                                       hwlm_group_t groups);
hwlm_error_t vsa_gpu_fdrExec(const struct FDR *fdr, const uint8_t *buf, size_t len,
                             size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                             hwlm_group_t groups);
hwlm_error_t vsa_gpu_noodExec(const struct noodTable *n, const uint8_t *buf, size_t len,
                              size_t start, HWLMCallback cb, struct hs_scratch *scratch);

/* Registration of an immutable bytecode blob for the drop-ins: between
 * vsa_hwlm_register(blob) and vsa_hwlm_unregister(blob) the bytes at blob
 * do not change, so the drop-ins' device-copy cache serves them without
 * comparing the whole blob on every call (unregistered blobs are compared,
 * ~20 us per call for a 0.4 MB FDR blob).  bare_type -1: an HWLM
 * (hwlmExec / hwlmExecStreaming); 12 (HWLM_ENGINE_FDR) / 16
 * (HWLM_ENGINE_NOOD): a bare FDR or noodle engine (fdrExec / noodExec
 * pointers).  The reference-side call sites are where the database is
 * loaded and freed. */
int vsa_hwlm_register(const void *blob, int bare_type);
int vsa_hwlm_unregister(const void *blob);

/* Batching service for concurrent drop-in calls (many host threads, each
 * scanning its blocks through hwlmExec: rose/block.c:259, hsbench -T).  A
 * worker thread with its own GPU context takes the calls that arrive within
 * window_us of each other (at most max_batch), stages their buffers in one
 * DMA and scans them as the blocks of one launch; each caller then gets its
 * records replayed through its own callback on its own thread, with
 * hwlmExec's contract (same order, groups / NOREPEAT / squash / flood).
 * vsa_batcher_hwlmExec blocks until the caller's matches are delivered.
 * The accel pre-skip is not applied on this path (it only moves `start`).
 * vsa_batcher_stats: launches so far and calls served by them. */
typedef struct vsa_batcher vsa_batcher_t;
int vsa_batcher_create(int device, uint32_t max_batch, uint32_t window_us, vsa_batcher_t **b);
int vsa_batcher_destroy(vsa_batcher_t *b);
int vsa_batcher_stats(vsa_batcher_t *b, uint64_t *batches, uint64_t *calls);
hwlm_error_t vsa_batcher_hwlmExec(vsa_batcher_t *b, const struct HWLM *tab, const uint8_t *buf,
                                  size_t len, size_t start, HWLMCallback cb,
                                  struct hs_scratch *scratch, hwlm_group_t groups);

/* Replaces hwlmExec, src/hwlm/hwlm.h:116 (impl. src/hwlm/hwlm.c:178).
 * Copies buf to the GPU, scans, replays confirmed matches through cb in the
 * reference order (end, bucket, confirm-chain order) applying groups /
 * NOREPEAT / terminate / INCLUDED_JUMP squash exactly as confWithBit. */
hwlm_error_t hwlmExec(const struct HWLM *tab, const uint8_t *buf, size_t len,
                      size_t start, HWLMCallback callback,
                      struct hs_scratch *scratch, hwlm_group_t groups);

/* Replaces fdrExec, src/fdr/fdr.h:58 (impl. src/fdr/fdr.c:801). */
hwlm_error_t fdrExec(const struct FDR *fdr, const uint8_t *buf, size_t len,
                     size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                     hwlm_group_t groups);

/* Replaces noodExec, src/hwlm/noodle_engine.h:47 (impl. noodle_engine.cpp:123). */
hwlm_error_t noodExec(const struct noodTable *n, const uint8_t *buf, size_t len,
                      size_t start, HWLMCallback cb, struct hs_scratch *scratch);

/* Streaming (history + current buffer; ends relative to buf, literals may
 * begin up to hlen bytes into the history).  The 16 bytes before hbuf + hlen
 * must be readable, as the reference requires (fdr.c:835-841).
 * hwlmExecStreaming (hwlm.h:137, hwlm.c:207) reads buf / hbuf / hlen from
 * scratch->core_info (scratch.h:91-110; offsets: vsa_set_scratch_core_info).
 * fdrExecStreaming (fdr.h:75, fdr.c:827), noodExecStreaming
 * (noodle_engine.h:52, noodle_engine.cpp:136). */
hwlm_error_t hwlmExecStreaming(const struct HWLM *tab, size_t len, size_t start,
                               HWLMCallback callback, struct hs_scratch *scratch,
                               hwlm_group_t groups);
hwlm_error_t fdrExecStreaming(const struct FDR *fdr, const uint8_t *hbuf, size_t hlen,
                              const uint8_t *buf, size_t len, size_t start,
                              HWLMCallback cb, struct hs_scratch *scratch,
                              hwlm_group_t groups);
hwlm_error_t noodExecStreaming(const struct noodTable *n, const uint8_t *hbuf, size_t hlen,
                               const uint8_t *buf, size_t len, HWLMCallback cb,
                               struct hs_scratch *scratch);

/* Accel find-first / find-last (src/nfa/shufti.h:46-55, truffle.h:45-49,
 * vermicelli.hpp:47-95, accel.h:148).  Return values as the reference:
 * forward scans return buf_end when nothing is found, reverse scans
 * buf - 1.  These signatures have no error channel: on a device failure
 * they return the no-skip answer (buf forward, buf_end - 1 reverse, c for
 * run_accel) and vsa_last_error() reports VSA_E_DEVICE. */
const uint8_t *shuftiExec(vsa_m128_t mask_lo, vsa_m128_t mask_hi,
                          const uint8_t *buf, const uint8_t *buf_end);
const uint8_t *rshuftiExec(vsa_m128_t mask_lo, vsa_m128_t mask_hi,
                           const uint8_t *buf, const uint8_t *buf_end);
/* shufti.h:52-55; masks from shuftiBuildDoubleMasks (bit clear = member).
 * Reproduces the reference's per-block results for VECTORSIZE set by
 * vsa_set_accel_vector_size (default 64, the AVX-512 build), including the
 * matches at the last byte of each 16-byte lane it reports. */
const uint8_t *shuftiDoubleExec(vsa_m128_t mask1_lo, vsa_m128_t mask1_hi,
                                vsa_m128_t mask2_lo, vsa_m128_t mask2_hi,
                                const uint8_t *buf, const uint8_t *buf_end);
const uint8_t *truffleExec(vsa_m128_t mask1, vsa_m128_t mask2,
                           const uint8_t *buf, const uint8_t *buf_end);
const uint8_t *rtruffleExec(vsa_m128_t mask1, vsa_m128_t mask2,
                            const uint8_t *buf, const uint8_t *buf_end);
const uint8_t *vermicelliExec(char c, char nocase, const uint8_t *buf,
                              const uint8_t *buf_end);
const uint8_t *nvermicelliExec(char c, char nocase, const uint8_t *buf,
                               const uint8_t *buf_end);
const uint8_t *rvermicelliExec(char c, char nocase, const uint8_t *buf,
                               const uint8_t *buf_end);
const uint8_t *rnvermicelliExec(char c, char nocase, const uint8_t *buf,
                                const uint8_t *buf_end);
const uint8_t *vermicelliDoubleExec(char c1, char c2, char nocase,
                                    const uint8_t *buf, const uint8_t *buf_end);
const uint8_t *rvermicelliDoubleExec(char c1, char c2, char nocase, const uint8_t *buf,
                                     const uint8_t *buf_end);
const uint8_t *vermicelliDoubleMaskedExec(char c1, char c2, char m1, char m2,
                                          const uint8_t *buf,
                                          const uint8_t *buf_end);
const uint8_t *run_accel(const union AccelAux *accel, const uint8_t *c,
                         const uint8_t *c_end);

/* ------------------------------------------------------------------ *
 * Part 2 — device batch API (new)
 * ------------------------------------------------------------------ */

#define VSA_OK 0
#define VSA_E_INVALID (-1)
#define VSA_E_NOMEM (-2)
#define VSA_E_NOT_BUILDABLE (-3)
#define VSA_E_DEVICE (-4)
#define VSA_E_OVERFLOW (-5)

typedef struct vsa_ctx vsa_ctx_t; /* stream + workspace, one per thread */
typedef struct vsa_db vsa_db_t;   /* device copy of one HWLM blob */

/* Sorted confirmed match: end = key >> 24, bucket = (key >> 20) & 15,
 * LitInfo offset from its FDRConfirm in 8-byte units = key & 0xfffff (the
 * confirm-chain order); id = literal id. */
typedef struct {
    uint64_t key;
    uint32_t id;
    uint32_t pad;
} vsa_match_t;

int vsa_device_count(void);
int vsa_ctx_create(int device, vsa_ctx_t **ctx);
int vsa_ctx_destroy(vsa_ctx_t *ctx);
/* A second workspace on `base`'s device and stream: scans queued through
 * either run in queue order, so a pipelined caller (scan k + 1 queued before
 * waiting for scan k, VSA_SCAN_ASYNC) keeps one kernel at a time on the GPU
 * and clean per-scan kernel times.  The stream lives until the last context
 * using it is destroyed. */
int vsa_ctx_create_shared(vsa_ctx_t *base, vsa_ctx_t **ctx);
void *vsa_ctx_stream(vsa_ctx_t *ctx);
/* Leave n CUs free of the literal scan's persistent grid (one 1024-thread
 * workgroup per CU that fills the register file): plans built afterwards on
 * this context (per-call ones, and vsa_plan_create's) use num_cus - n
 * workgroups, so a kernel on another stream -- a multi-GPU step's RCCL
 * collective of the previous step -- finds a CU while the next scan runs
 * instead of queueing behind it.  Shared contexts inherit the value of the
 * context they are made from.  0 (default) uses every CU. */
int vsa_ctx_set_reserved_cus(vsa_ctx_t *ctx, int n);

/* Upload an HWLM blob (reference layout, 64-byte aligned host copy). */
int vsa_db_load(vsa_ctx_t *ctx, const void *hwlm, size_t size, vsa_db_t **db);
int vsa_db_free(vsa_db_t *db);
/* engine kind: 16 = noodle, 0 = FDR, 3..18 = Teddy engine id */
int vsa_db_engine(const vsa_db_t *db);

/* Device memory helpers (plain hipMalloc / hipMemcpy). */
int vsa_malloc(vsa_ctx_t *ctx, size_t bytes, void **dptr);
int vsa_free(vsa_ctx_t *ctx, void *dptr);
int vsa_memcpy_h2d(vsa_ctx_t *ctx, void *dst, const void *src, size_t bytes);
int vsa_memcpy_d2h(vsa_ctx_t *ctx, void *dst, const void *src, size_t bytes);
int vsa_sync(vsa_ctx_t *ctx);

/* Blocks per launch (scan_blocks / plans / hs corpora / hs_scan_vector
 * pieces): the confirm records carry a 20-bit block index.  Larger batches
 * are refused with VSA_E_INVALID (VSA_HS_INVALID at the hs level); split
 * them into several calls. */
#define VSA_MAX_BLOCKS (1u << 20)

/* Scan nblocks device-resident blocks (each = one hwlmExec(start=starts[i],
 * groups=ALL)) in one launch.  offsets[i], lens[i] are relative to d_data;
 * starts may be NULL (all 0).  Matches are sorted on the device into the
 * reference order; ends are offsets relative to d_data.  flags bit0: skip
 * the sort; bit1: asynchronous (do not wait for the count; *n_matches is
 * filled by vsa_scan_wait).  A scan started while an asynchronous one is
 * still pending first completes it (count, output-overflow rescan, sort) and
 * then supersedes its results. */
#define VSA_SCAN_UNSORTED 1u
#define VSA_SCAN_ASYNC 2u
int vsa_scan_blocks(vsa_ctx_t *ctx, const vsa_db_t *db, const uint8_t *d_data,
                    const uint64_t *offsets, const uint64_t *lens,
                    const uint64_t *starts, uint32_t nblocks, uint32_t flags,
                    uint64_t *n_matches);
/* As vsa_scan_blocks, plus report_lo[i] (may be NULL): ends below it are not
 * reported, while the FDR start state still applies from starts[i].  A
 * stripe of one block cut at lo is scanned as the window [lo - 7, hi) with
 * start 0 and report_lo 7 (literals are <= 8 bytes, hwlm.h:75): exactly the
 * block's matches ending in [lo, hi), see vectorscan_amd/stripe.py. */
int vsa_scan_blocks_ex(vsa_ctx_t *ctx, const vsa_db_t *db, const uint8_t *d_data,
                       const uint64_t *offsets, const uint64_t *lens,
                       const uint64_t *starts, const uint64_t *report_lo,
                       uint32_t nblocks, uint32_t flags, uint64_t *n_matches);
/* As vsa_scan_blocks, each block a streaming call: hlens[i] bytes of
 * history sit immediately before offsets[i] in d_data (only those bytes are
 * read before the block, at most 16 of them); hlens[i] = 0 is a
 * block-mode scan.  A stream cut into consecutive chunks is scanned as one
 * launch this way. */
int vsa_scan_blocks_stream(vsa_ctx_t *ctx, const vsa_db_t *db, const uint8_t *d_data,
                           const uint64_t *offsets, const uint64_t *lens,
                           const uint64_t *starts, const uint64_t *hlens, uint32_t nblocks,
                           uint32_t flags, uint64_t *n_matches);
/* A batch's block table and segment map built and uploaded once for
 * repeated scans of the same device blocks (e.g. hsbench's repeats): the
 * arguments of vsa_scan_blocks_ex / _stream (starts, hlens, report_lo may
 * be NULL).  At most 2^20 blocks per batch.  A plan belongs to its context
 * and must outlive the scans that use it. */
typedef struct vsa_plan vsa_plan_t;
/* Host-only: the schedule (segment descriptors, per-workgroup list bounds)
 * the planner makes for a batch on num_cus CUs with ns scanning waves each,
 * for tests and tools; returns the word count.  wg_weights (NULL: equal)
 * weights workgroup b's static share, as the schedule feedback does (one
 * float per workgroup, at least num_cus of them). */
int vsa_plan_describe(const uint8_t *d_data, const uint64_t *offsets, const uint64_t *lens,
                      const uint64_t *starts, const uint64_t *hlens, const uint64_t *report_lo,
                      uint32_t nblocks, uint32_t num_cus, uint32_t ns, uint32_t *words,
                      uint64_t cap, uint64_t *nsegs, uint32_t *grid,
                      const float *wg_weights);
/* Host-only (tests): the block table the planner builds for a batch (one
 * 72-byte record per block, kernels.h struct VsaBlock: base, len, start,
 * seg_first, zbase, org, rlo, hlen, hist, flags) into out[nblocks]; d_data
 * only sets the alignment.  Returns VSA_OK or a VSA_E_* code. */
int vsa_plan_blocks(const uint8_t *d_data, const uint64_t *offsets, const uint64_t *lens,
                    const uint64_t *starts, const uint64_t *hlens, const uint64_t *report_lo,
                    uint32_t nblocks, void *out);

/* Host-only (tests): the dynamic shares the planner grants a batch on
 * num_cus CUs with ns scanning waves each (kernels.hip dyn_bounds: each
 * launch cuts the live KiB at per-XCD weights it derives from the previous
 * launch's end times): out[0] = the live KiB (0: static lists), out[1] = how
 * far (KiB) a boundary may move from the equal-share one.  Returns VSA_OK
 * or a VSA_E_* code. */
int vsa_plan_dyn(const uint8_t *d_data, const uint64_t *offsets, const uint64_t *lens,
                 const uint64_t *starts, const uint64_t *hlens, const uint64_t *report_lo,
                 uint32_t nblocks, uint32_t num_cus, uint32_t ns, uint32_t *out);
/* Host-only (tests): the schedule feedback's per-XCD weight updates over
 * `launches` synthetic launches of `grid` workgroups (b on XCD b % 8) whose
 * XCDs run at rate[0..7], with relative timing noise `jitter`; the applied
 * weights go to w_out[8], the return value counts their changes. */
int vsa_feedback_simulate(const double *rate, uint32_t grid, uint32_t launches, double jitter,
                          float *w_out);
int vsa_plan_create(vsa_ctx_t *ctx, const uint8_t *d_data, const uint64_t *offsets,
                    const uint64_t *lens, const uint64_t *starts, const uint64_t *hlens,
                    const uint64_t *report_lo, uint32_t nblocks, vsa_plan_t **plan);
int vsa_plan_free(vsa_plan_t *plan);
/* Segment maps a plan rebuilt so far to follow the schedule feedback's
 * weights (tests: the feedback reaches prebuilt plans). */
uint32_t vsa_plan_rebuilds(const vsa_plan_t *plan);
/* vsa_scan_blocks over a plan (same flags, results and waiting) */
int vsa_scan_plan(vsa_ctx_t *ctx, const vsa_db_t *db, const vsa_plan_t *plan, uint32_t flags,
                  uint64_t *n_matches);
int vsa_scan_wait(vsa_ctx_t *ctx, uint64_t *n_matches);
/* Device pointers to the last scan's sorted keys (u64) and ids (u32).  The
 * scan is completed and the context's stream synchronized first, so the
 * pointers can be read on any stream. */
/* Pack the last scan's sorted records for a collective, into caller device
 * memory d_dst (u64 words): [header | keys (cap) | ids (cap x u32, i.e.
 * cap / 2 words)], header = record count, bit 62 set when the records are
 * not usable as packed (the scan overflowed its output, or a crowded sort
 * bin means the scan runs again without bins: complete the scan with
 * vsa_scan_wait, which does so, and pack again), then min(count, cap)
 * records.  After an asynchronous binned scan
 * the pack is queued on the context's stream behind it with no host wait
 * (RCCL gathers of stripes, vectorscan_amd/stripe.py); otherwise the scan
 * is completed first. */
int vsa_scan_pack(vsa_ctx_t *ctx, void *d_dst, uint64_t cap);
/* vsa_scan_plan(..., VSA_SCAN_ASYNC) whose binned sort also writes the
 * records into d_dst in vsa_scan_pack's layout, header included: the pack
 * launch behind the sort is gone (one kernel boundary and one copy of the
 * records less per multi-GPU step).  For this launch only: when it is not
 * binned (or a crowded bin / output overflow makes the header NOT_READY)
 * the caller completes the scan and repacks with vsa_scan_pack, as after a
 * plain scan. */
int vsa_scan_plan_pack(vsa_ctx_t *ctx, const vsa_db_t *db, const vsa_plan_t *plan, void *d_dst,
                       uint64_t cap);
int vsa_scan_results(vsa_ctx_t *ctx, const uint64_t **d_keys,
                     const uint32_t **d_ids);
/* Copy up to cap results of the last scan to the host. */
int vsa_scan_copy(vsa_ctx_t *ctx, vsa_match_t *out, uint64_t cap,
                  uint64_t *n_copied);
/* Device-to-device copy (on the context's stream, not waited for) of up to
 * cap results of the last scan into caller-owned device buffers (either may
 * be NULL), e.g. tensors handed to an RCCL gather. */
int vsa_scan_copy_device(vsa_ctx_t *ctx, uint64_t *d_keys, uint32_t *d_ids, uint64_t cap,
                         uint64_t *n_copied);
/* Candidates handed to the confirm stage (after the LDS slot prefilter) in
 * the last scan. */
uint64_t vsa_scan_candidates(vsa_ctx_t *ctx);
/* Diagnostics of the last literal scan (device counters 0..15): [0]
 * matches, [2] confirm candidates; with VSA_DEBUG_FLAGS bit 6 the confirm
 * waves' cycles: [4] gathering, [5] expanding, [6] confirming, [7] idle,
 * and counts: [8] gather rounds, [9] chunk entries, [10] expansion rounds,
 * [11] confirm batches. */
int vsa_scan_debug_counters(vsa_ctx_t *ctx, uint64_t out[16]);
/* Device time (ms, hipEvents on the scan stream) of the last scan kernel;
 * -1 when that launch carried no timing events (vsa_ctx_set_timing). */
double vsa_scan_kernel_ms(vsa_ctx_t *ctx);
/* Time every `every`-th literal-scan launch of this context (1, the default:
 * all; 0: none).  The events ride on the dispatch and cost a few us per
 * launch; a pipelined caller can sample.  No reference counterpart. */
int vsa_ctx_set_timing(vsa_ctx_t *ctx, uint32_t every);
/* Literal-scan launches this context has queued (every rescan of an
 * output overflow or a crowded sort bin counts): a diagnostic of the rerun
 * cost, no reference counterpart. */
uint64_t vsa_scan_launches(vsa_ctx_t *ctx);
/* 1 when the context's last literal-scan launch sorted its records inside
 * the scan kernel (the fused finish: no vsa_bin_finish launch behind it),
 * else 0.  A diagnostic, no reference counterpart. */
int vsa_scan_last_fused(vsa_ctx_t *ctx);
/* 1 when the context's last literal-scan launch set its workgroups' shares
 * itself (dynamic shares: per-XCD weights from the previous launch's end
 * times; VSA_DYN_SHARES=0 turns them off), else 0.  A diagnostic, no
 * reference counterpart. */
int vsa_scan_last_dyn(vsa_ctx_t *ctx);
/* Dynamic shares (an option; measured even with the host's schedule
 * feedback on the headline) for the context's FDR launches of at least
 * min_bytes over eligible plans (>= 64 workgroups, >= 256 MiB of parts of
 * blocks in address order): each launch cuts its workgroups' ranges from
 * the previous launch's per-XCD end times.  on = 1, off = 0 (the default
 * unless VSA_DYN_SHARES=1; VSA_DYN_MIN_MIB sets the default min_bytes,
 * 2048 MiB).  Results are identical either way. */
int vsa_ctx_set_dyn_shares(vsa_ctx_t *ctx, int on, uint64_t min_bytes);
/* Sort inside the scan kernel when the plan allows it (the fused finish:
 * no vsa_bin_finish launch behind the scan, the scan's workgroups sort
 * their own records and the last one publishes the count), on = 1; off = 0
 * (the default, or VSA_FUSED_FINISH=1 at start-up).  Results are identical
 * either way; no reference counterpart. */
int vsa_ctx_set_fused_finish(vsa_ctx_t *ctx, int on);
/* Measurement helper, not a scan (no reference counterpart): the streaming-
 * read ceiling of this device over d_data -- the first len rounded down to
 * 64 KiB read once per run by a plain 16-byte-load kernel on the ctx stream,
 * best of `runs` after one untimed run.  *bytes = the bytes read per run.
 * Synchronous.  bench.py reports it as roofline.peak_measured. */
int vsa_read_ceiling(vsa_ctx_t *ctx, const uint8_t *d_data, uint64_t len, uint32_t runs,
                     double *best_ms, uint64_t *bytes);

/* Byte-class scan over a device buffer: class = 256-bit membership bitmap
 * (bit c of byte c>>3).  class2 non-NULL: pair mode (class at i, class2 at
 * i+1).  d_bitmap (optional) receives 1 bit per byte ((len+63)/64 u64).
 * first/last/count are host outputs (first = len if none, last = index of
 * the last set bit + 1, 0 if none). */
int vsa_class_scan(vsa_ctx_t *ctx, const uint8_t cls[32], const uint8_t *cls2,
                   const uint8_t *d_data, uint64_t len, uint64_t *d_bitmap,
                   uint64_t *first, uint64_t *last, uint64_t *count,
                   uint32_t flags);
/* The same over a shufti (kind 0: lo, hi) or truffle (kind 1: m1, m2) mask
 * pair, the bytecode shuftiExec / truffleExec take (shufti.h:46,
 * truffle.h:45): the class is the set of bytes the masks accept. */
int vsa_class_scan_masks(vsa_ctx_t *ctx, int kind, const uint8_t a[16], const uint8_t b[16],
                         const uint8_t *d_data, uint64_t len, uint64_t *d_bitmap,
                         uint64_t *first, uint64_t *last, uint64_t *count);

/* ------------------------------------------------------------------ *
 * Part 3 — HWLM bytecode builder (reference layout; see compile.cpp)
 * ------------------------------------------------------------------ */

/* hwlmLiteral, src/hwlm/hwlm_literal.h:51 */
typedef struct {
    const uint8_t *s;
    uint32_t len;
    uint32_t id;
    uint8_t nocase;
    uint8_t noruns;
    uint8_t msk_len;
    uint8_t pad;
    uint64_t groups;
    const uint8_t *msk;
    const uint8_t *cmp;
} vsa_literal_t;

typedef struct {
    int32_t engine_hint; /* -1 choose; 0 FDR (domain 9, stride 1); 3..18 Teddy */
    uint8_t allow_noodle;
    uint8_t allow_teddy;
    uint8_t allow_fat_teddy;
    uint8_t allow_flood;
} vsa_build_opts_t;

void vsa_build_opts_default(vsa_build_opts_t *o);
/* Builds an HWLM blob (64-byte aligned, free with vsa_blob_free). */
int vsa_hwlm_build(const vsa_literal_t *lits, size_t n,
                   const vsa_build_opts_t *opts, void **blob, size_t *size);
void vsa_blob_free(void *blob);
/* Set HWLM.accel0 / accel1 (+accel1_groups) of a built blob. */
int vsa_hwlm_set_accel(void *blob, const union AccelAux *accel0,
                       const union AccelAux *accel1, uint64_t accel1_groups);
/* shufticompile.cpp:54 — returns buckets used or -1. */
int vsa_shufti_build_masks(const uint8_t cls[32], uint8_t lo[16], uint8_t hi[16]);
/* trufflecompile.cpp:60 */
void vsa_truffle_build_masks(const uint8_t cls[32], uint8_t m1[16], uint8_t m2[16]);

/* Pointer-argument forms of the accel drop-ins (for FFI callers that cannot
 * pass vector registers).  Return an index: forward = first hit or len,
 * reverse = last hit or -1. */
int64_t vsa_shufti_find(const uint8_t lo[16], const uint8_t hi[16],
                        const uint8_t *buf, size_t len, int reverse);
int64_t vsa_truffle_find(const uint8_t m1[16], const uint8_t m2[16],
                         const uint8_t *buf, size_t len, int reverse);
/* shuftiDoubleExec by pointer: first match index or len (-2 on error). */
int64_t vsa_shufti_double_find(const uint8_t lo1[16], const uint8_t hi1[16],
                               const uint8_t lo2[16], const uint8_t hi2[16],
                               const uint8_t *buf, size_t len);
/* VECTORSIZE of the reference build whose shuftiDoubleExec is emulated
 * (16 SSE, 32 AVX2, 64 AVX-512; default 64). */
void vsa_set_accel_vector_size(uint32_t vsize);

/* Diagnostic: device buffer of 8 x u64 per scanning wave (workgroup * 16 +
 * wave) that literal scans run with VSA_DEBUG_FLAGS bit 4096 fill (start and
 * end timestamps at 100 MHz, segments, 1 KiB iterations, workgroup, wave,
 * XCC id, HW_ID); NULL turns it off. */
void vsa_set_wave_log(void *d_log);
/* shufticompile.cpp:135 shuftiBuildDoubleMasks: onechar = 256-bit class
 * (may be NULL), pairs = npairs (first, second) bytes.  0 ok, -1 = more
 * than 8 buckets needed. */
int vsa_shufti_build_double_masks(const uint8_t onechar[32], const uint8_t *pairs,
                                  size_t npairs, uint8_t lo1[16], uint8_t hi1[16],
                                  uint8_t lo2[16], uint8_t hi2[16]);
/* mode: 0 verm, 1 nverm, 2 rverm, 3 rnverm, 4 dverm, 5 dverm masked,
 * 6 rdverm (reverse double: index of c2 of the last pair, or -1) */
int64_t vsa_verm_find(int mode, uint8_t c1, uint8_t c2, uint8_t m1, uint8_t m2,
                      int nocase, const uint8_t *buf, size_t len);

/* Host-only: the first-stage table the engine derives from an FDR / Teddy
 * blob's confirm records (FDR: 2^14 u64 entries, 8 positions x 8 buckets,
 * key = (b[p] & 0x7f) | (b[p+1] & 0x7f) << 7; Teddy: 256 entries, 8 x 8; Fat Teddy:
 * 256 entries, 4 x 16).  Returns entries written or a VSA_E_* code. */
int vsa_derive_first_stage(const void *hwlm, size_t size, uint64_t *table, uint32_t cap,
                           uint32_t *key_bits, uint32_t *field_bits);
/* Host-only: the 4-field FDR first stage the engine scans with by default
 * (2^bits u32 entries, bits 14 / 15: field f (byte f) = the buckets dead at
 * end p + f; key = (b[p-1] & 0x7f) | (b[p] & 0x7f) << 7 | (b[p-2] & 1) << 14
 * at 15 bits).  Returns entries written or a VSA_E_* code. */
int vsa_derive_fdr4_table(const void *hwlm, size_t size, uint32_t bits, uint32_t *table,
                          uint32_t cap);

/* Host-only (tests / tools): the 15-bit 4-field table of one split pass --
 * par 0 / 1: the literals whose last byte can have bit 0 == par, the table
 * a large set's pass over the ends with that end-byte bit uses; -1: the
 * one-pass table -- and in *text_rate (may be NULL) the candidate bits per
 * text byte estimated from it (the rule that turns the split passes on past
 * 0.015).  table may be NULL (rate only).  Returns the entries written or a
 * VSA_E_* code.  No reference counterpart: the split is this engine's
 * schedule for sets the reference scans with one FDR pass (fdr.c:776-796). */
int vsa_derive_fdr4_pass(const void *hwlm, size_t size, int par, uint32_t *table, uint32_t cap,
                         double *text_rate);

/* 1 when the database scans in split passes (vsa_derive_fdr4_pass), 0 if
 * not, or a VSA_E_* code. */
int vsa_db_split(const vsa_db_t *db);

/* Optional: hs_scratch field offsets for INCLUDED_JUMP squash replay
 * (offsetof(struct hs_scratch, fdr_conf / fdr_conf_offset)); the defaults
 * are the x86-64 layout of src/scratch.h:172-219. */
void vsa_set_scratch_layout(long fdr_conf_off, long fdr_conf_offset_off);
void vsa_get_scratch_layout(long *fdr_conf_off, long *fdr_conf_offset_off);

/* Optional: offsets of core_info.buf / hbuf / hlen inside hs_scratch for
 * hwlmExecStreaming (defaults: x86-64 layout of scratch.h:91-191). */
void vsa_set_scratch_core_info(long buf_off, long hbuf_off, long hlen_off);
void vsa_get_scratch_core_info(long *buf_off, long *hbuf_off, long *hlen_off);

/* VSA_E_DEVICE if a pointer-returning drop-in of this thread hit a device
 * failure since the last call (then cleared), else VSA_OK. */
int vsa_last_error(void);

const char *vsa_version(void);

#ifdef __cplusplus
}
#endif

#endif /* VECTORSCAN_AMD_H */
