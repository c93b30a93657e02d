/*
 * vsa_internal.h — host-side declarations shared by compile.cpp and the
 * runtime (runtime.hip).  Not part of the public ABI (see
 * include/vectorscan_amd.h).
 */
#ifndef VSA_INTERNAL_H
#define VSA_INTERNAL_H

#include "hs_layout.h"

#include <string>
#include <vector>

#define VSA_OK 0
#define VSA_E_INVALID (-1)
#define VSA_E_NOMEM (-2)
#define VSA_E_NOT_BUILDABLE (-3)
#define VSA_E_DEVICE (-4)
#define VSA_E_OVERFLOW (-5)

namespace vsa {

/* hwlmLiteral, src/hwlm/hwlm_literal.h:51-130 */
struct Literal {
    std::string s;
    u32 id = 0;
    bool nocase = false;
    bool noruns = false;
    u64a groups = HWLM_ALL_GROUPS;
    std::vector<u8> msk;
    std::vector<u8> cmp;
};

/* The Grey knobs that change engine choice (src/grey.cpp:66-68) plus the
 * unit-test engine hint (fdr_compile.cpp:899-910). */
struct BuildOptions {
    bool allow_noodle = true;
    bool allow_teddy = true;
    bool allow_fat_teddy = true; /* the GPU runs 16-bucket Teddy natively */
    bool allow_flood = true;     /* Grey::fdrAllowFlood (grey.cpp:68) */
    int engine_hint = -1;        /* -1: choose; 0: FDR d9 s1; 3..18 Teddy id */
};

/* One flood shortcut taken by the reference main loop (flood.cpp): the
 * flood ids of `fl` are reported at ends [i, i + size) and the main loop
 * skips those ends. */
struct FloodEvent {
    u32 i;
    u32 size;
    const FDRFlood *fl;
};
/* Flood events of one fdrExec / fdrExecStreaming call on the engine `eng`
 * (FDR or Teddy) over the host buffer (its address matters), in order.
 * vsize selects the Teddy build emulated (16 SSE, 32 AVX2, 64 VBMI). */
void flood_events(const u8 *buf, size_t len, size_t start, const u8 *eng, u32 vsize,
                  std::vector<FloodEvent> &out);

} // namespace vsa

struct hs_scratch;
struct vsa_ctx;
struct vsa_db;
struct vsa_plan;

namespace vsa {

/* HWLMCallback (hwlm.h:63-73) */
typedef u64a (*LitCallback)(size_t end, u32 id, ::hs_scratch *scratch);

/* runtime.hip: the writes of one stream (history hist[0, hist_len) before
 * the first) scanned in one GPU launch and replayed write by write through
 * cb(end relative to the write, HWLM literal id, cbctx); on_piece(cbctx, i)
 * runs before write i's records.  Zero-length writes are skipped. */
int exec_pieces(vsa_ctx *c, const vsa_db *db, const u8 *hist, size_t hist_len,
                const u8 *const *bufs, const size_t *lens, size_t n, LitCallback cb,
                void *cbctx, void (*on_piece)(void *, size_t));

/* runtime.hip: one launch over device blocks (hlens NULL = block mode);
 * the sorted records to the host when keys != NULL, else only counted */
/* pipelined corpus repeats (vsa_hs_corpus_scan_repeats): the last
 * completed scan's n records copied into host buffers asynchronously
 * (records_fetch_async, then records_wait), so the next scan can be queued
 * while the host replays; pinned host buffers.  records_mark after queuing
 * a scan notes its end on the scan stream; records_fetch_async then copies
 * on the context's copy stream after that mark (beside the scan queued
 * after it) and holds the scan stream's next work until the copy is done
 * (the context's next scan rewrites the records).  Without a mark (or
 * remark, after a rescan) the copy follows everything queued so far. */
int records_mark(vsa_ctx *c);
int records_fetch_async(vsa_ctx *c, uint64_t n, uint64_t *h_keys, uint32_t *h_ids,
                        bool remark = false);
int records_wait(vsa_ctx *c);
void *host_pinned_alloc(size_t bytes);
void host_pinned_free(void *p);

int scan_records(vsa_ctx *c, const vsa_db *db, const u8 *d_data, const uint64_t *offsets,
                 const uint64_t *lens, const uint64_t *hlens, uint32_t nblocks,
                 std::vector<uint64_t> *keys, std::vector<uint32_t> *ids, uint64_t *n,
                 const vsa_plan *plan = nullptr);
/* one call's records (ends relative to its buffer) through cb, no floods */
int replay_records(const vsa_db *db, const uint64_t *keys, const uint32_t *ids, uint64_t n,
                   LitCallback cb, void *cbctx);

Literal makeLiteral(const u8 *s, size_t len, bool nocase, bool noruns, u32 id,
                    u64a groups, const u8 *msk, const u8 *cmp, size_t mlen);
int buildHwlm(std::vector<Literal> lits, const BuildOptions &opt, u8 **out,
              size_t *outSize);
int shuftiMasks(const u8 cls[32], u8 lo[16], u8 hi[16]);
bool shuftiDoubleMasks(const u8 onechar[32], const u8 *pairs, size_t npairs, u8 lo1[16],
                       u8 hi1[16], u8 lo2[16], u8 hi2[16]);
void truffleMasks(const u8 cls[32], u8 m1[16], u8 m2[16]);

/* the host copy of a loaded database's HWLM blob (hs_clone_scratch reloads
 * it into another context) */
int dbHostBlob(const struct vsa_db *db, const uint8_t **blob, size_t *size);
/* the GPU a context was created on (hs_clone_scratch builds the clone's
 * context on the source's device) */
int ctxDevice(const struct vsa_ctx *c);

} // namespace vsa

#endif
