/*
 * runtime_internal.h -- what the host runtime's translation units share
 * (not installed, not part of the C ABI):
 *
 *   runtime.hip  contexts, device workspace, database load (derived first
 *                stages), literal-scan launch / completion, the binned sort
 *                behind it, schedule feedback, the batch and class-scan API
 *   plan.hip     launch plans: block table, segment lists, owned sort bins
 *                (build_plan) and the prebuilt-plan API (vsa_plan_*)
 *   dropin.hip   the reference's entry points (hwlmExec, fdrExec, noodExec,
 *                streaming forms, shufti / truffle / vermicelli, run_accel):
 *                blob registry, host replay of the records, accel pre-skip,
 *                the hs_lit.cpp bridge (namespace vsa) and the builder API
 *   batcher.hip  the batching service (vsa_batcher_*)
 */
#ifndef VSA_RUNTIME_INTERNAL_H
#define VSA_RUNTIME_INTERNAL_H

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include <sched.h>

#include "../../include/vectorscan_amd.h"
#include "hs_layout.h"
#include "kernels.h"
#include "vsa_internal.h"

template <int MODE, bool XP, bool SPLIT>
__global__ void vsa_lit_scan(VsaLitParams P);
__global__ void vsa_class_scan(VsaClassParams P);
__global__ void vsa_bin_finish(const uint32_t *counts, uint32_t *counts_next,
                               const uint64_t *skeys, const uint32_t *sids, uint64_t *okeys, uint32_t *oids, uint64_t out_cap,
                               unsigned long long *ctr,
                               unsigned long long *h, unsigned long long seq,
                               const unsigned long long *fb, unsigned long long *hfb,
                               uint32_t nfb, uint64_t *pk, uint64_t pk_cap);
__global__ void vsa_class_scan_lut(VsaClassParams P, uint64_t span);
__global__ void vsa_publish(unsigned long long *ctr, unsigned long long *h, unsigned long long seq,
                            uint32_t nzero, const uint64_t *keys, const uint32_t *ids,
                            uint32_t kmax);
__global__ void vsa_pack(const unsigned long long *saved, uint64_t out_cap, const uint64_t *keys,
                         const uint32_t *ids, uint64_t cap, uint64_t *dst);
__global__ void vsa_pair_scan(VsaPairParams P);
__global__ void vsa_read_probe(const uint8_t *A, uint64_t n, uint32_t *sink);

#define VSA_CHECK(x)                                                          \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            if (!getenv("VSA_QUIET"))                                         \
                fprintf(stderr, "vsa: %s failed: %s (%s:%d)\n", #x,           \
                        hipGetErrorString(e_), __FILE__, __LINE__);           \
            return VSA_E_DEVICE;                                              \
        }                                                                     \
    } while (0)

namespace vsa_rt {


const int LIT_WAVES = 16;
const int LIT_THREADS = 1024;
const size_t LDS_BUDGET = 160 * 1024 - 4096; /* minus static LDS (confirm params,
                                                ring cursors) */
const uint32_t SLOT_WORDS_MAX = 3072;        /* 12 KiB of slot bitmaps (coarsened
                                                beyond, see vsa_db_load) */

/* d_counters layout (u64): [0..15] scan counters, [144..159] the last
 * binned scan's counters kept for vsa_pack, [PAIR_BASE + 16 k]
 * double-shufti stage results, [CLASS_BASE + 16 s + {0,1,2}] class-scan
 * first / last / count partials of slot s (one line per slot) */
constexpr int CLASS_SLOTS = 64;
constexpr int PAIR_BASE = 160; /* double-shufti stage results, 16 apart */
constexpr int CLASS_BASE = 256;
constexpr int N_COUNTERS = CLASS_BASE + 16 * CLASS_SLOTS;
/* h_pub (vsa_publish): [0] sequence, [1..16] counters, then up to PUB_RECS
 * raw records of a drop-in scan (keys, then ids as u32) */
constexpr uint32_t PUB_RECS = 1024;
constexpr size_t PUB_WORDS = 17 + PUB_RECS + PUB_RECS / 2;

struct Workspace {
    uint8_t *d_in = nullptr;
    size_t in_cap = 0;
    uint8_t *h_in = nullptr; /* pinned staging of drop-in inputs (one DMA) */
    size_t h_in_cap = 0;
    uint64_t *d_keys[2] = {nullptr, nullptr};
    uint32_t *d_ids[2] = {nullptr, nullptr};
    uint64_t out_cap = 0;
    void *d_tmp = nullptr;
    size_t tmp_bytes = 0;
    unsigned long long *d_counters = nullptr; /* layout above */
    uint32_t *d_bins = nullptr; /* binned sort: two count buffers of
                                   VSA_SORT_BINS, used in turn (vsa_bin_finish
                                   reads one and clears the other) */
    /* staged records of the binned sort: VSA_SORT_BIN_MAX per bin, keys
     * (u64) then ids (u32) */
    uint8_t *d_bstage = nullptr;
    unsigned long long *h_counters = nullptr; /* pinned mirror */
    /* fine-grained host memory the device publishes a binned scan's
     * counters into (vsa_publish): [0] = sequence, [1..16] = counters */
    unsigned long long *h_pub = nullptr, *d_pub = nullptr;
    VsaBlock *d_blocks = nullptr; /* this call's block table, then its segment map */
    VsaBlock *h_blocks = nullptr; /* pinned mirror */
    size_t tab_cap = 0;           /* bytes of both */
    uint32_t *d_segblk = nullptr; /* block of each segment (inside d_blocks) */
    uint32_t *h_segblk = nullptr;
    /* the fused finish (kernels.hip fused_finish): staged records in local
     * bins, VSA_LBINS x VSA_SORT_BIN_MAX per workgroup (keys, then ids), for
     * fstage_grid workgroups; the workgroups' epoch-tagged totals */
    uint8_t *d_fstage = nullptr;
    uint32_t fstage_grid = 0;
    unsigned long long *d_fagg = nullptr; /* 2 x VSA_FIN_MAX_GRID words */
};


} // namespace vsa_rt

using namespace vsa_rt;

/* The block table and segment map of one batch (the kernel's schedule).
 * Segments are 1 KiB-aligned ranges of end positions: a block longer than
 * half a segment is cut into segments of its own; runs of consecutive
 * shorter blocks are packed whole into one segment (up to 255 blocks, one
 * segment's bytes), so a batch of small blocks costs one ticket and one
 * descriptor lookup per segment, not per block.  segblk[s] = first block |
 * count << 24 (count 0: part of one block). */
struct BatchPlan {
    std::vector<VsaBlock> blocks;
    /* 4 words per segment (kernels.h seg_desc), then grid + 1 list
     * bounds */
    std::vector<uint32_t> segblk;
    uint64_t nsegs = 0;
    uint32_t grid = 0; /* workgroups (one segment list each) */
    int end_bits = 0;
    uint64_t bytes = 0; /* scanned bytes (len - start summed) */
    /* the fused finish's local-bin table follows the owned bins in segblk
     * and is usable (plan_fused) */
    bool fin_ok = false;
    /* dynamic shares (kernels.hip dyn_bounds): the live KiB the workgroups
     * split at launch, 0 = the static lists; the boundaries' margin (KiB) */
    uint32_t dyn_kib = 0, dyn_margin = 0;
    std::vector<int64_t> spans, live; /* build_plan scratch */
};

/* the dynamic shares' state of one stream (shared by the contexts on it):
 * the launches' end-time records and weights, double-buffered by launch
 * (a launch reads the previous one's, complete by stream order, and writes
 * its own) */
struct DynState {
    unsigned long long *d = nullptr; /* [2][512] records, then [2][8] u32 weights */
    uint64_t epoch = 0;              /* dynamic-share launches queued */
    uint32_t grid = 0;               /* the last one's grid (0: none yet) */
    int kind = -1;                   /* ... and its scan mode */
    ~DynState() {
        if (d) (void)hipFree(d);
    }
};

struct vsa_plan;

struct vsa_ctx {
    int device = 0;
    int num_cus = 256;
    /* CUs the literal scan's persistent grid leaves free
     * (vsa_ctx_set_reserved_cus): plans use num_cus - reserved_cus */
    int reserved_cus = 0;
    int plan_cus() const { return std::max(1, num_cus - reserved_cus); }
    hipStream_t stream = nullptr;
    /* the stream's owner: shared by contexts made with vsa_ctx_create_shared,
     * destroyed with the last of them */
    std::shared_ptr<void> stream_ref;
    std::shared_ptr<DynState> dyn; /* the stream's dynamic-share state */
    Workspace ws;
    int cur = 0;          /* which key/id buffer holds the last results */
    uint64_t last_n = 0;
    uint64_t last_cand = 0;
    bool pending = false; /* async scan in flight */
    /* the last launch (relaunched after an output overflow; the block and
     * segment tables it reads stay in the pinned/device workspace until the
     * next scan) */
    struct {
        const vsa_db *db = nullptr;
        const uint8_t *d_data = nullptr;
        uint32_t nb = 0;
        uint64_t segs = 0;
        uint32_t grid = 0; /* the plan's workgroups (one segment list each) */
        int end_bits = 0;
        uint32_t flags = 0;
        bool bins = false;     /* the scan counts records into the sort bins */
        bool dev_sort = false; /* ... and the binned sort is queued behind it */
        bool published = false; /* ... and vsa_publish after it (finish_scan
                                   polls h_pub instead of copying) */
        bool fin_ok = false;    /* the plan allows the fused finish */
        bool timed = false;     /* the dispatch carries ev0 / ev1 */
        bool fused = false;     /* ... and this launch sorts inside the scan */
        uint32_t dyn_kib = 0, dyn_margin = 0; /* the plan's (BatchPlan) */
        bool dyn = false;       /* this launch sets its shares (dyn_bounds) */
        uint64_t dyn_epoch = 0; /* ... its DynState epoch */
        uint64_t bytes = 0; /* scanned bytes (len - start summed) */
        const VsaBlock *d_blocks = nullptr;
        const uint32_t *d_segblk = nullptr;
        /* the kernel-timing events the next literal-scan dispatch carries
         * itself (launch_lit: start on the first kernel, stop on the last
         * of split passes); null = untimed */
        hipEvent_t ev_start = nullptr, ev_stop = nullptr;
        /* vsa_scan_plan_pack: the binned sort also writes the records into
         * this collective buffer (vsa_pack's layout), for the next launch
         * only */
        void *pack_dst = nullptr;
        uint64_t pack_cap = 0;
    } launch;
    /* kernel-only timing of the last scan (hipEvents on the scan stream) */
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_done = nullptr; /* polled by wait_stream */
    hipEvent_t ev_rec = nullptr;  /* records_fetch_async's copies done */
    hipEvent_t ev_mark = nullptr; /* records_mark: the end of a queued scan */
    bool marked = false;
    hipStream_t copy_stream = nullptr; /* records_fetch_async's copies */
    double last_kernel_ms = 0.0;
    bool kms_stale = false; /* last_kernel_ms not yet read for the last scan */
    /* eligible launches sort inside the scan kernel (kernels.hip
     * fused_finish; vsa_ctx_set_fused_finish, default VSA_FUSED_FINISH) */
    bool fused_finish = false;
    /* every timing_every-th literal-scan launch carries the kernel-timing
     * events (vsa_ctx_set_timing; 1 = all, 0 = none) */
    uint32_t timing_every = 1;
    /* eligible plans' launches set their own shares (kernels.hip
     * dyn_bounds; vsa_ctx_set_dyn_shares, default VSA_DYN_SHARES) */
    bool dyn_shares = true;
    uint64_t dyn_min = 0; /* ... of at least this many bytes */
    uint32_t bin_skip = 0;   /* launches left without the binned sort */
    /* the bin_skip a crowded bin sets: 16, x4 for every crowded binned
     * launch in a row (up to 4096), back to 16 after a binned launch that
     * fit: a persistently dense workload pays the rerun (finish_scan) about
     * once per 4096 launches instead of once per 17 */
    uint32_t bin_backoff = 16;
    uint64_t lit_launches = 0; /* literal-scan launches queued (vsa_scan_launches) */
    bool bins_clean[2] = {false, false}; /* bin count buffer b is zero (no memset) */
    uint32_t bin_par = 0;                /* the count buffer the next binned scan uses */
    /* host bytes already in ws.d_in (set only inside one drop-in call, so the
     * accel pre-skip and the literal scan share one upload) */
    const uint8_t *res_host = nullptr;
    size_t res_len = 0;
    BatchPlan plan; /* the per-call batch plan (reused storage) */
    /* the inputs of the plan now in ws.d_blocks: a call with the same block
     * list (a scan repeated over the same buffers) reuses the device tables
     * instead of rebuilding and uploading them */
    struct {
        bool valid = false;
        const uint8_t *d_data = nullptr;
        uint64_t waves = 0;
        uint32_t nb = 0;
        uint64_t fb_key = 0; /* the feedback weights it was built with (fb_key_of) */
        std::vector<uint64_t> in[5]; /* offs, lens, starts, hlens, rlos ({} = NULL) */
    } memo;
    bool host_sort = false; /* the last scan's records are left unsorted */
    /* the scan counters [0, 144) are zero (the last launch published and
     * cleared them), so the next launch needs no memset */
    bool ctr_clean = false;
    uint64_t pub_seq = 0; /* sequence of the last vsa_publish queued */
    /* live plans of this context (vsa_ctx_destroy detaches them, so a plan
     * freed after its context never touches it) */
    std::vector<vsa_plan *> plans;
    /* schedule feedback (take_feedback): per-XCD weights of the
     * workgroups' static shares, learned from the workgroups' end times of
     * large launches (the kernels write them into fine-grained host
     * memory); one set per kind of launch, as compute-bound and streaming
     * scans see different XCD speeds: 0 = FDR / Teddy, 1 = noodle */
    struct FbSet {
        float w[8] = {1, 1, 1, 1, 1, 1, 1, 1};  /* the running estimate */
        float wa[8] = {1, 1, 1, 1, 1, 1, 1, 1}; /* the weights plans use */
        uint8_t xcc[1024];       /* the XCD workgroup b ran on last time */
        float wg[1024];          /* wa[xcc[b]]: the share weights */
        uint32_t version = 0;    /* bumped when wa changes (plans rebuild) */
        uint32_t since = 0;      /* records taken since wa last changed */
        bool known = false;      /* xcc[] holds measured XCDs */
    };
    struct {
        FbSet set[2];
        unsigned long long *h = nullptr, *d = nullptr; /* 2 x 1024 u64 */
        int armed = -1;          /* the set the launch in flight records for */
        /* ... into device memory (d_rec), published with the counters by
         * vsa_bin_finish, instead of stores to host memory from the scan */
        bool dev = false;
        unsigned long long *d_rec = nullptr;
        uint32_t grid = 0;       /* the launch's workgroups */
    } fb;
};

/* A batch's block table and segment map built and uploaded once, then
 * reused by every vsa_scan_plan (a corpus scanned repeatedly: hsbench's
 * repeats, a database swap over the same data). */
struct vsa_plan {
    /* the owning context (nullptr once it is destroyed) */
    vsa_ctx *ctx = nullptr;
    const uint8_t *d_data = nullptr;
    uint32_t nb = 0;
    uint64_t segs = 0;
    uint32_t grid = 0;
    int end_bits = 0;
    uint64_t bytes = 0;
    uint32_t rebuilds = 0; /* segment maps rebuilt for the feedback weights */
    bool fin_ok = false;   /* its map allows the fused finish (plan_fused) */
    uint32_t dyn_kib = 0, dyn_margin = 0; /* dynamic shares (BatchPlan) */
    VsaBlock *d_blocks = nullptr;
    uint32_t *d_segblk = nullptr;
    /* schedule feedback: the inputs (to rebuild the segment map with the
     * context's current weights), the words d_segblk holds room for, and
     * the weights it was built with (fb_key_of; ~0: equal shares) */
    std::vector<uint64_t> in[5];
    size_t segblk_cap = 0;
    uint64_t fb_key = ~0ULL;
    void *h_stage = nullptr; /* pinned staging of a rebuilt block table + map */
    std::vector<uint32_t> flags; /* the block flags on the device (the only
                                    block field a rebuild can change that the
                                    kernel reads: VSA_BLK_RUN) */
};

/* drop-in scans: results of at most HOST_SORT_MAX records are sorted on the
 * host after the copy back (internal scan flag) */
constexpr uint32_t SCAN_HOST_SORT_SMALL = 1u << 16;
constexpr uint64_t HOST_SORT_MAX = 1024;

struct vsa_db {
    vsa_ctx *ctx = nullptr;
    std::vector<uint8_t> host; /* copy of the HWLM blob (64-B aligned data) */
    uint8_t *hblob = nullptr;  /* aligned pointer into host */
    size_t size = 0;
    uint8_t *d_blob = nullptr;
    uint64_t *d_table = nullptr; /* derived FDR table / Teddy combined table */
    int type = 0;                /* HWLM_ENGINE_NOOD / FDR */
    uint32_t engine_id = 0;
    int mode = 0;                /* VsaLitMode */
    /* split passes (FDR4, large literal sets): two launches, one per bit 0
     * of the end byte, each with the table of the literals that end in such
     * a byte (derive_fdr4_table par 0 / 1; d_table2 = par 1) */
    bool split = false;
    uint32_t *d_table2 = nullptr;
    double est_rate = 0.0;       /* fdr4_text_rate of the one-pass table */
    uint32_t table_entries = 0;
    uint32_t dmask = 0;
    uint64_t state_lo = 0, state_hi = 0;
    uint32_t conf_off[16] = {0};
    uint32_t nbuckets = 8;
    noodTable nood;
    uint32_t *d_slots = nullptr; /* litIndex-occupancy bitmaps (prefilter) */
    uint32_t slot_words = 0;
    uint32_t slot_off[16];
    uint8_t slot_bits[16] = {0}; /* prefilter hash bits per bucket (<= nBits) */
    uint64_t pf_mult = 0;
    bool flood_live = false;     /* some FDRFlood record can fire (idCount < max) */
    /* confirm waves per workgroup: the largest count the confirm-candidate
     * rate of any representative launch (>= 16 MiB) of the db asked for, on
     * any context (a sparse first launch, e.g. a warm-up, does not pin a
     * dense db to one wave); atomic, as dbs are shared by contexts and
     * threads.  It only grows (1 -> 2 -> 3) and feeds the segment sizes, so
     * a db's launch plans change at most twice. */
    mutable std::atomic<uint32_t> nconf{1};
    /* scanner expansion (use_xp): on once a representative launch measured
     * more than 4e-4 confirm candidates per byte; only turns on */
    mutable std::atomic<bool> xp{false};
};

/* drop-in scans: results of at most HOST_SORT_MAX records are sorted on the
 * host after the copy back (internal scan flag) -- see above */

namespace vsa_rt {

/* VECTORSIZE of the reference build emulated where results depend on it
 * (dropin.hip: shuftiDoubleExec's lanes, the flood shortcut's loop shape) */
extern uint32_t g_vector_size;
/* diagnostic per-wave log (vsa_set_wave_log; the scan kernel writes it
 * under debug flag 4096) */
extern unsigned long long *g_wave_log;

/* the per-call block table and segment map share one device allocation and
 * one pinned mirror, laid out per call */
constexpr size_t TAB_ALIGN = 256;
/* drop-in inputs up to this size are staged through pinned memory: one
 * host memcpy and one asynchronous DMA instead of a pageable copy */
constexpr size_t PIN_STAGE_MAX = (size_t)8 << 20;

/* Each launch is checked with hipGetLastError() right after it.  That call
 * returns (and clears) the thread's last error from ANY earlier HIP call,
 * including ignored statuses of free / destroy paths or another library's
 * calls on this thread, so the stale value is dropped immediately before the
 * launch: the check after it then sees this launch's error only. */
inline void drop_stale_error() { (void)hipGetLastError(); }

/* ---- runtime.hip ---- */
int ensure_out(vsa_ctx *c, uint64_t need);
int ensure_in(vsa_ctx *c, size_t need);
int ensure_hin(vsa_ctx *c, size_t need);
int ensure_tables(vsa_ctx *c, uint32_t nb, uint64_t nsegs, bool keep_blocks = false);
int env_int(const char *name, int dflt);
uint32_t steal_min();
int bits_for(uint64_t v);
uint32_t bin_shift_for(int end_bits);
bool xcd_feedback_on();
bool fused_finish_default();
int fb_set_of(const vsa_db *db);
uint64_t fb_key_of(const vsa_ctx *c, const vsa_db *db);
bool feedback_update(vsa_ctx::FbSet &F, const volatile unsigned long long *h, uint32_t G);
hipError_t wait_stream(vsa_ctx *c);
int finish_pending(vsa_ctx *c);
int complete_scan(vsa_ctx *c, uint64_t *n_out);
int launch_planned(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data, const VsaBlock *d_blocks,
                   const uint32_t *d_segblk, uint32_t nb, uint64_t segs, uint32_t grid,
                   int end_bits, uint64_t bytes, uint32_t flags, uint64_t *n_out,
                   bool fin_ok = false, uint32_t dyn_kib = 0, uint32_t dyn_margin = 0);
bool dyn_shares_on();
uint64_t dyn_min_bytes();
int scan_blocks_impl(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data,
                     const uint64_t *offs, const uint64_t *lens, const uint64_t *starts,
                     uint32_t nb, uint32_t flags, uint64_t *n_out,
                     const uint64_t *hlens = nullptr, const uint64_t *rlos = nullptr);

/* ---- plan.hip ---- */
int build_plan(const uint8_t *d_data, const uint64_t *offs, const uint64_t *lens,
               const uint64_t *starts, const uint64_t *hlens, const uint64_t *rlos,
               uint32_t nb, uint64_t waves, BatchPlan &pl, VsaBlock *out = nullptr,
               uint64_t ns = LIT_WAVES - 1, const float *wg_w = nullptr);
int upload_plan(vsa_ctx *c, const BatchPlan &pl, VsaBlock *d_blocks, uint32_t *d_segblk);

/* ---- dropin.hip ---- */
extern thread_local vsa_ctx *t_ctx;
vsa_ctx *default_ctx();
struct RegKey {
    const void *p;
    size_t size;
    bool operator<(const RegKey &o) const {
        if (p != o.p) return p < o.p;
        return size < o.size;
    }
};
/* per thread: the device copies of the blobs the drop-ins were called with */
extern thread_local std::map<RegKey, vsa_db *> t_registry;
vsa_db *registry_get(const void *ptr, int bare_type);
/* bytes of the engine after an HWLM header: noodTable / FDR.size / Teddy.size */
size_t engine_size(const uint8_t *eng, int type);
hwlm_error_t replay_nood(const uint64_t *keys, const uint32_t *ids, uint64_t n,
                         HWLMCallback cb, hs_scratch *scratch);
hwlm_error_t replay_lit(const vsa_db *db, const uint64_t *keys, uint64_t n,
                        HWLMCallback cb, hs_scratch *scratch, hwlm_group_t groups,
                        const std::vector<vsa::FloodEvent> *floods = nullptr,
                        bool scratch_is_real = true);
const std::vector<vsa::FloodEvent> *floods_for(const vsa_db *db, const uint8_t *buf, size_t len,
                                               size_t start,
                                               std::vector<vsa::FloodEvent> &ev);
int fetch_records(vsa_ctx *c, uint64_t n, std::vector<uint64_t> &keys,
                  std::vector<uint32_t> &ids);
int scan_host(vsa_db *db, const uint8_t *buf, size_t len, size_t start,
              std::vector<uint64_t> &keys, std::vector<uint32_t> &ids,
              const uint8_t *hend = nullptr, size_t hlen = 0);
void cls_from_shufti(const uint8_t *lo, const uint8_t *hi, uint8_t cls[32]);
void cls_from_truffle(const uint8_t *m1, const uint8_t *m2, uint8_t cls[32]);

} // namespace vsa_rt

#endif
