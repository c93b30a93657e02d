/*
 * runtime.hip — host runtime of libvectorscan_amd.so.
 *
 *  - vsa_ctx: one HIP stream + device workspace (input staging, match
 *    buffers, radix-sort scratch, counters).  One per thread (the reference
 *    is reentrant per hs_scratch, src/scratch.h:249-272).
 *  - vsa_db: device copy of an HWLM blob plus the derived launch parameters
 *    (side registry keyed by the bytecode pointer: hs_database and
 *    hs_scratch layouts stay untouched).
 *  - vsa_scan_blocks: launch -> count -> (grow + relaunch on overflow) ->
 *    device radix sort into the reference callback order.
 *  - replay: the host half of the drop-in boundary.  The GPU emits every
 *    confirmed (end, bucket, chain) record with groups = ALL; the host walks
 *    them in order applying exactly confWithBit's sequential state
 *    (fdr_confirm_runtime.h:43-102): NOREPEAT against the last reported id,
 *    li->groups & control with control fed back from the callback,
 *    termination, and the INCLUDED_JUMP squash of later buckets at the same
 *    end (program_runtime.c:2985-2997).
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>
#include <chrono>
#include <cmath>
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

namespace {

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
};

} // namespace

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
    std::vector<int64_t> spans, live; /* build_plan scratch */
};

struct vsa_plan;

struct vsa_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    /* the stream's owner: shared by contexts made with vsa_ctx_create_shared,
     * destroyed with the last of them */
    std::shared_ptr<void> stream_ref;
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
    double last_kernel_ms = 0.0;
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

/* confirm waves for a measured confirm-candidate rate (candidates per
 * scanned byte): one confirm wave keeps up with ~1e-4 (cfg 4); past that it
 * becomes the bound and more waves (fewer scanners) pay off */
static uint32_t nconf_for_rate(double rate) {
    /* measured (4 GiB, FDR): 5k literals (5e-5) best at 1; 10k (2.5e-4)
     * equal; 20k (5.7e-3) 9.4 -> 5.2 ms at 2; 50k (0.26) 124 -> 68 ms at 2.
     * With scanner expansion (use_xp, on from 2 waves; 16-B ring entries):
     * 20k 2.47 / 2.32 / 2.70 ms at 1 / 2 / 3 waves, 50k 62.9 / 34.1 / 30.6
     * ms (profiles/r03_xp.jsonl; 4 fits no better than 3 beside a
     * domain-14 table) */
    /* Round 4, with scanner expansion on from 4e-4 (1e-3 until late round 4) (xp_for_rate), the
     * confirm waves only confirm: 20k literals (2.7e-3) 1.80 / 1.85 / 1.99
     * ms at 1 / 2 / 3 waves, 50k in split passes (8.9e-3 per pass) 6.22 /
     * 5.34 / 6.13 (profiles/r04j_xp_cost.jsonl) */
    return rate > 0.05 ? 3u : rate > 5e-3 ? 2u : 1u;
}

/* scanner expansion past this confirm-candidate rate (use_xp): 4 GiB
 * cfg-4 corpus, one confirm wave, expansion off / on
 * (profiles/r04al_xp_10k.jsonl): 10k literals (1.4e-4) 1.18 / 1.27 ms, 15k
 * (6.6e-4) 1.51-1.53 / 1.47 ms, 20k (2.7e-3) 2.49 / 1.80 (r04j) */
static bool xp_for_rate(double rate) { return rate > 4e-4; }

/* VECTORSIZE of the reference build emulated where results depend on it:
 * shuftiDoubleExec's per-block lanes and the Teddy loop shape of the flood
 * shortcut (flood.cpp) */
static uint32_t g_vector_size = 64;

namespace {

/* ----------------------------------------------------------- helpers -- */

int ensure_out(vsa_ctx *c, uint64_t need) {
    Workspace &w = c->ws;
    if (need <= w.out_cap && w.d_tmp) return VSA_OK;
    uint64_t cap = std::max<uint64_t>(need + need / 4, 1u << 16);
    for (int i = 0; i < 2; i++) {
        if (w.d_keys[i]) (void)hipFree(w.d_keys[i]);
        if (w.d_ids[i]) (void)hipFree(w.d_ids[i]);
        w.d_keys[i] = nullptr;
        w.d_ids[i] = nullptr;
        VSA_CHECK(hipMalloc(&w.d_keys[i], cap * 8));
        VSA_CHECK(hipMalloc(&w.d_ids[i], cap * 4));
    }
    if (w.d_tmp) (void)hipFree(w.d_tmp);
    w.d_tmp = nullptr;
    size_t bytes = 0;
    hipcub::DoubleBuffer<uint64_t> kb(w.d_keys[0], w.d_keys[1]);
    hipcub::DoubleBuffer<uint32_t> vb(w.d_ids[0], w.d_ids[1]);
    VSA_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kb, vb, (int)std::min<uint64_t>(cap, 0x7fffffff), 0, 64, c->stream));
    VSA_CHECK(hipMalloc(&w.d_tmp, bytes));
    w.tmp_bytes = bytes;
    w.out_cap = cap;
    return VSA_OK;
}

int ensure_in(vsa_ctx *c, size_t need) {
    Workspace &w = c->ws;
    if (need <= w.in_cap) return VSA_OK;
    if (w.d_in) (void)hipFree(w.d_in);
    w.d_in = nullptr;
    size_t cap = std::max<size_t>(need + 64, 1u << 20);
    VSA_CHECK(hipMalloc(&w.d_in, cap));
    w.in_cap = cap;
    return VSA_OK;
}

/* the per-call block table and segment map share one device allocation and
 * one pinned mirror, laid out per call (the map right after this call's
 * blocks), so a call uploads them with a single copy of just their bytes */
constexpr size_t TAB_ALIGN = 256;

/* drop-in inputs up to this size are staged through pinned memory: one
 * host memcpy and one asynchronous DMA instead of a pageable copy */
constexpr size_t PIN_STAGE_MAX = (size_t)8 << 20;

int ensure_hin(vsa_ctx *c, size_t need) {
    Workspace &w = c->ws;
    if (need <= w.h_in_cap) return VSA_OK;
    if (w.h_in) (void)hipHostFree(w.h_in);
    w.h_in = nullptr;
    w.h_in_cap = 0;
    const size_t cap = std::max<size_t>(need, 64 << 10);
    VSA_CHECK(hipHostMalloc((void **)&w.h_in, cap, hipHostMallocDefault));
    w.h_in_cap = cap;
    return VSA_OK;
}

int ensure_tables(vsa_ctx *c, uint32_t nb, uint64_t nsegs, bool keep_blocks = false) {
    Workspace &w = c->ws;
    const size_t seg_off = ((size_t)nb * sizeof(VsaBlock) + TAB_ALIGN - 1) & ~(TAB_ALIGN - 1);
    const size_t need = seg_off + nsegs * sizeof(uint32_t);
    if (need > w.tab_cap) {
        VsaBlock *old = w.h_blocks;
        if (w.d_blocks) (void)hipFree(w.d_blocks);
        w.d_blocks = w.h_blocks = nullptr;
        w.tab_cap = 0;
        const size_t cap = std::max<size_t>(need + need / 4, 64 << 10);
        VSA_CHECK(hipMalloc(&w.d_blocks, cap));
        VSA_CHECK(hipHostMalloc((void **)&w.h_blocks, cap, hipHostMallocDefault));
        /* the block table already written into the old mirror */
        if (keep_blocks && old) memcpy(w.h_blocks, old, (size_t)nb * sizeof(VsaBlock));
        if (old) (void)hipHostFree(old);
        w.tab_cap = cap;
    }
    w.d_segblk = (uint32_t *)((uint8_t *)w.d_blocks + seg_off);
    w.h_segblk = (uint32_t *)((uint8_t *)w.h_blocks + seg_off);
    return VSA_OK;
}

/* Each launch is checked with hipGetLastError() right after it.  That call
 * returns (and clears) the thread's last error from ANY earlier HIP call,
 * including ignored statuses of free / destroy paths or another library's
 * calls on this thread, so the stale value is dropped immediately before the
 * launch: the check after it then sees this launch's error only. */
inline void drop_stale_error() { (void)hipGetLastError(); }

int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

/* work stealing inside a workgroup (kernels.hip): a wave out of segments
 * steals when another has at least this many sweep groups (4 KiB)
 * unclaimed; VSA_STEAL=0 turns it off (the plan then cuts large blocks into
 * shrinking segments instead) */
uint32_t steal_min() {
    static const uint32_t v = (uint32_t)std::max(0, env_int("VSA_STEAL", 4));
    return v;
}

int bits_for(uint64_t v) {
    int b = 0;
    while (v) {
        b++;
        v >>= 1;
    }
    return b;
}

template <int MODE, bool XP = false, bool SPLIT = false>
int launch_lit(vsa_ctx *c, const VsaLitParams &P, size_t lds) {
    auto fn = vsa_lit_scan<MODE, XP, SPLIT>;
    /* the dynamic-LDS limit is raised once per device and kernel (the call
     * costs a few us, a drop-in scan ~25 us) */
    static std::atomic<int> lds_set[64];
    std::atomic<int> &ls = lds_set[c->device & 63];
    if (ls.load(std::memory_order_relaxed) < (int)lds) {
        VSA_CHECK(hipFuncSetAttribute((const void *)fn,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        int cur = ls.load(std::memory_order_relaxed);
        while (cur < (int)lds && !ls.compare_exchange_weak(cur, (int)lds)) {
        }
    }
    /* one persistent 16-wave workgroup per segment list (at most one per
     * CU: build_plan) */
    const uint32_t grid = std::max<uint32_t>(1, c->launch.grid);
    /* diagnostic (VSA_PRINT_LAUNCH=1): every literal-scan launch's shape */
    static const bool print_launch = getenv("VSA_PRINT_LAUNCH") != nullptr;
    if (print_launch)
        fprintf(stderr,
                "vsa launch: mode %d xp %d grid %u nsegs %llu nblocks %u lds %zu qcap %u nconf %u "
                "end_par %u data %p blocks %p seg_desc %p out_cap %llu bins %p\n",
                MODE, (int)XP, grid, (unsigned long long)P.nsegs, P.nblocks, lds, P.qcap, P.nconf,
                P.end_par, (const void *)P.data, (const void *)P.blocks,
                (const void *)P.seg_desc, (unsigned long long)P.out_cap, (void *)P.bin_counts);
    /* the timing events ride on the dispatch packet itself
     * (hipExtLaunchKernel): separate hipEventRecord markers before and after
     * put two more packets between the scan and its sort on the stream */
    hipEvent_t e0 = c->launch.ev_start;
    hipEvent_t e1 = P.end_par == 1 ? nullptr : c->launch.ev_stop; /* split: the 2nd pass */
    c->launch.ev_start = nullptr;
    if (e1) c->launch.ev_stop = nullptr;
    drop_stale_error();
    hipExtLaunchKernelGGL(fn, dim3(grid), dim3(LIT_THREADS), (uint32_t)lds, c->stream, e0, e1, 0u,
                          P);
    VSA_CHECK(hipGetLastError());
    return VSA_OK;
}

/* dynamic LDS = table + one candidate ring per scanning wave (power of
 * two, 4..64 chunk entries of ent bytes: 48 FDR / Teddy, 64 Fat Teddy, 32
 * noodle; a push of up to 64 lanes is split into ring-sized batches) + slot
 * bitmaps */
size_t plan_lds(size_t tab, uint32_t slot_words, size_t ent, uint32_t *qcap,
                size_t budget = LDS_BUDGET, uint32_t nconf = 1) {
    const size_t waves = LIT_WAVES - nconf;
    /* the confirm waves' private queues (kernels.hip PQ_ENTRIES x 16 B) */
    const size_t extra = nconf == 1 ? 512 * 16 : (size_t)nconf * 256 * 16;
    const size_t slots = ((size_t)slot_words * 4 + 15) & ~(size_t)15;
    tab = (tab + 15) & ~(size_t)15;
    size_t rest = budget > tab + slots + extra ? budget - tab - slots - extra : 0;
    uint32_t q = 4;
    while (q < 64 && waves * (size_t)(2 * q) * ent <= rest) q *= 2;
    *qcap = q;
    return tab + waves * (size_t)q * ent + slots + extra;
}

/* the confirm-wave count of a launch: the db's adapted value (or
 * VSA_NCONF), lowered until the LDS plan fits */
uint32_t launch_nconf(const vsa_db *db, size_t tab, size_t ent, size_t budget) {
    uint32_t nc = db->nconf.load(std::memory_order_relaxed);
    if (const char *e = getenv("VSA_NCONF")) nc = (uint32_t)std::min(4, std::max(1, atoi(e)));
    uint32_t q;
    while (nc > 1 && plan_lds(tab, db->slot_words, ent, &q, budget, nc) > budget) nc--;
    return nc;
}

/* Scanner expansion (kernels.hip xp_push) for large literal sets: the
 * scanning waves expand candidate bits and apply the slot-bitmap prefilter,
 * the confirm waves only confirm.  On once the db's measured candidate rate
 * passed 4e-4 per byte (xp_for_rate); VSA_XP=0 / 1 forces it off / on. */
bool use_xp(const vsa_db *db) {
    if (const char *e = getenv("VSA_XP")) return atoi(e) != 0;
    return db->xp.load(std::memory_order_relaxed);
}

/* the binned sort (kernels.hip vsa_bin_finish) replaces the library sort
 * unless the caller wants the records unsorted (or a recent launch crowded
 * a bin, bin_skip) */
bool use_bins(const vsa_ctx *c) {
    return !(c->launch.flags & VSA_SCAN_UNSORTED) && c->bin_skip == 0;
}

/* bins of 2^bin_shift end positions, at most VSA_SORT_BINS over the span */
uint32_t bin_shift_for(int end_bits) {
    return end_bits > (int)VSA_SORT_BIN_BITS ? (uint32_t)end_bits - VSA_SORT_BIN_BITS : 0u;
}

uint64_t *bstage_keys(Workspace &w) { return (uint64_t *)w.d_bstage; }
uint32_t *bstage_ids(Workspace &w) {
    return (uint32_t *)(w.d_bstage + (size_t)VSA_SORT_BINS * VSA_SORT_BIN_MAX * sizeof(uint64_t));
}
uint32_t *bin_counts_of(vsa_ctx *c, uint32_t par) { return c->ws.d_bins + par * VSA_SORT_BINS; }

/* The binned sort behind the scan: the scan kernel stages each record
 * in its bin as it emits it (VsaLitParams.bin_keys / bin_ids; the records
 * are written nowhere else), and one
 * vsa_bin_finish launch sorts the bins into place, clears the other count
 * buffer for the next launch and publishes the counters to the host.  It
 * reads the record count and the overflow flags from d_counters, so it is
 * queued before the host has seen either (an overflowed launch leaves it
 * idle).  Measured and dropped (rounds 3-4): the four-launch chain (count,
 * scan, scatter, per-bin sort; 29 us against 18 us of step - kernel,
 * profiles/r04c_sort_ab.jsonl), its histogram as a separate launch, a side
 * stream for the sort (no gain, profiles/r03_sidesort.jsonl), and fused
 * launches behind a last-workgroup ticket (107 + 342 us: every workgroup's
 * agent-scope release serializes, profiles/r03_sort_fused_trace.csv). */
int queue_bin_sort(vsa_ctx *c) {
    Workspace &w = c->ws;
    const uint32_t par = c->bin_par;
    const bool fbd = c->fb.armed >= 0 && c->fb.dev;
    drop_stale_error();
    hipLaunchKernelGGL(vsa_bin_finish, dim3(VSA_SORT_BINS / 64), dim3(1024), 0, c->stream,
                       bin_counts_of(c, par), bin_counts_of(c, par ^ 1u), bstage_keys(w),
                       bstage_ids(w), w.d_keys[1], w.d_ids[1], (uint64_t)w.out_cap,
                       c->ws.d_counters, c->ws.d_pub, (unsigned long long)++c->pub_seq,
                       fbd ? c->fb.d_rec : nullptr, fbd ? c->fb.d : nullptr,
                       fbd ? 2 * c->fb.grid : 0u, (uint64_t *)c->launch.pack_dst,
                       c->launch.pack_cap);
    /* the pack buffer is filled by this launch only: a rescan (complete_scan)
     * must not write into a buffer a collective may be reading; the caller
     * repacks after it (vsa_scan_pack) */
    c->launch.pack_dst = nullptr;
    VSA_CHECK(hipGetLastError());
    c->bins_clean[par ^ 1u] = true;
    c->bin_par = par ^ 1u;
    return VSA_OK;
}

/* Schedule feedback: the XCDs of a box do not run equally fast (measured
 * 4-10 % apart on a 4 GiB scan: profiles/r04e_waves_4g.txt, r04g_waves_*),
 * and with equal static shares the slowest sets the kernel's end.  A large
 * per-workgroup-list launch (>= 64 workgroups, >= 256 MiB) records each
 * workgroup's entry and end (and XCD) into fine-grained host memory; after
 * it the host moves each XCD's weight toward the rate it showed (half the
 * way, within 0.7-1.3 of the mean: noodle at 1 GiB reached the earlier
 * 0.85-1.15 clamp, its XCDs streaming 25 % apart, profiles/r04m_waves_noodle_1g.txt)
 * and the next plan gives each
 * workgroup a share in proportion (build_plan wg_w).  Results are
 * unaffected (order-exact output); VSA_XCD_FEEDBACK=0 turns it off. */
bool xcd_feedback_on() {
    static const bool v = env_int("VSA_XCD_FEEDBACK", 1) != 0;
    return v;
}

/* arm the feedback record of the next launch (set: FbSet kind) */
void arm_feedback(vsa_ctx *c, int set, uint32_t grid, uint64_t bytes, bool small) {
    c->fb.armed = xcd_feedback_on() && c->fb.h && grid >= 64 && grid <= 1024 &&
                  bytes >= (256u << 20) && !small ? set : -1;
    c->fb.grid = grid;
    /* a scan whose counters vsa_bin_finish publishes records in device
     * memory and rides on the publish; otherwise host stores */
    c->fb.dev = c->fb.armed >= 0 && c->fb.d_rec && c->launch.bins && !small;
    if (c->fb.armed >= 0) memset(c->fb.h, 0, 2 * grid * sizeof(unsigned long long));
}

/* the feedback kind of a literal scan */
int fb_set_of(const vsa_db *db) { return db && db->type == HWLM_ENGINE_NOOD ? 1 : 0; }

/* which weights a plan was built with: kind and version */
uint64_t fb_key_of(const vsa_ctx *c, const vsa_db *db) {
    const int si = fb_set_of(db);
    return ((uint64_t)si << 32) | c->fb.set[si].version;
}

/* One feedback record (h: [b] = xcc << 60 | end, [G + b] = entry, 100 MHz)
 * into a weight set; false if the record is incomplete. */
bool feedback_update(vsa_ctx::FbSet &F, const volatile unsigned long long *h, uint32_t G) {
    const unsigned long long M60 = (1ULL << 60) - 1;
    unsigned long long t0 = ~0ULL;
    for (uint32_t b = 0; b < G; b++) {
        if (!h[b] || !h[G + b]) return false; /* a workgroup without a record */
        t0 = std::min(t0, (unsigned long long)h[G + b]);
    }
    double sum[8] = {0}, cnt[8] = {0};
    uint8_t xs[1024];
    for (uint32_t b = 0; b < G; b++) {
        const uint32_t x = (uint32_t)(h[b] >> 60) & 7u;
        const unsigned long long e = h[b] & M60;
        if (e <= t0) return false;
        xs[b] = (uint8_t)x;
        sum[x] += (double)(e - t0);
        cnt[x] += 1;
    }
    memcpy(F.xcc, xs, G);
    double tm = 0, nx = 0;
    for (int x = 0; x < 8; x++)
        if (cnt[x]) {
            tm += sum[x] / cnt[x];
            nx += 1;
        }
    if (nx < 2) return false;
    tm /= nx;
    float nw[8];
    double mean = 0;
    /* the launch ran with the applied weights wa: the weights that would
     * have ended every XCD together are wa * tm / tx; the estimate w moves
     * half-way toward them (an average over launches, not a walk: basing
     * it on w itself while wa lagged ran w into the clamps, r04s) */
    for (int x = 0; x < 8; x++) {
        nw[x] = F.w[x];
        if (cnt[x]) {
            const double tx = sum[x] / cnt[x];
            nw[x] = (float)(0.5 * F.w[x] + 0.5 * F.wa[x] * tm / tx);
        }
    }
    for (int x = 0; x < 8; x++) mean += nw[x];
    mean /= 8;
    /* the estimate moves every launch; the weights plans are built with
     * follow it only when it left them by more than 2 % (per-launch noise
     * is ~1 %), and then at most once per 16 records after the first few:
     * a changed plan is a rebuild, for a prebuilt plan an upload queued on
     * the scan stream (vsa_scan_plan), measured at ~10-20 us of step time
     * each (profiles/r04r/: applied at every > 1 % move, step - kernel grew
     * from 14 to 20-28 us) */
    bool moved = false;
    for (int x = 0; x < 8; x++) {
        nw[x] = std::min(1.3f, std::max(0.7f, (float)(nw[x] / mean)));
        moved = moved || std::fabs(nw[x] - F.wa[x]) > 0.02f;
    }
    memcpy(F.w, nw, sizeof(nw));
    const bool first = !F.known;
    F.known = true;
    F.since++;
    const bool settling = F.version < 4;
    if (!first && (!moved || (!settling && F.since < 16))) return true;
    F.since = 0;
    memcpy(F.wa, nw, sizeof(nw));
    for (int b = 0; b < 1024; b++) F.wg[b] = F.wa[F.xcc[b] & 7];
    F.version++;
    return true;
}

void take_feedback(vsa_ctx *c) {
    const int si = c->fb.armed;
    if (si < 0) return;
    c->fb.armed = -1;
    (void)feedback_update(c->fb.set[si], c->fb.h, c->fb.grid);
}

/* diagnostic per-wave log (vsa_set_wave_log; the kernel writes it under
 * debug flag 4096) */
static unsigned long long *g_wave_log = nullptr;

int launch_scan_kernel(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data, uint32_t nb,
                       uint64_t nsegs);

int launch_scan(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data, uint32_t nb,
                uint64_t nsegs) {
    if (!c->ctr_clean)
        VSA_CHECK(hipMemsetAsync(c->ws.d_counters, 0, 144 * sizeof(unsigned long long), c->stream));
    c->ctr_clean = false;
    c->launch.published = false;
    /* not for the drop-in calls, whose few records the host sorts (a
     * larger result takes the library sort) */
    c->launch.bins = use_bins(c) && !(c->launch.flags & SCAN_HOST_SORT_SMALL);
    if (c->launch.bins && !c->ws.d_bstage)
        VSA_CHECK(hipMalloc(&c->ws.d_bstage, (size_t)VSA_SORT_BINS * VSA_SORT_BIN_MAX *
                                                 (sizeof(uint64_t) + sizeof(uint32_t))));
    const uint32_t par = c->bin_par;
    if (c->launch.bins && !c->bins_clean[par])
        VSA_CHECK(hipMemsetAsync(bin_counts_of(c, par), 0, VSA_SORT_BINS * sizeof(uint32_t),
                                 c->stream));
    c->bins_clean[par] = false;
    /* drop-in calls (a few records, sorted by the host) skip the kernel
     * timing and get their counters and records published (no copies) */
    const bool small = (c->launch.flags & SCAN_HOST_SORT_SMALL) != 0;
    c->launch.ev_start = small ? nullptr : c->ev0;
    c->launch.ev_stop = small ? nullptr : c->ev1;
    arm_feedback(c, fb_set_of(db), c->launch.grid, c->launch.bytes, small);
    c->lit_launches++;
    int r = launch_scan_kernel(c, db, d_data, nb, nsegs);
    c->launch.ev_start = c->launch.ev_stop = nullptr;
    if (r != VSA_OK) return r;
    if (small) {
        drop_stale_error();
        hipLaunchKernelGGL(vsa_publish, dim3(1), dim3(256), 0, c->stream, c->ws.d_counters,
                           c->ws.d_pub, (unsigned long long)++c->pub_seq, 144u,
                           (const uint64_t *)c->ws.d_keys[0], (const uint32_t *)c->ws.d_ids[0],
                           PUB_RECS);
        VSA_CHECK(hipGetLastError());
        c->launch.published = true;
        c->launch.dev_sort = false;
        c->ctr_clean = true;
        return VSA_OK;
    }
    /* the binned sort queues behind the scan with no host round trip: its
     * kernels read the record count and the overflow flag on the device
     * (finish_scan falls back to the library sort if a bin overflowed) */
    c->launch.dev_sort = c->launch.bins;
    if (!c->launch.dev_sort) return VSA_OK;
    /* the sort zeroes the next launch's bin counts and publishes the
     * counters to the host, zeroing them */
    int r2 = queue_bin_sort(c);
    if (r2 != VSA_OK) return r2;
    c->launch.published = true;
    c->ctr_clean = true;
    return VSA_OK;
}

int launch_scan_kernel(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data, uint32_t nb,
                       uint64_t nsegs) {
    Workspace &w = c->ws;
    VsaLitParams P;
    memset(&P, 0, sizeof(P));
    P.data = d_data;
    P.blocks = c->launch.d_blocks;
    P.seg_desc = c->launch.d_segblk;
    P.wg_seg = c->launch.d_segblk + 4 * nsegs;
    P.wg_bins = c->launch.d_segblk + 4 * nsegs + c->launch.grid + 1; /* plan_wg_bins */
    P.nblocks = nb;
    P.steal = steal_min();
    P.nsegs = nsegs;
    P.out_keys = w.d_keys[0];
    P.out_ids = w.d_ids[0];
    P.out_cap = w.out_cap;
    P.bin_counts = c->launch.bins ? bin_counts_of(c, c->bin_par) : nullptr;
    P.bin_shift = bin_shift_for(c->launch.end_bits);
    P.bin_keys = c->launch.bins ? bstage_keys(w) : nullptr;
    P.bin_ids = c->launch.bins ? bstage_ids(w) : nullptr;
    P.counters = w.d_counters;
    P.wg_time = c->fb.armed >= 0 ? (c->fb.dev ? c->fb.d_rec : c->fb.d) : nullptr;
    P.wave_log = g_wave_log;
    {
        const char *e = getenv("VSA_DEBUG_FLAGS");
        P.dbg = e ? (uint32_t)atoi(e) : 0u;
    }
    if (db->type == HWLM_ENGINE_NOOD) {
        const uint32_t ml = db->nood.msk_len; /* 1..8 */
        P.nood_msk = db->nood.msk << (8 * (8 - ml));
        P.nood_cmp = db->nood.cmp << (8 * (8 - ml));
        P.nood_len = ml;
        P.nood_id = db->nood.id;
        for (int b = 0; b < 16; b++) P.slot_off[b] = 0xffffffffu;
        P.nconf = 1;
        size_t lds = plan_lds(0, 0, 32, &P.qcap);
        return launch_lit<VSA_MODE_NOOD>(c, P, lds);
    }
    const uint8_t *d_eng = db->d_blob + VSA_ROUNDUP_CL(sizeof(HWLM));
    P.table = db->d_table; /* derived FDR4 table / Teddy byte table */
    P.table_entries = db->table_entries;
    P.dmask = db->dmask;
    P.state_lo = db->state_lo;
    P.state_hi = db->state_hi;
    const uint32_t conf_offset_in_eng = ((const uint32_t *)(db->hblob + VSA_ROUNDUP_CL(sizeof(HWLM))))[4];
    P.conf_base = d_eng + conf_offset_in_eng;
    memcpy(P.conf_off, db->conf_off, sizeof(P.conf_off));
    P.slotmap = db->d_slots;
    P.slot_words = db->slot_words;
    memcpy(P.slot_off, db->slot_off, sizeof(P.slot_off));
    memcpy(P.slot_bits, db->slot_bits, sizeof(P.slot_bits));
    P.pf_mult = db->pf_mult;
    if (db->mode == VSA_MODE_FDR4) {
        const size_t tb = (size_t)db->table_entries * 4;
        const bool xp = use_xp(db);
        const size_t ent = xp ? 16 : 48; /* QEnt or chunk entries */
        P.nconf = launch_nconf(db, tb, ent, LDS_BUDGET);
        size_t lds = plan_lds(tb, db->slot_words, ent, &P.qcap, LDS_BUDGET, P.nconf);
        if (lds > LDS_BUDGET) return VSA_E_INVALID;
        if (!db->split)
            return xp ? launch_lit<VSA_MODE_FDR4, true>(c, P, lds)
                      : launch_lit<VSA_MODE_FDR4>(c, P, lds);
        auto go = [&](const VsaLitParams &Q) {
            return xp ? launch_lit<VSA_MODE_FDR4, true, true>(c, Q, lds)
                      : launch_lit<VSA_MODE_FDR4, false, true>(c, Q, lds);
        };
        /* split passes: the ends whose byte has bit 0 clear, with the table
         * of the literals ending in such a byte, then the others; each end
         * is one pass's, and the confirm (the blob's, unchanged) can only
         * accept a literal whose last byte is the end's, so no record is
         * found twice.  The records of both go to the same output and bins. */
        P.end_par = 1;
        if (int r = go(P)) return r;
        P.end_par = 2;
        P.table = (const uint64_t *)db->d_table2;
        return go(P);
    }
    /* Teddy / Fat Teddy: the 64 KiB table sits at LDS 0x10000 (kernels.hip
     * TEDDY_TAB_LDS), ring + slot bitmaps below it after the static LDS */
    const size_t below = 0x10000 - (160 * 1024 - LDS_BUDGET);
    const size_t teddy_dyn = 128 * 1024;
    if (db->mode == VSA_MODE_TEDDY) {
        P.nconf = launch_nconf(db, 0, 48, below);
        if (plan_lds(0, db->slot_words, 48, &P.qcap, below, P.nconf) > below) return VSA_E_INVALID;
        return launch_lit<VSA_MODE_TEDDY>(c, P, teddy_dyn);
    }
    P.nconf = launch_nconf(db, 0, 64, below);
    if (plan_lds(0, db->slot_words, 64, &P.qcap, below, P.nconf) > below) return VSA_E_INVALID;
    return launch_lit<VSA_MODE_FAT>(c, P, teddy_dyn);
}

/* wait for the scan stream by polling an event: a blocking wait wakes on a
 * coarse tick (measured ~1 ms after a 0.3 ms scan), which would set the
 * wall time of every scan shorter than that.  Past 50 ms of polling the
 * wait blocks (long scans do not need the precision). */
hipError_t wait_stream(vsa_ctx *c) {
    hipError_t e = hipEventRecord(c->ev_done, c->stream);
    if (e != hipSuccess) return e;
    /* spin ~100 us, then yield the core between polls (the host replay
     * pool and the CPU baseline share the host) */
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; i++) {
        e = hipEventQuery(c->ev_done);
        if (e != hipErrorNotReady) return e;
        /* not ready is a poll's answer, not an error: it must not stay the
         * thread's last error for the next launch check */
        (void)hipGetLastError();
        if ((i & 15) == 15) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(50)) return hipStreamSynchronize(c->stream);
            if (dt > std::chrono::microseconds(100)) sched_yield();
        }
    }
}

/* wait for the vsa_publish of sequence seq (spin ~100 us, then yield;
 * past 50 ms the stream is synchronized and checked) */
hipError_t wait_published(vsa_ctx *c, uint64_t seq) {
    volatile unsigned long long *h = c->ws.h_pub;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; i++) {
        if (h[0] == seq) break;
        if ((i & 15) == 15) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(50)) {
                hipError_t e = hipStreamSynchronize(c->stream);
                if (e != hipSuccess) return e;
                if (h[0] != seq) return hipErrorUnknown;
                break;
            }
            if (dt > std::chrono::microseconds(100)) sched_yield();
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return hipSuccess;
}

int finish_scan(vsa_ctx *c, uint32_t flags, int end_bits, uint64_t *n_out) {
    Workspace &w = c->ws;
    if (c->launch.published) {
        VSA_CHECK(wait_published(c, c->pub_seq));
        for (int i = 0; i < 16; i++) w.h_counters[i] = w.h_pub[1 + i];
    } else {
        VSA_CHECK(hipMemcpyAsync(w.h_counters, w.d_counters, 16 * sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(wait_stream(c));
    }
    uint64_t n = w.h_counters[0];
    c->last_cand = w.h_counters[2];
    take_feedback(c);
    /* adapt the db's confirm-wave count to the measured candidate rate
     * (over a representative launch; not under diagnostic flags) */
    if (c->launch.db && c->launch.bytes >= (16u << 20) && !getenv("VSA_DEBUG_FLAGS")) {
        /* split passes: each launch confirms about half the candidates */
        const double passes = c->launch.db->split ? 2.0 : 1.0;
        const double rate = (double)c->last_cand / passes / (double)c->launch.bytes;
        const uint32_t want = nconf_for_rate(rate);
        uint32_t cur = c->launch.db->nconf.load(std::memory_order_relaxed);
        while (want > cur && !c->launch.db->nconf.compare_exchange_weak(cur, want)) {
        }
        if (xp_for_rate(rate)) c->launch.db->xp.store(true, std::memory_order_relaxed);
    }
    if (getenv("VSA_DEBUG_FLAGS") && w.h_counters[3]) {
        fprintf(stderr, "vsa: %llu queued confirm keys differ from HBM\n",
                (unsigned long long)w.h_counters[3]);
    }
    if (!(flags & SCAN_HOST_SORT_SMALL)) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->last_kernel_ms = ms;
        /* a not-yet-observed event (the published path completes on the
         * publish, not on ev1) must not leave hipErrorNotReady as the
         * thread's last error for the next launch check */
        (void)hipGetLastError();
    }
    if (c->bin_skip) c->bin_skip--;
    /* A crowded bin (> VSA_SORT_BIN_MAX records): the launch's records exist
     * only in the bins, so it runs again without them (complete_scan), and
     * the next launches (likely as dense) skip them too, for longer after
     * each crowded binned launch in a row (bin_backoff).  Checked before the
     * output overflow, so a launch that both crowded a bin and outgrew the
     * output (a first dense scan on a fresh context: out_cap starts at 64 K)
     * runs once more, without bins, not twice. */
    const bool crowded = c->launch.dev_sort && w.h_counters[VSA_CTR_BIN_OVERFLOW];
    if (crowded) {
        c->bin_skip = c->bin_backoff;
        c->bin_backoff = std::min<uint32_t>(4096u, c->bin_backoff * 4u);
    } else if (c->launch.dev_sort) {
        c->bin_backoff = 16;
    }
    if (crowded || n > w.out_cap) return VSA_E_OVERFLOW;
    c->cur = 0;
    /* internal: a few records are sorted by the host caller after its copy
     * (the device sort's launches cost more than sorting them there) */
    c->host_sort = (flags & SCAN_HOST_SORT_SMALL) && n <= HOST_SORT_MAX;
    if (c->launch.dev_sort) {
        /* sorted by the binned sort queued in launch_scan, into buffer 1
         * (a single record too: buffer 0 is not written in this mode) */
        c->cur = 1;
    } else if (n > 1 && !(flags & VSA_SCAN_UNSORTED) && !c->host_sort) {
        hipcub::DoubleBuffer<uint64_t> kb(w.d_keys[0], w.d_keys[1]);
        hipcub::DoubleBuffer<uint32_t> vb(w.d_ids[0], w.d_ids[1]);
        size_t bytes = w.tmp_bytes;
        int eb = std::min(64, end_bits + VSA_KEY_END_SHIFT);
        VSA_CHECK(hipcub::DeviceRadixSort::SortPairs(w.d_tmp, bytes, kb, vb, (int)n, 0, eb,
                                                      c->stream));
        c->cur = kb.selector;
    }
    c->last_n = n;
    *n_out = n;
    return VSA_OK;
}

int complete_scan(vsa_ctx *c, uint64_t *n_out);

/* complete an asynchronous scan still in flight (as vsa_scan_wait) */
int finish_pending(vsa_ctx *c) {
    if (!c->pending) return VSA_OK;
    c->pending = false;
    uint64_t n = 0;
    return complete_scan(c, &n);
}

constexpr uint32_t SEG_GROUP_SHIFT = 24;
constexpr uint32_t SEG_GROUP_MAX = 255;
constexpr uint32_t PLAN_MAX_BLOCKS = VSA_MAX_BLOCKS; /* 20-bit block field of the keys */

/* Sort bins a workgroup owns alone (kernels.hip counts their records in
 * LDS: no global returning atomic per record).  Workgroup b may report ends
 * only inside its segments; their hull [lo_b, hi_b) (data-relative, the
 * coordinates the bins are cut in) is taken over its segments' end ranges
 * (a part of a block: its KiB range cut to the block; a group: its blocks).
 * When the hulls of different workgroups do not overlap -- shares are cut
 * in block order, so they do not unless blocks overlap or come out of
 * order -- every bin lying wholly inside hull b holds only workgroup b's
 * records.  Appended to segblk after the list bounds: 2 words per
 * workgroup, the bins [lo, hi) (hi - lo <= VSA_LBINS; 0, 0 = none). */
void plan_wg_bins(BatchPlan &pl, const VsaBlock *blocks, int64_t mis) {
    const uint32_t G = pl.grid;
    const uint64_t base = 4 * pl.nsegs;
    std::vector<int64_t> hlo(G, INT64_MAX), hhi(G, INT64_MIN);
    for (uint32_t b = 0; b < G; b++) {
        for (uint32_t sg = pl.segblk[base + b]; sg < pl.segblk[base + b + 1]; sg++) {
            const uint32_t *d = &pl.segblk[4 * (uint64_t)sg];
            const uint32_t first = d[0] & 0xffffffu, cnt = d[0] >> 24;
            int64_t lo, hi;
            if (cnt == 0) {
                const VsaBlock &B = blocks[first];
                const int64_t s0 = B.org - mis + ((int64_t)d[1] << 10);
                lo = std::max<int64_t>((int64_t)B.base, s0);
                hi = std::min<int64_t>((int64_t)(B.base + B.len), s0 + ((int64_t)d[2] << 10));
            } else {
                lo = INT64_MAX;
                hi = INT64_MIN;
                for (uint32_t k = 0; k < cnt; k++) {
                    const VsaBlock &B = blocks[first + k];
                    if (!B.len) continue;
                    lo = std::min<int64_t>(lo, (int64_t)B.base);
                    hi = std::max<int64_t>(hi, (int64_t)(B.base + B.len));
                }
            }
            if (hi > lo) {
                hlo[b] = std::min(hlo[b], lo);
                hhi[b] = std::max(hhi[b], hi);
            }
        }
    }
    std::vector<uint32_t> order;
    for (uint32_t b = 0; b < G; b++)
        if (hhi[b] > hlo[b]) order.push_back(b);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hlo[a] < hlo[b]; });
    bool ok = true;
    for (size_t i = 1; i < order.size() && ok; i++) ok = hhi[order[i - 1]] <= hlo[order[i]];
    const uint32_t shift = bin_shift_for(pl.end_bits);
    const int64_t bs = (int64_t)1 << shift;
    for (uint32_t b = 0; b < G; b++) {
        uint32_t lo = 0, hi = 0;
        if (ok && hhi[b] > hlo[b]) {
            const int64_t l = (hlo[b] + bs - 1) >> shift, h = hhi[b] >> shift;
            if (h > l) {
                lo = (uint32_t)l;
                hi = (uint32_t)std::min<int64_t>(h, l + VSA_LBINS);
            }
        }
        pl.segblk.push_back(lo);
        pl.segblk.push_back(hi);
    }
}

int build_plan(const uint8_t *d_data, const uint64_t *offs, const uint64_t *lens,
               const uint64_t *starts, const uint64_t *hlens, const uint64_t *rlos,
               uint32_t nb, uint64_t waves, BatchPlan &pl, VsaBlock *out = nullptr,
               uint64_t ns = LIT_WAVES - 1, const float *wg_w = nullptr) {
    if (nb > PLAN_MAX_BLOCKS) return VSA_E_INVALID;
    /* the block table goes to `out` (a pinned mirror) or pl.blocks */
    if (!out) {
        pl.blocks.resize(nb);
        out = pl.blocks.data();
    }
    pl.segblk.clear();
    uint64_t span = 0;
    for (uint32_t i = 0; i < nb; i++) span = std::max(span, offs[i] + lens[i]);
    const int64_t mis = (int64_t)((uintptr_t)d_data & 15);
    /* scratch kept in the plan: a fresh multi-MB vector per call costs its
     * page faults every call */
    std::vector<int64_t> &spans = pl.spans, &live = pl.live;
    spans.assign(nb, -1); /* -1: nothing to scan */
    live.clear();
    live.reserve(nb);
    pl.bytes = 0;
    for (uint32_t i = 0; i < nb; i++) {
        VsaBlock &b = out[i];
        b.base = offs[i];
        b.len = lens[i];
        b.start = starts ? starts[i] : 0;
        b.rlo = rlos ? (int64_t)rlos[i] : 0;
        b.seg_first = 0;
        const int64_t len = (int64_t)b.len, st = (int64_t)b.start;
        b.hlen = hlens ? hlens[i] : 0;
        /* only the history is readable before the block: a write at offset
         * 1 with 1 history byte must not load the 15 bytes before the
         * buffer (the prologue's masked loads reach base - 8; a buffer at the
         * start of a mapping faulted, test_gpu_split_passes' stream part;
         * tests/test_plan.py checks the bound) */
        b.hist = (uint32_t)std::min<uint64_t>(b.hlen, 16);
        b.flags = b.hlen ? VSA_BLK_STREAM : 0;
        /* prepareZones fdr.c:625-659: short zone anchors at len - 16; with
         * history the look-back also covers start - 1 (getInitState) */
        b.zbase = (len - st > 16) ? st : len - 16;
        if (b.hlen) b.zbase = (len - st > 16) ? st - 1 : std::min(len - 16, st - 1);
        /* segments are 1 KiB-aligned (in data-aligned coordinates) and start
         * just before `start`: earlier positions cannot reach ends >= start */
        const int64_t blo = (int64_t)b.base + mis;
        b.org = (blo + std::max<int64_t>(0, st - 16)) & ~(int64_t)1023;
        if (st < len) {
            spans[i] = blo + len - b.org;
            live.push_back(spans[i]);
            pl.bytes += (uint64_t)(len - st);
        }
    }
    /* VSA_SEG_KB (tests): every piece and packed group at most this size */
    const uint64_t seg_kb = (uint64_t)std::max(0, env_int("VSA_SEG_KB", 0)) << 10;
    const bool group = !getenv("VSA_NO_GROUPS");
    const bool no_runs = getenv("VSA_NO_RUNS") != nullptr;
    uint32_t g_first = 0, g_n = 0;
    bool g_run = false; /* the open group can still be a run */
    int64_t g_span = 0;
    pl.nsegs = 0;
    pl.grid = 0;
    /* one 16-byte descriptor per segment (kernels.h VsaLitParams.seg_desc) */
    auto push_desc = [&](uint32_t info, uint64_t off, uint64_t len) {
        pl.segblk.push_back(info);
        pl.segblk.push_back((uint32_t)(off >> 10));
        pl.segblk.push_back((uint32_t)((len + 1023) >> 10));
        pl.segblk.push_back(0u);
        pl.nsegs++;
    };
    /* a packed segment of back-to-back blocks >= 1 KiB scanned from their
     * first byte is one range for the scan (VSA_BLK_RUN); a streaming write
     * in it has its history right before it (the hs corpus and vectored
     * layouts) */
    auto runnable = [&]() {
        if (no_runs || g_n < 2 || g_n > VSA_RUN_MAX) return false;
        for (uint32_t k = g_first; k < g_first + g_n; k++) {
            const VsaBlock &b = out[k];
            if (b.start || b.rlo || b.len < VSA_RUN_MIN_LEN) return false;
            if (k > g_first && b.base != out[k - 1].base + out[k - 1].len) return false;
        }
        return true;
    };
    auto flush = [&]() {
        if (g_n) {
            if (runnable()) out[g_first].flags |= VSA_BLK_RUN;
            push_desc(g_first | (g_n << SEG_GROUP_SHIFT), 0, 0);
        }
        g_n = 0;
        g_span = 0;
    };
    /* Per-workgroup lists (kernels.hip): the live bytes, in block order, are
     * split into G equal shares (or shares weighted per workgroup: schedule
     * feedback, wg_w), one list per workgroup.  With stealing a large block
     * is cut into one segment per wave of the share; without it
     * (VSA_STEAL=0) into segments of clamp(r / ns, min, max), r = the bytes
     * of the share still uncut (guided sizes).  Blocks shorter than half the
     * current size are packed whole (groups of up to SEG_GROUP_MAX blocks,
     * runs of up to VSA_RUN_MAX).  A wave's share of the list per group
     * (K = 1) measured 4-13 % faster on 2-64 KiB blocks than K = 2
     * (profiles/r04af_wg_k.txt).  A shared pool of small segments after the
     * lists (round 4) measured slower: 4 GiB 892 against 870 us, 32 MiB 47
     * against 28 us (profiles/r04f_pool_sweep.jsonl). */
    uint64_t T = 0;
    for (int64_t sp : live) T += (uint64_t)sp;
    const uint64_t smax = seg_kb ? seg_kb : (256u << 10);
    const uint64_t smin = seg_kb ? seg_kb : T <= (64u << 10) ? 1024u : (4u << 10);
    const uint64_t gmax = std::max<uint64_t>(1, waves / ns);
    const uint64_t G = std::max<uint64_t>(1, std::min(gmax, (T + ns * smin - 1) / (ns * smin)));
    std::vector<uint32_t> wg_first(G + 1, 0);
    uint64_t g = 0, acc = 0;
    /* the end of workgroup k's share: equal shares, or weighted per
     * workgroup */
    std::vector<double> cw;
    if (wg_w) {
        cw.resize(G);
        double a = 0;
        for (uint64_t k = 0; k < G; k++) cw[k] = (a += wg_w[k]);
    }
    auto cum = [&](uint64_t k) {
        if (!cw.empty()) return k + 1 >= G ? T : (uint64_t)((double)T * (cw[k] / cw[G - 1]));
        return (uint64_t)((unsigned __int128)T * (k + 1) / G);
    };
    auto advance = [&]() {
        while (g + 1 < G && acc >= cum(g)) wg_first[++g] = (uint32_t)pl.nsegs;
    };
    const uint64_t big = seg_kb ? seg_kb
                                : std::min<uint64_t>(16u << 20,
                                                     std::max(smin, ((T / G / ns) + 1023) &
                                                                        ~(uint64_t)1023));
    auto size_now = [&]() -> uint64_t {
        const uint64_t c = cum(g);
        const uint64_t r = c > acc ? c - acc : 0;
        uint64_t v = (r / ns + 1023) & ~(uint64_t)1023;
        return std::min(smax, std::max(smin, v));
    };
    for (uint32_t i = 0; i < nb; i++) {
        const int64_t sp = spans[i];
        if (sp < 0) {
            flush();
            continue;
        }
        uint64_t sz = size_now();
        if (group && 2 * (uint64_t)sp <= sz) {
            /* a group that can still be a run (runnable) is cut at
             * VSA_RUN_MAX blocks, so back-to-back 1 KiB blocks scan as runs
             * of 128 rather than as groups of 255 single blocks */
            const VsaBlock &bi = out[i];
            const bool elig = !no_runs && !bi.start && !bi.rlo && bi.len >= VSA_RUN_MIN_LEN;
            const bool cont = g_n && g_run && elig && bi.base == out[i - 1].base + out[i - 1].len;
            const uint32_t gcap = cont ? VSA_RUN_MAX : SEG_GROUP_MAX;
            if (g_n && (g_span + sp > (int64_t)sz || g_n >= gcap)) {
                flush();
                advance();
            }
            if (!g_n) g_run = elig;
            else g_run = g_run && elig && bi.base == out[i - 1].base + out[i - 1].len;
            if (!g_n) g_first = i;
            out[i].seg_first = pl.nsegs;
            g_n++;
            g_span += sp;
            acc += (uint64_t)sp;
            if (acc >= cum(g)) { /* the share ends here */
                flush();
                advance();
            }
            continue;
        }
        flush();
        advance();
        out[i].seg_first = pl.nsegs;
        for (uint64_t off = 0; off < (uint64_t)sp;) {
            /* with stealing, a part of a large block is one wave's share of
             * its workgroup's bytes: the waves balance by stealing sweep
             * groups, so no segment needs to be small (fewer segment
             * starts); without it, the guided size */
            sz = steal_min() ? big : size_now();
            /* a piece ends at its share's end: every workgroup gets its
             * share to the KiB */
            const uint64_t cg = cum(g);
            if (cg > acc) sz = std::min(sz, (cg - acc + 1023) & ~(uint64_t)1023);
            uint64_t piece = std::min<uint64_t>(sz, (uint64_t)sp - off);
            /* no sliver shorter than the minimum after this piece */
            if ((uint64_t)sp - off - piece < smin) piece = (uint64_t)sp - off;
            push_desc(i, off, piece);
            off += piece;
            acc += piece;
            advance();
        }
    }
    flush();
    for (uint64_t k = g + 1; k <= G; k++) wg_first[k] = (uint32_t)pl.nsegs;
    pl.grid = (uint32_t)G;
    pl.segblk.insert(pl.segblk.end(), wg_first.begin(), wg_first.end());
    pl.end_bits = bits_for(span);
    plan_wg_bins(pl, out, (int64_t)((uintptr_t)d_data & 15));
    return VSA_OK;
}

/* upload a plan's tables to device arrays */
int upload_plan(vsa_ctx *c, const BatchPlan &pl, VsaBlock *d_blocks, uint32_t *d_segblk) {
    if (!pl.blocks.empty()) {
        VSA_CHECK(hipMemcpyAsync(d_blocks, pl.blocks.data(), pl.blocks.size() * sizeof(VsaBlock),
                                 hipMemcpyHostToDevice, c->stream));
    }
    if (!pl.segblk.empty()) {
        VSA_CHECK(hipMemcpyAsync(d_segblk, pl.segblk.data(), pl.segblk.size() * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, c->stream));
    }
    return VSA_OK;
}

/* launch a planned batch whose tables are on the device */
int launch_planned(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data, const VsaBlock *d_blocks,
                   const uint32_t *d_segblk, uint32_t nb, uint64_t segs,
                   uint32_t grid, int end_bits, uint64_t bytes, uint32_t flags, uint64_t *n_out) {
    int r;
    if ((r = ensure_out(c, 1)) != VSA_OK) return r;
    if (segs == 0) {
        c->last_n = 0;
        c->pending = false;
        *n_out = 0;
        return VSA_OK;
    }
    c->launch.db = db;
    c->launch.d_data = d_data;
    c->launch.d_blocks = d_blocks;
    c->launch.d_segblk = d_segblk;
    c->launch.nb = nb;
    c->launch.segs = segs;
    c->launch.grid = grid;
    c->launch.end_bits = end_bits;
    c->launch.bytes = bytes;
    c->launch.flags = flags;
    if ((r = launch_scan(c, db, d_data, nb, segs)) != VSA_OK) return r;
    if (flags & VSA_SCAN_ASYNC) {
        c->pending = true;
        *n_out = 0;
        return VSA_OK;
    }
    return complete_scan(c, n_out);
}

int scan_blocks_impl(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data,
                     const uint64_t *offs, const uint64_t *lens, const uint64_t *starts,
                     uint32_t nb, uint32_t flags, uint64_t *n_out,
                     const uint64_t *hlens = nullptr, const uint64_t *rlos = nullptr) {
    if (!c || !db || !d_data || !offs || !lens || (!nb)) return VSA_E_INVALID;
    /* an asynchronous scan still in flight may be reading the block and
     * segment tables rewritten below: it is completed first (count, overflow
     * rescan, sort); its results are then superseded by this scan */
    if (int r0 = finish_pending(c)) return r0;
    BatchPlan &pl = c->plan;
    auto T0 = std::chrono::steady_clock::now();
    /* one load of the confirm-wave count (another context may raise it):
     * the plan's waves and scanning waves per workgroup must agree, or its
     * workgroup count would exceed the CUs */
    const uint64_t ns_plan = LIT_WAVES - db->nconf.load();
    const uint64_t waves = (uint64_t)c->num_cus * ns_plan;
    const uint64_t *in[5] = {offs, lens, starts, hlens, rlos};
    auto &M = c->memo;
    bool same = M.valid && M.d_data == d_data && M.nb == nb && M.waves == waves &&
                M.fb_key == fb_key_of(c, db);
    for (int k = 0; same && k < 5; k++)
        same = in[k] ? (M.in[k].size() == nb && !memcmp(M.in[k].data(), in[k], nb * 8))
                     : M.in[k].empty();
    int r;
    Workspace &w = c->ws;
    auto T1 = T0, T2 = T0;
    if (!same) {
        /* the block table is built straight into the pinned mirror (pageable
         * copies stage synchronously), the segment map after it; one copy of
         * both */
        M.valid = false;
        if ((r = ensure_tables(c, nb, 0)) != VSA_OK) return r;
        if ((r = build_plan(d_data, offs, lens, starts, hlens, rlos, nb, waves, pl,
                            w.h_blocks, ns_plan,
                            c->fb.set[fb_set_of(db)].known ? c->fb.set[fb_set_of(db)].wg
                                                           : nullptr)) != VSA_OK)
            return r;
        T1 = std::chrono::steady_clock::now();
        if ((r = ensure_tables(c, nb, pl.segblk.size(), true)) != VSA_OK) return r;
        memcpy(w.h_segblk, pl.segblk.data(), pl.segblk.size() * sizeof(uint32_t));
        const size_t tab_bytes =
            (size_t)((uint8_t *)(w.h_segblk + pl.segblk.size()) - (uint8_t *)w.h_blocks);
        T2 = std::chrono::steady_clock::now();
        VSA_CHECK(hipMemcpyAsync(w.d_blocks, w.h_blocks, tab_bytes, hipMemcpyHostToDevice,
                                 c->stream));
        M.d_data = d_data;
        M.nb = nb;
        M.waves = waves;
        M.fb_key = fb_key_of(c, db);
        for (int k = 0; k < 5; k++) {
            if (in[k]) M.in[k].assign(in[k], in[k] + nb);
            else M.in[k].clear();
        }
        M.valid = true;
    }
    int rr = launch_planned(c, db, d_data, c->ws.d_blocks, c->ws.d_segblk, nb, pl.nsegs,
                          pl.grid, pl.end_bits, pl.bytes, flags, n_out);
    auto T3 = std::chrono::steady_clock::now();
    /* diagnostic: host-side cost of a per-call plan (tools/exp_host.py) */
    static const bool timing = getenv("VSA_HOST_TIMING") != nullptr;
    if (timing)
        fprintf(stderr, "host: nb %u segs %llu build %.3f memcpy %.3f launch+wait %.3f ms (kernel %.3f)\n", nb, (unsigned long long)pl.nsegs,
                std::chrono::duration<double, std::milli>(T1 - T0).count(),
                std::chrono::duration<double, std::milli>(T2 - T1).count(),
                std::chrono::duration<double, std::milli>(T3 - T2).count(), c->last_kernel_ms);
    return rr;
}

/* Count + sort of the last launch; on an output overflow the buffers grow
 * to the reported count and the same launch runs again (twice at most: the
 * count of an identical launch does not change). */
int complete_scan(vsa_ctx *c, uint64_t *n_out) {
    for (int attempt = 0; attempt < 3; attempt++) {
        int r = finish_scan(c, c->launch.flags, c->launch.end_bits, n_out);
        if (r != VSA_E_OVERFLOW) return r;
        /* the rescan reads the launch's tables: gone if its plan was freed */
        if (!c->launch.d_blocks || !c->launch.d_segblk) return VSA_E_INVALID;
        if ((r = ensure_out(c, c->ws.h_counters[0])) != VSA_OK) return r;
        if ((r = launch_scan(c, c->launch.db, c->launch.d_data, c->launch.nb, c->launch.segs)) !=
            VSA_OK)
            return r;
    }
    return VSA_E_OVERFLOW;
}

/* ------------------------------------------------------------ registry */

thread_local vsa_ctx *t_ctx = nullptr;

vsa_ctx *default_ctx() {
    if (!t_ctx) {
        int dev = 0;
        const char *e = getenv("VSA_DEVICE");
        if (e) dev = atoi(e);
        if (vsa_ctx_create(dev, &t_ctx) != VSA_OK) t_ctx = nullptr;
    }
    return t_ctx;
}

/* Keyed by (pointer, size); a lookup of an unregistered blob also compares
 * the whole blob with the cached host copy, so a database freed and
 * re-allocated at the same address is never served from a stale device
 * copy (memcmp runs at memory speed, ~20 us for a 0.4 MB FDR blob).  A blob
 * registered with vsa_hwlm_register is immutable until its unregister (the
 * integration registers it where the database is loaded),
 * so its lookups skip the compare. */
std::mutex g_reg_mu;
std::map<const void *, size_t> g_registered; /* pointer -> size */

bool is_registered(const void *p, size_t size) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_registered.find(p);
    return it != g_registered.end() && it->second == size;
}

struct RegKey {
    const void *p;
    size_t size;
    bool operator<(const RegKey &o) const {
        if (p != o.p) return p < o.p;
        return size < o.size;
    }
};

thread_local std::map<RegKey, vsa_db *> t_registry;

size_t engine_size(const uint8_t *eng, int type) {
    if (type == HWLM_ENGINE_NOOD) return sizeof(noodTable);
    return ((const uint32_t *)eng)[1]; /* FDR.size / Teddy.size */
}

/* look up (or upload) the device copy of a blob given as HWLM or as a bare
 * engine (type = -1: HWLM header present) */
vsa_db *registry_get(const void *ptr, int bare_type) {
    vsa_ctx *c = default_ctx();
    if (!c) return nullptr;
    const uint8_t *p = (const uint8_t *)ptr;
    size_t size;
    int type;
    if (bare_type < 0) {
        type = p[0];
        size = VSA_ROUNDUP_CL(sizeof(HWLM)) + engine_size(p + VSA_ROUNDUP_CL(sizeof(HWLM)), type);
    } else {
        type = bare_type;
        size = engine_size(p, type);
    }
    RegKey k{ptr, size};
    auto it = t_registry.find(k);
    if (it != t_registry.end()) {
        vsa_db *old = it->second;
        const uint8_t *cached = old->hblob + (bare_type < 0 ? 0 : VSA_ROUNDUP_CL(sizeof(HWLM)));
        if (is_registered(ptr, size) || memcmp(cached, p, size) == 0) return old;
        vsa_db_free(old); /* erases the registry entry */
    }
    vsa_db *db = nullptr;
    int r;
    if (bare_type < 0) {
        r = vsa_db_load(c, ptr, size, &db);
    } else {
        /* wrap the bare engine in an HWLM header */
        size_t tot = VSA_ROUNDUP_CL(sizeof(HWLM)) + size;
        std::vector<uint8_t> tmp(tot + 64, 0);
        uint8_t *al = (uint8_t *)VSA_ROUNDUP_N((uintptr_t)tmp.data(), 64);
        al[0] = (uint8_t)type;
        memcpy(al + VSA_ROUNDUP_CL(sizeof(HWLM)), p, size);
        r = vsa_db_load(c, al, tot, &db);
    }
    if (r != VSA_OK) return nullptr;
    t_registry[k] = db;
    return db;
}

/* ----------------------------------------------------------- replay --- */

/* offsets inside struct hs_scratch (src/scratch.h:172-219), x86-64 */
struct ScratchLayoutProbe {
    struct RoseContext_ {
        uint8_t mpv_inactive;
        uint64_t groups, lit_offset_adjust, delayLastEndOffset, lastEndOffset,
            lastMatchOffset, lastCombMatchOffset, minMatchOffset,
            minNonMpvMatchOffset, next_mpv_offset;
        uint32_t filledDelayedSlots, curr_qi;
        const uint8_t *ll_buf;
        size_t ll_len;
        const uint8_t *ll_buf_nocase;
        size_t ll_len_nocase;
    };
    struct catchup_pq_ {
        void *qm;
        uint32_t qm_size;
    };
    struct core_info_ {
        void *userContext;
        void *userCallback;
        const void *rose;
        char *state, *exhaustionVector, *logicalVector, *combVector;
        const uint8_t *buf;
        size_t len;
        const uint8_t *hbuf;
        size_t hlen;
        uint64_t buf_offset;
        uint8_t status;
    };
    struct match_deduper_ {
        void *log[2];
        void *som_log[2];
        uint64_t *som_start_log[2];
        uint32_t dkey_count, log_size;
        uint64_t current_report_offset;
        uint8_t som_log_dirty;
    };
    uint32_t magic;
    uint8_t in_use;
    uint32_t queueCount, activeQueueArraySize, bStateSize, tStateSize, fullStateSize;
    RoseContext_ tctxt;
    char *bstate, *tstate, *fullState;
    void *queues, *aqa, **delay_slots, **al_log;
    uint64_t al_log_sum;
    catchup_pq_ catchup_pq;
    core_info_ core_info;
    match_deduper_ deduper;
    uint32_t anchored_literal_region_len, anchored_literal_fatbit_size;
    void *handled_roles;
    uint64_t *som_store, *som_attempted_store;
    void *som_set_now, *som_attempted_set;
    uint64_t som_set_now_offset;
    uint32_t som_store_count, som_fatbit_size, handledKeyFatbitSize, delay_fatbit_size,
        scratchSize;
    char *scratch_alloc;
    uint64_t *fdr_conf;
    uint8_t fdr_conf_offset;
};

std::atomic<long> g_core_buf_off{(long)(offsetof(ScratchLayoutProbe, core_info) +
                                        offsetof(ScratchLayoutProbe::core_info_, buf))};
std::atomic<long> g_core_hbuf_off{(long)(offsetof(ScratchLayoutProbe, core_info) +
                                         offsetof(ScratchLayoutProbe::core_info_, hbuf))};
std::atomic<long> g_core_hlen_off{(long)(offsetof(ScratchLayoutProbe, core_info) +
                                         offsetof(ScratchLayoutProbe::core_info_, hlen))};
std::atomic<long> g_fdr_conf_off{(long)offsetof(ScratchLayoutProbe, fdr_conf)};
std::atomic<long> g_fdr_conf_offset_off{(long)offsetof(ScratchLayoutProbe, fdr_conf_offset)};

hwlm_error_t replay_nood(const uint64_t *keys, const uint32_t *ids, uint64_t n,
                         HWLMCallback cb, hs_scratch *scratch) {
    for (uint64_t i = 0; i < n; i++) {
        if (cb(keys[i] >> VSA_KEY_END_SHIFT, ids[i], scratch) == HWLM_TERMINATE_MATCHING) {
            return HWLM_TERMINATED;
        }
    }
    return HWLM_SUCCESS;
}

/* the flood shortcut's reports (flood_runtime.h:191-319): per group of
 * S = 4 (idCount <= 2) or 2 ends, each end reports every flood id whose
 * groups meet the live control, the run stopping once control leaves
 * allGroups; no confirm, no NOREPEAT */
bool emit_flood(const vsa::FloodEvent &ev, HWLMCallback cb, hs_scratch *scratch,
                uint64_t &control) {
    const FDRFlood *fl = ev.fl;
    if (fl->idCount && (control & fl->allGroups)) {
        const uint32_t S = fl->idCount <= 2 ? 4 : 2;
        for (uint32_t t = 0; t < ev.size && (control & fl->allGroups); t += S)
            for (uint32_t k = 0; k < S; k++)
                for (uint32_t d = 0; d < fl->idCount; d++)
                    if (control & fl->groups[d])
                        control = cb((size_t)(ev.i + t + k), fl->ids[d], scratch);
    }
    return control != HWLM_TERMINATE_MATCHING;
}

/* The confirmed records of one call, in reference order, through the
 * callback with confWithBit's sequential state; `floods` (ascending) replace
 * the ends they skip. */
hwlm_error_t replay_lit(const vsa_db *db, const uint64_t *keys, uint64_t n,
                        HWLMCallback cb, hs_scratch *scratch, hwlm_group_t groups,
                        const std::vector<vsa::FloodEvent> *floods = nullptr,
                        bool scratch_is_real = true) {
    const uint8_t *eng = db->hblob + VSA_ROUNDUP_CL(sizeof(HWLM));
    const uint8_t *confBase = eng + ((const uint32_t *)eng)[4];
    const bool squash_ok = scratch && scratch_is_real && db->mode == VSA_MODE_FDR4;
    const long co = g_fdr_conf_off.load(), coo = g_fdr_conf_offset_off.load();
    const size_t nf = floods ? floods->size() : 0;
    size_t fe = 0;
    uint64_t skip_lo = 0, skip_hi = 0; /* ends a flood replaced */
    uint64_t control = groups;
    uint32_t last_match = ~0u;
    uint64_t i = 0;
    while (i < n || fe < nf) {
        const uint64_t end = i < n ? keys[i] >> VSA_KEY_END_SHIFT : ~0ULL;
        if (fe < nf && (*floods)[fe].i <= end) {
            const vsa::FloodEvent &ev = (*floods)[fe++];
            if (!emit_flood(ev, cb, scratch, control)) return HWLM_TERMINATED;
            skip_lo = ev.i;
            skip_hi = (uint64_t)ev.i + ev.size;
            continue;
        }
        uint64_t j = i;
        while (j < n && (keys[j] >> VSA_KEY_END_SHIFT) == end) j++;
        if (end >= skip_lo && end < skip_hi) {
            i = j;
            continue;
        }
        uint32_t squashed = 0;
        for (uint64_t k = i; k < j; k++) {
            const uint32_t b = (uint32_t)(keys[k] >> VSA_KEY_BUCKET_SHIFT) & 15;
            const uint32_t lidx = (uint32_t)(keys[k] & VSA_KEY_LI_MASK);
            if (squashed & (1u << b)) continue;
            const LitInfo *li =
                (const LitInfo *)(confBase + db->conf_off[b] + (size_t)lidx * 8);
            if (last_match == li->id && (li->flags & FDR_LIT_FLAG_NOREPEAT)) continue;
            if (!(li->groups & control)) continue;
            last_match = li->id;
            if (squash_ok && co >= 0) {
                /* live conf word: later buckets still pending at this end */
                uint64_t conf = 0;
                for (uint64_t m = k + 1; m < j; m++) {
                    uint32_t bb = (uint32_t)(keys[m] >> VSA_KEY_BUCKET_SHIFT) & 15;
                    if (bb > b) conf |= 1ull << bb;
                }
                const uint64_t before = conf;
                uint64_t **slot = (uint64_t **)((char *)scratch + co);
                *slot = &conf;
                *((uint8_t *)scratch + coo) = (uint8_t)b;
                control = cb(end, li->id, scratch);
                *slot = nullptr;
                squashed |= (uint32_t)(before & ~conf);
            } else {
                control = cb(end, li->id, scratch);
            }
            if (control == HWLM_TERMINATE_MATCHING) return HWLM_TERMINATED;
        }
        i = j;
    }
    return HWLM_SUCCESS;
}

/* flood events of one call when the blob's flood table is live */
const std::vector<vsa::FloodEvent> *floods_for(const vsa_db *db, const uint8_t *buf, size_t len,
                                               size_t start,
                                               std::vector<vsa::FloodEvent> &ev) {
    if (!db->flood_live || db->type != HWLM_ENGINE_FDR) return nullptr;
    vsa::flood_events(buf, len, start, db->hblob + VSA_ROUNDUP_CL(sizeof(HWLM)),
                      g_vector_size, ev);
    return ev.empty() ? nullptr : &ev;
}

/* the last drop-in scan's n records on the host, in reference order: from
 * the published copy (vsa_publish, <= PUB_RECS records) or the device */
int fetch_records(vsa_ctx *c, uint64_t n, std::vector<uint64_t> &keys,
                  std::vector<uint32_t> &ids) {
    keys.resize(n);
    ids.resize(n);
    if (!n) return VSA_OK;
    if (c->launch.published && (c->launch.flags & SCAN_HOST_SORT_SMALL) && c->host_sort &&
        n <= PUB_RECS) {
        const unsigned long long *h = c->ws.h_pub;
        memcpy(keys.data(), h + 17, n * 8);
        memcpy(ids.data(), (const uint32_t *)(h + 17 + PUB_RECS), n * 4);
    } else {
        VSA_CHECK(hipMemcpyAsync(keys.data(), c->ws.d_keys[c->cur], n * 8,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipMemcpyAsync(ids.data(), c->ws.d_ids[c->cur], n * 4,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipStreamSynchronize(c->stream));
    }
    if (c->host_sort && n > 1) {
        /* keys are unique (end, bucket, LitInfo) */
        std::vector<std::pair<uint64_t, uint32_t>> kv(n);
        for (uint64_t i = 0; i < n; i++) kv[i] = {keys[i], ids[i]};
        std::sort(kv.begin(), kv.end());
        for (uint64_t i = 0; i < n; i++) {
            keys[i] = kv[i].first;
            ids[i] = kv[i].second;
        }
    }
    return VSA_OK;
}

/* scan one host buffer with the default context */
/* One hwlmExec-equivalent scan of a host buffer.  hend != NULL: streaming
 * with history (the 16 bytes before hend are copied in front of buf, as
 * the reference reads them, fdr.c:380-560). */
int scan_host(vsa_db *db, const uint8_t *buf, size_t len, size_t start,
              std::vector<uint64_t> &keys, std::vector<uint32_t> &ids,
              const uint8_t *hend = nullptr, size_t hlen = 0) {
    vsa_ctx *c = db->ctx;
    int r;
    const size_t pre = hend ? 16 : 0;
    const bool resident = !pre && c->res_host == buf && c->res_len == len;
    if (!resident) c->res_host = nullptr;
    if ((r = ensure_in(c, pre + len + 16)) != VSA_OK) return r;
    if (!resident && pre + len <= PIN_STAGE_MAX) {
        /* history + block staged in pinned memory, one DMA */
        if ((r = ensure_hin(c, pre + len)) != VSA_OK) return r;
        if (pre) memcpy(c->ws.h_in, hend - 16, 16);
        if (len) memcpy(c->ws.h_in + pre, buf, len);
        VSA_CHECK(hipMemcpyAsync(c->ws.d_in, c->ws.h_in, pre + len, hipMemcpyHostToDevice,
                                 c->stream));
    } else {
        if (pre) {
            VSA_CHECK(hipMemcpyAsync(c->ws.d_in, hend - 16, 16, hipMemcpyHostToDevice,
                                     c->stream));
        }
        if (len && !resident) {
            VSA_CHECK(hipMemcpyAsync(c->ws.d_in + pre, buf, len, hipMemcpyHostToDevice,
                                     c->stream));
        }
    }
    uint64_t off = 0, l = len, st = start, n = 0, hl = hlen;
    if ((r = scan_blocks_impl(c, db, c->ws.d_in + pre, &off, &l, &st, 1, SCAN_HOST_SORT_SMALL,
                              &n, pre ? &hl : nullptr)) != VSA_OK)
        return r;
    return fetch_records(c, n, keys, ids);
}

/* class scan over a host buffer: returns first / last+1 */
int class_host(const uint8_t cls[32], const uint8_t *cls2, const uint8_t *buf, size_t len,
               uint64_t *first, uint64_t *last) {
    vsa_ctx *c = default_ctx();
    if (!c) return VSA_E_DEVICE;
    uint64_t cnt;
    if (c->res_host && buf >= c->res_host && buf + len <= c->res_host + c->res_len) {
        /* inside the buffer this drop-in call already uploaded (hwlmExec
         * reserved twice its size): scan it in place when 16-B aligned,
         * else from an aligned device-side copy behind it */
        const uint8_t *d = c->ws.d_in + (buf - c->res_host);
        if ((uintptr_t)d & 15) {
            uint8_t *cp = c->ws.d_in + ((c->res_len + 16 + 15) & ~(size_t)15);
            if (cp + len > c->ws.d_in + c->ws.in_cap) return VSA_E_INVALID;
            VSA_CHECK(hipMemcpyAsync(cp, d, len, hipMemcpyDeviceToDevice, c->stream));
            d = cp;
        }
        return vsa_class_scan(c, cls, cls2, d, len, nullptr, first, last, &cnt, 0);
    }
    c->res_host = nullptr;
    int r;
    if ((r = ensure_in(c, len + 16)) != VSA_OK) return r;
    if (len) {
        VSA_CHECK(hipMemcpyAsync(c->ws.d_in, buf, len, hipMemcpyHostToDevice, c->stream));
    }
    return vsa_class_scan(c, cls, cls2, c->ws.d_in, len, nullptr, first, last, &cnt, 0);
}

/* shuftiDoubleExec on the device (VsaPairParams); `vsize` = the reference
 * build's VECTORSIZE, the buffer's host address fixes the block alignment. */
int64_t pair_host(const uint8_t *lo1, const uint8_t *hi1, const uint8_t *lo2,
                  const uint8_t *hi2, const uint8_t *buf, size_t len, uint32_t vsize) {
    vsa_ctx *c = default_ctx();
    if (!c) return -2;
    if (!len) return 0;
    if (ensure_in(c, len + 16) != VSA_OK) return -2;
    Workspace &w = c->ws;
    if (hipMemcpyAsync(w.d_in, buf, len, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return -2;
    unsigned long long *first = w.d_counters + PAIR_BASE;
    if (hipMemsetAsync(first, 0xff, 48 * 8, c->stream) != hipSuccess) return -2;
    VsaPairParams P;
    memset(&P, 0, sizeof(P));
    P.data = w.d_in;
    P.len = len;
    for (int ch = 0; ch < 256; ch++) {
        P.n1[ch] = (uint8_t)~(lo1[ch & 15] | hi1[ch >> 4]);
        P.n2[ch] = (uint8_t)~(lo2[ch & 15] | hi2[ch >> 4]);
    }
    P.vsize = vsize;
    P.mis = (uint32_t)((uintptr_t)buf % vsize);
    P.first = first;
    uint64_t want = (len + 255) / 256;
    uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->num_cus * 4));
    drop_stale_error();
    hipLaunchKernelGGL(vsa_pair_scan, dim3(grid), dim3(256), 0, c->stream, P);
    if (hipGetLastError() != hipSuccess) return -2;
    if (hipMemcpyAsync(w.h_counters + PAIR_BASE, first, 48 * 8, hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess)
        return -2;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -2;
    const unsigned long long *h = w.h_counters + PAIR_BASE;
    if (h[0] != ~0ULL) return (int64_t)h[0];
    if (h[16] != ~0ULL) return (int64_t)h[16];
    if (h[32] != ~0ULL && h[32] < len) return (int64_t)h[32];
    return (int64_t)len;
}

void cls_from_shufti(const uint8_t *lo, const uint8_t *hi, uint8_t cls[32]) {
    memset(cls, 0, 32);
    for (int ch = 0; ch < 256; ch++) {
        if (lo[ch & 15] & hi[ch >> 4]) cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
    }
}

void cls_from_truffle(const uint8_t *m1, const uint8_t *m2, uint8_t cls[32]) {
    memset(cls, 0, 32);
    for (int ch = 0; ch < 256; ch++) {
        const uint8_t *m = (ch & 0x80) ? m2 : m1;
        if ((m[ch & 15] >> ((ch >> 4) & 7)) & 1) cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
    }
}

void cls_from_masked(uint8_t c, uint8_t m, bool negate, uint8_t cls[32]) {
    memset(cls, 0, 32);
    for (int ch = 0; ch < 256; ch++) {
        bool in = ((uint8_t)ch & m) == c;
        if (in != negate) cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
    }
}

bool cls_has(const uint8_t cls[32], uint8_t ch) { return (cls[ch >> 3] >> (ch & 7)) & 1; }

} // namespace

/* ================================================================ API == */

extern "C" {

const char *vsa_version(void) { return "vectorscan_amd 0.1 (gfx950)"; }

int vsa_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int vsa_ctx_create(int device, vsa_ctx_t **out) {
    if (!out) return VSA_E_INVALID;
    std::unique_ptr<vsa_ctx> c(new vsa_ctx());
    c->device = device;
    VSA_CHECK(hipSetDevice(device));
    int cus = 0;
    VSA_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    c->num_cus = cus > 0 ? cus : 256;
    VSA_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->stream_ref.reset((void *)c->stream, [](void *st) { (void)hipStreamDestroy((hipStream_t)st); });
    VSA_CHECK(hipEventCreate(&c->ev0));
    VSA_CHECK(hipEventCreate(&c->ev1));
    VSA_CHECK(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
    VSA_CHECK(hipMalloc(&c->ws.d_counters, N_COUNTERS * sizeof(unsigned long long)));
    VSA_CHECK(hipMalloc(&c->ws.d_bins, 2 * VSA_SORT_BINS * sizeof(uint32_t)));
    VSA_CHECK(hipHostMalloc((void **)&c->ws.h_counters, N_COUNTERS * sizeof(unsigned long long),
                            hipHostMallocDefault));
    VSA_CHECK(hipHostMalloc((void **)&c->ws.h_pub, PUB_WORDS * sizeof(unsigned long long),
                            hipHostMallocCoherent | hipHostMallocMapped));
    memset(c->ws.h_pub, 0, PUB_WORDS * sizeof(unsigned long long));
    VSA_CHECK(hipHostGetDevicePointer((void **)&c->ws.d_pub, c->ws.h_pub, 0));
    VSA_CHECK(hipHostMalloc((void **)&c->fb.h, 2048 * sizeof(unsigned long long),
                            hipHostMallocCoherent | hipHostMallocMapped));
    VSA_CHECK(hipHostGetDevicePointer((void **)&c->fb.d, c->fb.h, 0));
    VSA_CHECK(hipMalloc(&c->fb.d_rec, 2048 * sizeof(unsigned long long)));
    for (auto &F : c->fb.set)
        for (int b = 0; b < 1024; b++) {
            F.xcc[b] = (uint8_t)(b & 7);
            F.wg[b] = 1.0f;
        }
    *out = c.release();
    return VSA_OK;
}

int vsa_ctx_destroy(vsa_ctx_t *c) {
    if (!c) return VSA_E_INVALID;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    /* plans outliving the context keep only their own device tables */
    for (vsa_plan *p : c->plans) p->ctx = nullptr;
    Workspace &w = c->ws;
    for (int i = 0; i < 2; i++) {
        if (w.d_keys[i]) (void)hipFree(w.d_keys[i]);
        if (w.d_ids[i]) (void)hipFree(w.d_ids[i]);
    }
    if (w.d_tmp) (void)hipFree(w.d_tmp);
    if (w.d_in) (void)hipFree(w.d_in);
    if (w.d_counters) (void)hipFree(w.d_counters);
    if (w.d_bins) (void)hipFree(w.d_bins);
    if (w.d_bstage) (void)hipFree(w.d_bstage);
    if (w.h_counters) (void)hipHostFree(w.h_counters);
    if (w.h_pub) (void)hipHostFree(w.h_pub);
    if (c->fb.h) (void)hipHostFree(c->fb.h);
    if (c->fb.d_rec) (void)hipFree(c->fb.d_rec);
    if (w.h_in) (void)hipHostFree(w.h_in);
    if (w.d_blocks) (void)hipFree(w.d_blocks);
    if (w.h_blocks) (void)hipHostFree(w.h_blocks);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->ev_rec) (void)hipEventDestroy(c->ev_rec);
    if (t_ctx == c) t_ctx = nullptr;
    delete c; /* drops its hold on the stream */
    /* the statuses ignored above must not fail a later launch check */
    (void)hipGetLastError();
    return VSA_OK;
}

int vsa_ctx_create_shared(vsa_ctx_t *base, vsa_ctx_t **out) {
    if (!base || !out) return VSA_E_INVALID;
    vsa_ctx_t *c = nullptr;
    int rc = vsa_ctx_create(base->device, &c);
    if (rc != VSA_OK) return rc;
    (void)hipStreamSynchronize(c->stream);
    c->stream_ref = base->stream_ref; /* releases the stream it made */
    c->stream = base->stream;
    *out = c;
    return VSA_OK;
}

void *vsa_ctx_stream(vsa_ctx_t *c) { return c ? (void *)c->stream : nullptr; }

/* ------------------------------------------- derived FDR first stage -- */

/* The device first stage of an FDR engine, rebuilt at load time from the
 * engine's own confirm records (every LitInfo's v / msk, fdr_confirm.h:
 * 57-65), in the reference's bucket layout.  The reference's first stages
 * are filters whose only contract is "no false negatives": every literal
 * the confirm accepts is consistent at every window, so the set of
 * confirmed matches is exactly the reference's for any stride / domain of
 * the bytecode and any key function.  The 4-field table (VSA_MODE_FDR4):
 * bit (f * 8 + b) of T[key] is 0 when some literal of
 * bucket b is consistent with the three bytes ending f bytes before its end
 * (back offsets f + 2, f + 1, f; bytes before the literal are don't-cares,
 * msk 0), keyed by vsa_fdr4_key (kernels.h: 15 bits, 7 + 7 of the last
 * two and bit 0 of the first).  u32 entries, 4 fields.  On the cfg-4
 * set it passes half the candidate bits of the 8-field pair table (1.7e-4
 * against 3.3e-4 per byte, tools/sim_filter.py s1_tri177_f4) from the same
 * 128 KiB, and its even positions alone leave 4.0 % of ends live against
 * 6.9 % (the two-level sweep's level 1). */
static void derive_fdr4_table(const uint8_t *eng, const uint32_t conf_off[8], uint32_t bits,
                              std::vector<uint32_t> &T, int par = -1) {
    const uint32_t n = 1u << bits;
    T.assign(n, ~0u);
    uint32_t always = 0;
    const uint8_t *confBase = eng + ((const uint32_t *)eng)[4];
    auto proj = [](uint8_t m, uint8_t v, uint32_t keep) {
        /* the distinct (x & keep) over bytes x with (x & m) == v */
        std::vector<uint32_t> out;
        bool seen[256] = {false};
        for (uint32_t x = 0; x < 256; x++)
            if ((x & m) == v && !seen[x & keep]) {
                seen[x & keep] = true;
                out.push_back(x & keep);
            }
        return out;
    };
    for (uint32_t b = 0; b < 8; b++) {
        if (!conf_off[b]) continue;
        const uint8_t *fc = confBase + conf_off[b];
        const FDRConfirm *cf = (const FDRConfirm *)fc;
        const uint32_t *li = (const uint32_t *)(fc + sizeof(FDRConfirm));
        std::vector<uint32_t> offs;
        for (uint32_t h = 0; h < (1u << cf->nBits); h++) {
            uint32_t o = li[h];
            if (!o) continue;
            for (;;) {
                offs.push_back(o);
                const LitInfo *L = (const LitInfo *)(fc + o);
                if (!L->next) break;
                o += sizeof(LitInfo);
            }
        }
        std::sort(offs.begin(), offs.end());
        offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
        for (uint32_t o : offs) {
            const LitInfo *L = (const LitInfo *)(fc + o);
            /* split passes (par 0 / 1): only the literals whose last byte can
             * have bit 0 == par (every end byte with that bit 0 is a pass's) */
            if (par >= 0 && ((L->msk >> 56) & 1u) && (uint32_t)((L->v >> 56) & 1u) != (uint32_t)par)
                continue;
            auto mv = [&](uint32_t back, uint8_t *m, uint8_t *v) {
                /* the byte `back` before the end: byte 7 - back of the window */
                *m = (uint8_t)(L->msk >> (8 * (7 - back)));
                *v = (uint8_t)(L->v >> (8 * (7 - back))) & *m;
            };
            for (uint32_t f = 0; f < 4; f++) {
                const uint32_t bit = 1u << (f * 8 + b);
                uint8_t m0, v0, m1, v1, m2, v2;
                mv(f, &m0, &v0);
                mv(f + 1, &m1, &v1);
                mv(f + 2, &m2, &v2);
                const auto c0 = proj(m0, v0, 0x7f), c1 = proj(m1, v1, 0x7f);
                const auto c2 = proj(m2, v2, 1u);
                if (c0.size() * c1.size() * c2.size() >= n) {
                    always |= bit;
                    continue;
                }
                for (uint32_t x2 : c2)
                    for (uint32_t x1 : c1)
                        for (uint32_t x0 : c0) T[vsa_fdr4_key(x2, x1, x0)] &= ~bit;
            }
        }
    }
    if (always) {
        for (auto &t : T) t &= ~always;
    }
}

/* The candidate bits per byte a 4-field table (15-bit keys) passes on
 * text, estimated as if its lookups were independent and the bytes uniform
 * over 0x20..0x7e: sum over buckets of the product over fields of the live
 * fraction of the keys.  Against tools/sim_filter.py on the cfg-4 sets
 * (5k / 10k / 20k / 50k literals): 7.2e-5 / 7.3e-4 / 7.8e-3 / 0.142
 * estimated, 1.7e-4 / - / 9.1e-3 / 0.148 simulated.  It only chooses the
 * schedule (split_passes), never a result. */
static double fdr4_text_rate(const std::vector<uint32_t> &T) {
    uint32_t live[32] = {0}, n = 0;
    for (uint32_t b2 = 0; b2 < 2; b2++)
        for (uint32_t b0 = 0x20; b0 < 0x7f; b0++)
            for (uint32_t b1 = 0x20; b1 < 0x7f; b1++) {
                const uint32_t e = ~T[vsa_fdr4_key(b2, b1, b0)];
                n++;
                for (int k = 0; k < 32; k++) live[k] += (e >> k) & 1u;
            }
    double s = 0.0;
    for (int b = 0; b < 8; b++) {
        double p = 1.0;
        for (int f = 0; f < 4; f++) p *= (double)live[f * 8 + b] / n;
        s += p;
    }
    return s;
}

/* split passes past this estimated rate (VSA_SPLIT=0 / 1 forces off / on).
 * Measured, 4 GiB cfg-4 corpus, kernel ms one pass / split
 * (profiles/r04h_split.jsonl): 20k literals (est 7.8e-3) 1.82 / 2.29, 30k
 * (3.0e-2) 3.63 / 3.16, 50k (0.142) 11.4 / 5.44; confirm candidates 11.4M /
 * 2.3M, 57.8M / 10.9M, 375M / 76M.  The crossover lies near 1.5e-2. */
static bool split_passes(double est) {
    if (const char *e = getenv("VSA_SPLIT")) return atoi(e) != 0;
    return est > 0.015;
}

/* Teddy / Fat Teddy first stage, rebuilt at load like FDR's: bit (k * lb +
 * b) of W[c] is 0 when some literal of bucket b has byte c (under its
 * mask) k bytes before its end (LitInfo v / msk, fdr_confirm.h:57-65), for
 * k < nl.  Every literal the confirm accepts passes, so the confirmed set is
 * the reference's; the reference's nibble masks (teddy_compile.cpp:439-509,
 * teddy.c:921-971) pass every byte of a bucket's nibble product. */
static void derive_teddy_table(const uint8_t *eng, const uint32_t *conf_off, uint32_t nb,
                               uint32_t nl, uint32_t lb, std::vector<uint64_t> &W) {
    W.assign(256, ~0ULL);
    uint64_t always = 0;
    const uint8_t *confBase = eng + ((const uint32_t *)eng)[4];
    for (uint32_t b = 0; b < nb; b++) {
        if (!conf_off[b]) continue;
        const uint8_t *fc = confBase + conf_off[b];
        const FDRConfirm *cf = (const FDRConfirm *)fc;
        const uint32_t *li = (const uint32_t *)(fc + sizeof(FDRConfirm));
        std::vector<uint32_t> offs;
        for (uint32_t h = 0; h < (1u << cf->nBits); h++) {
            uint32_t o = li[h];
            if (!o) continue;
            for (;;) {
                offs.push_back(o);
                const LitInfo *L = (const LitInfo *)(fc + o);
                if (!L->next) break;
                o += sizeof(LitInfo);
            }
        }
        std::sort(offs.begin(), offs.end());
        offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
        for (uint32_t o : offs) {
            const LitInfo *L = (const LitInfo *)(fc + o);
            for (uint32_t k = 0; k < nl; k++) {
                const uint64_t bit = 1ULL << (k * lb + b);
                const uint8_t m = (uint8_t)(L->msk >> (8 * (7 - k)));
                const uint8_t v = (uint8_t)(L->v >> (8 * (7 - k))) & m;
                if (!m) {
                    always |= bit;
                    continue;
                }
                for (uint32_t ch = 0; ch < 256; ch++)
                    if ((ch & m) == v) W[ch] &= ~bit;
            }
        }
    }
    for (auto &w : W) w &= ~always;
}

int vsa_db_load(vsa_ctx_t *c, const void *hwlm, size_t size, vsa_db_t **out) {
    if (!c || !hwlm || !out || size < VSA_ROUNDUP_CL(sizeof(HWLM))) return VSA_E_INVALID;
    VSA_CHECK(hipSetDevice(c->device));
    std::unique_ptr<vsa_db> db(new vsa_db());
    db->ctx = c;
    db->host.resize(size + 64);
    db->hblob = (uint8_t *)VSA_ROUNDUP_N((uintptr_t)db->host.data(), 64);
    memcpy(db->hblob, hwlm, size);
    db->size = size;
    const HWLM *h = (const HWLM *)db->hblob;
    const uint8_t *eng = db->hblob + VSA_ROUNDUP_CL(sizeof(HWLM));
    db->type = h->type;
    if (db->type == HWLM_ENGINE_NOOD) {
        memcpy(&db->nood, eng, sizeof(noodTable));
        if (db->nood.msk_len < 1 || db->nood.msk_len > 8) return VSA_E_INVALID;
    } else if (db->type == HWLM_ENGINE_FDR) {
        db->engine_id = ((const uint32_t *)eng)[0];
        if (db->engine_id == VSA_ENGINE_FDR) {
            const FDR *f = (const FDR *)eng;
            if (f->domain < 9 || f->domain > 15) return VSA_E_INVALID;
            db->mode = VSA_MODE_FDR4;
            memcpy(&db->state_lo, f->start.b, 8);
            memcpy(&db->state_hi, f->start.b + 8, 8);
            db->nbuckets = 8;
        } else if (vsa_engine_is_teddy(db->engine_id)) {
            bool fat = vsa_engine_is_fat(db->engine_id);
            db->mode = fat ? VSA_MODE_FAT : VSA_MODE_TEDDY;
            db->nbuckets = fat ? 16 : 8;
            db->table_entries = 256;
            db->dmask = 0xff;
        } else {
            return VSA_E_INVALID;
        }
        const uint32_t *confBase = (const uint32_t *)(eng + ((const uint32_t *)eng)[4]);
        for (uint32_t b = 0; b < db->nbuckets; b++) db->conf_off[b] = confBase[b];
        {
            /* flood table (fdr_compile.cpp:204-211): 256 x u32 index, records */
            const uint8_t *fb = eng + ((const uint32_t *)eng)[5];
            const uint32_t *fidx = (const uint32_t *)fb;
            const FDRFlood *fr = (const FDRFlood *)(fb + 1024);
            for (int ch = 0; ch < 256 && !db->flood_live; ch++)
                db->flood_live = fr[fidx[ch]].idCount < FDR_FLOOD_MAX_IDS;
        }
        /* match keys carry a LitInfo's offset from its FDRConfirm in 8-byte
         * units in 20 bits (kernels.h): engines up to 8 MiB */
        if (engine_size(eng, HWLM_ENGINE_FDR) > ((size_t)8 << 20)) return VSA_E_INVALID;
        /* prefilter bitmaps: bit h of bucket b = (litIndex_b[h] != 0) */
        std::vector<uint32_t> slots;
        for (uint32_t b = 0; b < 16; b++) db->slot_off[b] = 0xffffffffu;
        db->pf_mult = 0;
        /* eligible buckets (one kernel-wide multiplier); when the exact
         * bitmaps exceed SLOT_WORDS_MAX the largest are coarsened: bit h >> k
         * of a 2^(nbits - k)-bit map = OR of the exact bits it covers (the
         * hash's top nbits - k bits), still a no-false-negative prefilter */
        uint32_t nb_full[16] = {0}, nb_use[16] = {0};
        for (uint32_t b = 0; b < db->nbuckets; b++) {
            if (!db->conf_off[b]) continue;
            const uint8_t *fc = (const uint8_t *)confBase + db->conf_off[b];
            const uint32_t nbits = *(const uint32_t *)(fc + 16);
            const uint64_t mult = *(const uint64_t *)(fc + 8);
            if (!db->pf_mult) db->pf_mult = mult;
            if (mult != db->pf_mult || nbits > 24 || nbits < 1) continue;
            nb_full[b] = nb_use[b] = nbits;
        }
        auto words_of = [](uint32_t bits) { return bits ? ((1u << bits) + 31) / 32 : 0u; };
        for (;;) {
            uint32_t tot = 0, big = 16;
            for (uint32_t b = 0; b < 16; b++) {
                tot += words_of(nb_use[b]);
                if (nb_use[b] > 5 && (big == 16 || nb_use[b] > nb_use[big])) big = b;
            }
            if (tot <= SLOT_WORDS_MAX || big == 16) break;
            nb_use[big]--;
        }
        for (uint32_t b = 0; b < db->nbuckets; b++) {
            if (!nb_use[b]) continue;
            const uint8_t *fc = (const uint8_t *)confBase + db->conf_off[b];
            const uint32_t n = 1u << nb_full[b], k = nb_full[b] - nb_use[b];
            const uint32_t words = words_of(nb_use[b]);
            if (slots.size() + words > SLOT_WORDS_MAX) continue;
            const uint32_t *li = (const uint32_t *)(fc + 32);
            db->slot_off[b] = (uint32_t)slots.size();
            db->slot_bits[b] = (uint8_t)nb_use[b];
            slots.resize(slots.size() + words, 0);
            for (uint32_t h = 0; h < n; h++) {
                const uint32_t c = h >> k;
                if (li[h]) slots[db->slot_off[b] + c / 32] |= 1u << (c % 32);
            }
        }
        db->slot_words = (uint32_t)slots.size();
        if (!slots.empty()) {
            VSA_CHECK(hipMalloc(&db->d_slots, slots.size() * 4));
            VSA_CHECK(hipMemcpy(db->d_slots, slots.data(), slots.size() * 4,
                                hipMemcpyHostToDevice));
        }
    } else {
        return VSA_E_INVALID;
    }
    VSA_CHECK(hipSetDevice(c->device));
    VSA_CHECK(hipMalloc(&db->d_blob, size));
    VSA_CHECK(hipMemcpy(db->d_blob, db->hblob, size, hipMemcpyHostToDevice));
    if (db->mode == VSA_MODE_FDR4) {
        /* the 4-field first stage (derive_fdr4_table, 15-bit keys): its 128
         * KiB always fit in LDS beside the rings and the slot bitmaps (<= 12
         * KiB, SLOT_WORDS_MAX) */
        const uint32_t bits = 15;
        std::vector<uint32_t> T;
        derive_fdr4_table(eng, db->conf_off, bits, T);
        db->table_entries = 1u << bits;
        db->dmask = (1u << bits) - 1;
        db->est_rate = fdr4_text_rate(T);
        db->split = split_passes(db->est_rate);
        if (db->split) {
            /* pass 0's table in d_table, pass 1's in d_table2 */
            std::vector<uint32_t> T1;
            derive_fdr4_table(eng, db->conf_off, bits, T, 0);
            derive_fdr4_table(eng, db->conf_off, bits, T1, 1);
            VSA_CHECK(hipMalloc(&db->d_table2, T1.size() * 4));
            VSA_CHECK(hipMemcpy(db->d_table2, T1.data(), T1.size() * 4, hipMemcpyHostToDevice));
        }
        VSA_CHECK(hipMalloc(&db->d_table, T.size() * 4));
        VSA_CHECK(hipMemcpy(db->d_table, T.data(), T.size() * 4, hipMemcpyHostToDevice));
    }
    if (db->mode == VSA_MODE_TEDDY || db->mode == VSA_MODE_FAT) {
        /* exact byte table from the confirm records (derive_teddy_table) */
        std::vector<uint64_t> W;
        if (db->mode == VSA_MODE_TEDDY) derive_teddy_table(eng, db->conf_off, 8, 8, 8, W);
        else derive_teddy_table(eng, db->conf_off, 16, 4, 16, W);
        VSA_CHECK(hipMalloc(&db->d_table, 256 * 8));
        VSA_CHECK(hipMemcpy(db->d_table, W.data(), 256 * 8, hipMemcpyHostToDevice));
    }
    *out = db.release();
    return VSA_OK;
}

int vsa_db_free(vsa_db_t *db) {
    if (!db) return VSA_E_INVALID;
    if (db->d_blob) (void)hipFree(db->d_blob);
    if (db->d_table) (void)hipFree(db->d_table);
    if (db->d_table2) (void)hipFree(db->d_table2);
    if (db->d_slots) (void)hipFree(db->d_slots);
    for (auto it = t_registry.begin(); it != t_registry.end(); ++it) {
        if (it->second == db) {
            t_registry.erase(it);
            break;
        }
    }
    delete db;
    return VSA_OK;
}

/* Host-only: the first stage vsa_db_load derives for a Teddy / Fat Teddy
 * blob (256 byte entries), for tests and tools (FDR engines:
 * vsa_derive_fdr4_table).  *key_bits = 8; *field_bits = buckets per field
 * (8 or 16).  Returns the number of entries written (<= cap), or a VSA_E_*
 * code. */
int vsa_derive_first_stage(const void *hwlm, size_t size, uint64_t *table, uint32_t cap,
                           uint32_t *key_bits, uint32_t *field_bits) {
    if (!hwlm || !table || size < VSA_ROUNDUP_CL(sizeof(HWLM))) return VSA_E_INVALID;
    const HWLM *h = (const HWLM *)hwlm;
    if (h->type != HWLM_ENGINE_FDR) return VSA_E_INVALID;
    const uint8_t *eng = (const uint8_t *)hwlm + VSA_ROUNDUP_CL(sizeof(HWLM));
    const uint32_t id = ((const uint32_t *)eng)[0];
    const uint32_t *confBase = (const uint32_t *)(eng + ((const uint32_t *)eng)[4]);
    uint32_t conf_off[16] = {0};
    std::vector<uint64_t> T;
    if (vsa_engine_is_teddy(id)) {
        const bool fat = vsa_engine_is_fat(id);
        for (int b = 0; b < (fat ? 16 : 8); b++) conf_off[b] = confBase[b];
        if (fat) derive_teddy_table(eng, conf_off, 16, 4, 16, T);
        else derive_teddy_table(eng, conf_off, 8, 8, 8, T);
        *key_bits = 8;
        *field_bits = fat ? 16 : 8;
    } else {
        return VSA_E_INVALID;
    }
    const uint32_t n = (uint32_t)std::min<size_t>(cap, T.size());
    memcpy(table, T.data(), n * sizeof(uint64_t));
    return (int)n;
}

/* Host-only: the 4-field first stage (derive_fdr4_table) of an FDR blob,
 * for tests and tools (bits must be 15: vsa_fdr4_key).  Returns the
 * entries written (<= cap) or a VSA_E_* code. */
int vsa_derive_fdr4_table(const void *hwlm, size_t size, uint32_t bits, uint32_t *table,
                          uint32_t cap) {
    if (!hwlm || !table || size < VSA_ROUNDUP_CL(sizeof(HWLM)) || bits != 15)
        return VSA_E_INVALID;
    const HWLM *h = (const HWLM *)hwlm;
    if (h->type != HWLM_ENGINE_FDR) return VSA_E_INVALID;
    const uint8_t *eng = (const uint8_t *)hwlm + VSA_ROUNDUP_CL(sizeof(HWLM));
    if (((const uint32_t *)eng)[0] != VSA_ENGINE_FDR) return VSA_E_INVALID;
    const uint32_t *confBase = (const uint32_t *)(eng + ((const uint32_t *)eng)[4]);
    uint32_t conf_off[8];
    for (int b = 0; b < 8; b++) conf_off[b] = confBase[b];
    std::vector<uint32_t> T;
    derive_fdr4_table(eng, conf_off, bits, T);
    const uint32_t n = (uint32_t)std::min<size_t>(cap, T.size());
    memcpy(table, T.data(), n * sizeof(uint32_t));
    return (int)n;
}

/* Host-only: the 15-bit 4-field table of one split pass (par 0 / 1: the
 * literals whose last byte can have bit 0 == par; -1: the one-pass table)
 * and, in *text_rate, fdr4_text_rate of it (the load's split_passes rule).
 * Returns the entries written (<= cap) or a VSA_E_* code. */
int vsa_derive_fdr4_pass(const void *hwlm, size_t size, int par, uint32_t *table, uint32_t cap,
                         double *text_rate) {
    if (!hwlm || size < VSA_ROUNDUP_CL(sizeof(HWLM)) || par < -1 || par > 1)
        return VSA_E_INVALID;
    const HWLM *h = (const HWLM *)hwlm;
    if (h->type != HWLM_ENGINE_FDR) return VSA_E_INVALID;
    const uint8_t *eng = (const uint8_t *)hwlm + VSA_ROUNDUP_CL(sizeof(HWLM));
    if (((const uint32_t *)eng)[0] != VSA_ENGINE_FDR) return VSA_E_INVALID;
    const uint32_t *confBase = (const uint32_t *)(eng + ((const uint32_t *)eng)[4]);
    uint32_t conf_off[8];
    for (int b = 0; b < 8; b++) conf_off[b] = confBase[b];
    std::vector<uint32_t> T;
    derive_fdr4_table(eng, conf_off, 15, T, par);
    if (text_rate) *text_rate = fdr4_text_rate(T);
    const uint32_t n = table ? (uint32_t)std::min<size_t>(cap, T.size()) : 0u;
    if (n) memcpy(table, T.data(), n * sizeof(uint32_t));
    return (int)n;
}

int vsa_db_split(const vsa_db_t *db) {
    if (!db) return VSA_E_INVALID;
    return db->split ? 1 : 0;
}

int vsa_db_engine(const vsa_db_t *db) {
    if (!db) return VSA_E_INVALID;
    return db->type == HWLM_ENGINE_NOOD ? HWLM_ENGINE_NOOD : (int)db->engine_id;
}

int vsa_malloc(vsa_ctx_t *c, size_t bytes, void **p) {
    if (!c || !p) return VSA_E_INVALID;
    VSA_CHECK(hipSetDevice(c->device));
    VSA_CHECK(hipMalloc(p, bytes ? bytes : 16));
    return VSA_OK;
}

int vsa_free(vsa_ctx_t *c, void *p) {
    (void)c;
    VSA_CHECK(hipFree(p));
    return VSA_OK;
}

int vsa_memcpy_h2d(vsa_ctx_t *c, void *dst, const void *src, size_t bytes) {
    VSA_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    VSA_CHECK(hipStreamSynchronize(c->stream));
    return VSA_OK;
}

int vsa_memcpy_d2h(vsa_ctx_t *c, void *dst, const void *src, size_t bytes) {
    VSA_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    VSA_CHECK(hipStreamSynchronize(c->stream));
    return VSA_OK;
}

int vsa_sync(vsa_ctx_t *c) {
    VSA_CHECK(hipStreamSynchronize(c->stream));
    return VSA_OK;
}

int vsa_scan_blocks(vsa_ctx_t *c, const vsa_db_t *db, const uint8_t *d_data,
                    const uint64_t *offsets, const uint64_t *lens, const uint64_t *starts,
                    uint32_t nblocks, uint32_t flags, uint64_t *n_matches) {
    uint64_t dummy;
    return scan_blocks_impl(c, db, d_data, offsets, lens, starts, nblocks, flags,
                            n_matches ? n_matches : &dummy);
}

int vsa_scan_wait(vsa_ctx_t *c, uint64_t *n_matches) {
    if (!c) return VSA_E_INVALID;
    if (!c->pending) {
        if (n_matches) *n_matches = c->last_n;
        return VSA_OK;
    }
    c->pending = false;
    uint64_t n = 0;
    int r = complete_scan(c, &n); /* overflow: grow and rescan synchronously */
    if (n_matches) *n_matches = n;
    return r;
}

int vsa_scan_results(vsa_ctx_t *c, const uint64_t **k, const uint32_t **ids) {
    if (!c) return VSA_E_INVALID;
    /* The pointers go to callers that read them on any stream (or the
     * host): the scan is completed and its whole queue (the binned sort
     * publishes the counters from its first workgroup, before the others
     * have written their bins) has finished before they are handed out. */
    if (int r = finish_pending(c)) return r;
    VSA_CHECK(hipStreamSynchronize(c->stream));
    if (k) *k = c->ws.d_keys[c->cur];
    if (ids) *ids = c->ws.d_ids[c->cur];
    return VSA_OK;
}

int vsa_scan_pack(vsa_ctx_t *c, void *d_dst, uint64_t cap) {
    if (!c || !d_dst) return VSA_E_INVALID;
    VSA_CHECK(hipSetDevice(c->device));
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((cap + 255) / 256, 256));
    if (c->pending && c->launch.published && c->launch.dev_sort) {
        /* the async binned scan's sorted records (buffer 1) and the counters
         * vsa_publish keeps on the device: queued behind it, no wait */
        drop_stale_error();
        hipLaunchKernelGGL(vsa_pack, dim3(grid), dim3(256), 0, c->stream,
                           (const unsigned long long *)c->ws.d_counters + 144,
                           (uint64_t)c->ws.out_cap, (const uint64_t *)c->ws.d_keys[1],
                           (const uint32_t *)c->ws.d_ids[1], cap, (uint64_t *)d_dst);
        VSA_CHECK(hipGetLastError());
        return VSA_OK;
    }
    /* otherwise the scan is completed on the host first (library sort,
     * overflow rescan) and its final records are packed */
    if (int r = finish_pending(c)) return r;
    unsigned long long *save = c->ws.d_counters + 144;
    unsigned long long hv[16] = {c->last_n, 0};
    VSA_CHECK(hipMemcpyAsync(save, hv, sizeof(hv), hipMemcpyHostToDevice, c->stream));
    drop_stale_error();
    hipLaunchKernelGGL(vsa_pack, dim3(grid), dim3(256), 0, c->stream,
                       (const unsigned long long *)save, (uint64_t)c->ws.out_cap,
                       (const uint64_t *)c->ws.d_keys[c->cur], (const uint32_t *)c->ws.d_ids[c->cur],
                       cap, (uint64_t *)d_dst);
    VSA_CHECK(hipGetLastError());
    VSA_CHECK(hipStreamSynchronize(c->stream)); /* hv is on the host stack */
    return VSA_OK;
}

int vsa_scan_copy(vsa_ctx_t *c, vsa_match_t *out, uint64_t cap, uint64_t *n_copied) {
    if (!c) return VSA_E_INVALID;
    uint64_t n = std::min(cap, c->last_n);
    if (n) {
        std::vector<uint64_t> k(n);
        std::vector<uint32_t> id(n);
        VSA_CHECK(hipMemcpyAsync(k.data(), c->ws.d_keys[c->cur], n * 8, hipMemcpyDeviceToHost,
                                 c->stream));
        VSA_CHECK(hipMemcpyAsync(id.data(), c->ws.d_ids[c->cur], n * 4, hipMemcpyDeviceToHost,
                                 c->stream));
        VSA_CHECK(hipStreamSynchronize(c->stream));
        for (uint64_t i = 0; i < n; i++) {
            out[i].key = k[i];
            out[i].id = id[i];
            out[i].pad = 0;
        }
    }
    if (n_copied) *n_copied = n;
    return VSA_OK;
}

int vsa_scan_copy_device(vsa_ctx_t *c, uint64_t *d_keys, uint32_t *d_ids, uint64_t cap,
                         uint64_t *n_copied) {
    if (!c) return VSA_E_INVALID;
    const uint64_t n = std::min(cap, c->last_n);
    if (n) {
        if (d_keys)
            VSA_CHECK(hipMemcpyAsync(d_keys, c->ws.d_keys[c->cur], n * 8,
                                     hipMemcpyDeviceToDevice, c->stream));
        if (d_ids)
            VSA_CHECK(hipMemcpyAsync(d_ids, c->ws.d_ids[c->cur], n * 4,
                                     hipMemcpyDeviceToDevice, c->stream));
    }
    if (n_copied) *n_copied = n;
    return VSA_OK;
}

uint64_t vsa_scan_candidates(vsa_ctx_t *c) { return c ? c->last_cand : 0; }

int vsa_scan_debug_counters(vsa_ctx_t *c, uint64_t out[16]) {
    if (!c || !out) return VSA_E_INVALID;
    /* the completed scan's counters as published to the host (the device
     * copies are zeroed for the next launch by the publish) */
    if (int r = finish_pending(c)) return r;
    VSA_CHECK(hipStreamSynchronize(c->stream));
    memcpy(out, c->ws.h_counters, 16 * sizeof(uint64_t));
    return VSA_OK;
}

double vsa_scan_kernel_ms(vsa_ctx_t *c) { return c ? c->last_kernel_ms : 0.0; }

uint64_t vsa_scan_launches(vsa_ctx_t *c) { return c ? c->lit_launches : 0; }

/* The box's streaming-read ceiling over a device buffer (bench.py's
 * roofline.peak_measured): vsa_read_probe reads the first len & ~64 KiB
 * bytes once per run on the ctx stream; best of `runs` (hipEvents) after
 * one untimed run.  Synchronous; not a scan, touches no scan state. */
int vsa_read_ceiling(vsa_ctx_t *c, const uint8_t *d_data, uint64_t len, uint32_t runs,
                     double *best_ms, uint64_t *bytes) {
    if (!c || !d_data || !best_ms || !runs) return VSA_E_INVALID;
    /* the probe reads 16-byte words (vsa_class_scan checks the same) */
    if ((uintptr_t)d_data & 15) return VSA_E_INVALID;
    const uint64_t n = len & ~((uint64_t)(64 << 10) - 1);
    if (!n) return VSA_E_INVALID;
    VSA_CHECK(hipSetDevice(c->device)); /* the sink goes on the context's device */
    uint32_t *sink = nullptr;
    VSA_CHECK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    hipError_t e = hipEventCreate(&e0);
    if (e == hipSuccess && (e = hipEventCreate(&e1)) != hipSuccess) (void)hipEventDestroy(e0);
    if (e != hipSuccess) {
        (void)hipFree(sink);
        VSA_CHECK(e);
    }
    float best = 1e30f;
    for (uint32_t r = 0; r <= runs && e == hipSuccess; r++) {
        e = hipEventRecord(e0, c->stream);
        if (e != hipSuccess) break;
        drop_stale_error();
        hipLaunchKernelGGL(vsa_read_probe, dim3(c->num_cus), dim3(1024), 0, c->stream, d_data, n,
                           sink);
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = hipEventRecord(e1, c->stream)) != hipSuccess) break;
        if ((e = hipEventSynchronize(e1)) != hipSuccess) break;
        float ms = 0.f;
        if ((e = hipEventElapsedTime(&ms, e0, e1)) != hipSuccess) break;
        if (r > 0 && ms < best) best = ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    VSA_CHECK(e);
    *best_ms = best;
    if (bytes) *bytes = n;
    return VSA_OK;
}

/* The shufti / truffle bytecode (masks, shufticompile.cpp:54 /
 * trufflecompile.cpp:60) over a device buffer: the class the masks accept,
 * as the drop-ins derive it (cls_from_shufti / cls_from_truffle), through
 * vsa_class_scan.  kind 0: shufti (a = lo, b = hi); 1: truffle (a = m1,
 * b = m2). */
int vsa_class_scan_masks(vsa_ctx_t *c, int kind, const uint8_t a[16], const uint8_t b[16],
                         const uint8_t *d_data, uint64_t len, uint64_t *d_bitmap,
                         uint64_t *first, uint64_t *last, uint64_t *count) {
    if (!a || !b || (kind != 0 && kind != 1)) return VSA_E_INVALID;
    uint8_t cls[32];
    if (kind == 0) cls_from_shufti(a, b, cls);
    else cls_from_truffle(a, b, cls);
    return vsa_class_scan(c, cls, nullptr, d_data, len, d_bitmap, first, last, count, 0);
}

int vsa_class_scan(vsa_ctx_t *c, const uint8_t cls[32], const uint8_t *cls2,
                   const uint8_t *d_data, uint64_t len, uint64_t *d_bitmap, uint64_t *first,
                   uint64_t *last, uint64_t *count, uint32_t flags) {
    (void)flags;
    if (!c || !cls) return VSA_E_INVALID;
    if (len == 0) {
        if (first) *first = 0;
        if (last) *last = 0;
        if (count) *count = 0;
        return VSA_OK;
    }
    if (!d_data || ((uintptr_t)d_data & 15)) return VSA_E_INVALID;
    Workspace &w = c->ws;
    unsigned long long *part = w.d_counters + CLASS_BASE;
    for (int i = 0; i < CLASS_SLOTS; i++) {
        w.h_counters[CLASS_BASE + 16 * i] = ~0ULL;
        w.h_counters[CLASS_BASE + 16 * i + 1] = 0;
        w.h_counters[CLASS_BASE + 16 * i + 2] = 0;
    }
    VSA_CHECK(hipMemcpyAsync(part, w.h_counters + CLASS_BASE, 16 * CLASS_SLOTS * 8,
                             hipMemcpyHostToDevice, c->stream));
    VsaClassParams P;
    memset(&P, 0, sizeof(P));
    P.data = d_data;
    P.len = len;
    memcpy(P.cls, cls, 32);
    if (cls2) {
        memcpy(P.cls2, cls2, 32);
        P.pair = 1;
    }
    P.bitmap = d_bitmap;
    P.first = part;
    P.last = part + 1;
    P.count = part + 2;
    P.slots = CLASS_SLOTS;
    const bool lut = !cls2 && len >= ((uint64_t)8 << 20);
    const uint64_t G = (uint64_t)c->num_cus;
    const uint64_t wspan = ((len + G - 1) / G + 4095) & ~(uint64_t)4095;
    const uint32_t lgrid = (uint32_t)((len + wspan - 1) / wspan);
    /* Schedule feedback (per-XCD weighted bounds) for the class scan measured
     * no gain at 256 MiB (0.0592 / 0.0597 / 0.0566 ms against 0.0593 /
     * 0.0587 / 0.0580, profiles/r04p_configs.jsonl, r04p_cfg2_nofb.jsonl)
     * and was removed in round 5: equal spans. */
    /* timing events on the dispatch packet (hipExtLaunchKernel), as the
     * literal scan's */
    if (lut) {
        /* large buffers: pair-LUT kernel, one 1024-thread workgroup per CU,
         * an equal 4 KiB-aligned share per workgroup, taken by its waves in
         * 4 KiB groups (kernels.hip vsa_class_scan_lut) */
        drop_stale_error();
        hipExtLaunchKernelGGL(vsa_class_scan_lut, dim3(lgrid), dim3(1024), 0u, c->stream, c->ev0,
                              c->ev1, 0u, P, wspan);
    } else {
        uint64_t chunks = (len + 15) / 16;
        uint64_t want = (chunks + 255) / 256;
        uint64_t cap = (uint64_t)c->num_cus * 8;
        uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min(want, cap));
        drop_stale_error();
        hipExtLaunchKernelGGL(vsa_class_scan, dim3(grid), dim3(256), 0u, c->stream, c->ev0, c->ev1,
                              0u, P);
    }
    VSA_CHECK(hipGetLastError());
    VSA_CHECK(hipMemcpyAsync(w.h_counters + CLASS_BASE, part, 16 * CLASS_SLOTS * 8,
                             hipMemcpyDeviceToHost, c->stream));
    VSA_CHECK(hipStreamSynchronize(c->stream));
    {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->last_kernel_ms = ms;
        /* a not-ready event status is not an error: it must not stay the
         * thread's last error for the next launch check */
        (void)hipGetLastError();
    }
    const unsigned long long *h = w.h_counters + CLASS_BASE;
    uint64_t f = ~0ULL, l = 0, n = 0;
    for (int i = 0; i < CLASS_SLOTS; i++) {
        f = std::min<uint64_t>(f, h[16 * i]);
        l = std::max<uint64_t>(l, h[16 * i + 1]);
        n += h[16 * i + 2];
    }
    if (first) *first = f == ~0ULL ? len : f;
    if (last) *last = l;
    if (count) *count = n;
    return VSA_OK;
}

/* run_hwlm_accel hwlm.c:48-80 (no minimum length, no offset) */
static const uint8_t *hwlm_accel(const union AccelAux *a, const uint8_t *p,
                                 const uint8_t *end) {
    const size_t len = (size_t)(end - p);
    int64_t r;
    switch (a->accel_type) {
    case ACCEL_VERM:
    case ACCEL_VERM_NOCASE:
        r = vsa_verm_find(0, a->verm.c, 0, 0, 0, a->accel_type == ACCEL_VERM_NOCASE, p, len);
        break;
    case ACCEL_DVERM:
    case ACCEL_DVERM_NOCASE:
        r = vsa_verm_find(4, a->dverm.c1, a->dverm.c2, 0, 0,
                          a->accel_type == ACCEL_DVERM_NOCASE, p, len);
        break;
    case ACCEL_SHUFTI:
        r = vsa_shufti_find(a->shufti.lo.b, a->shufti.hi.b, p, len, 0);
        break;
    case ACCEL_TRUFFLE:
        r = vsa_truffle_find(a->truffle.mask1.b, a->truffle.mask2.b, p, len, 0);
        break;
    default:
        return p;
    }
    return r < 0 ? p : p + r; /* device failure: no skip (the scan reports it) */
}

/* do_accel_block hwlm.c:85-105 */
static size_t hwlm_accel_block(const union AccelAux *aa, const uint8_t *buf, size_t len,
                               size_t start) {
    if (len - start < 16) return start;
    const uint8_t *ptr = hwlm_accel(aa, buf + start, buf + len);
    if (aa->generic.offset) {
        ptr -= aa->generic.offset;
        if (ptr < buf) ptr = buf;
    }
    return (size_t)(ptr - buf);
}

/* do_accel_streaming hwlm.c:114-175 */
static size_t hwlm_accel_stream(const union AccelAux *aux, const uint8_t *hbuf, size_t hlen,
                                const uint8_t *buf, size_t len, size_t start) {
    if (aux->accel_type == ACCEL_NONE || len - start < 16) return start;
    const uint8_t offset = aux->generic.offset;
    if (!start && hlen) {
        const uint8_t *ptr1 = hbuf, *end1 = hbuf + hlen;
        if (hlen >= 16) ptr1 = hwlm_accel(aux, ptr1, end1);
        const bool inaccurate =
            aux->accel_type == ACCEL_DVERM_NOCASE || aux->accel_type == ACCEL_DVERM;
        if ((hlen <= 16 || inaccurate) && end1 != ptr1 && end1 - ptr1 <= 16) {
            uint8_t temp[17];
            const ptrdiff_t tlen = end1 - ptr1;
            memcpy(temp, ptr1, (size_t)tlen);
            memset(temp + tlen, 0, 17 - (size_t)tlen);
            if (len) temp[tlen] = *buf;
            const uint8_t *tp = hwlm_accel(aux, temp, temp + 17);
            if (tp - temp >= tlen) ptr1 = end1;
        }
        if (ptr1 != end1) return start;
    }
    const uint8_t *ptr2 = buf + start;
    const uint8_t *found = hwlm_accel(aux, ptr2, buf + len);
    if (found >= ptr2 + offset) start += (size_t)(found - offset - ptr2);
    return start;
}

/* --------------------------------------------------- drop-in literal -- */

hwlm_error_t hwlmExec(const struct HWLM *tab, const uint8_t *buf, size_t len, size_t start,
                      HWLMCallback cb, struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!tab) return HWLM_ERROR_UNKNOWN;
    if (!groups) return HWLM_SUCCESS;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(tab, -1);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (db->type == HWLM_ENGINE_NOOD) {
        if (scan_host(db, buf, len, start, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
        return replay_nood(keys.data(), ids.data(), keys.size(), cb, scratch);
    }
    /* accel pre-skip (hwlm.c:85-105, 191-201) on the GPU, on the same
     * upload as the literal scan */
    const HWLM *h = (const HWLM *)db->hblob;
    const union AccelAux *aa = &h->accel0;
    if ((groups & ~h->accel1_groups) == 0) aa = &h->accel1;
    if (aa->accel_type != ACCEL_NONE && len - start >= 16) {
        vsa_ctx *c = db->ctx;
        if (ensure_in(c, 2 * len + 48) != VSA_OK ||
            hipMemcpyAsync(c->ws.d_in, buf, len, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            return HWLM_ERROR_UNKNOWN;
        c->res_host = buf;
        c->res_len = len;
        start = hwlm_accel_block(aa, buf, len, start);
    }
    if (start >= len) {
        db->ctx->res_host = nullptr;
        return HWLM_SUCCESS;
    }
    const int sr = scan_host(db, buf, len, start, keys, ids);
    db->ctx->res_host = nullptr;
    if (sr != VSA_OK) return HWLM_ERROR_UNKNOWN;
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(db, keys.data(), keys.size(), cb, scratch, groups,
                      floods_for(db, buf, len, start, ev));
}

hwlm_error_t fdrExec(const struct FDR *fdr, const uint8_t *buf, size_t len, size_t start,
                     HWLMCallback cb, struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!fdr) return HWLM_ERROR_UNKNOWN;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(fdr, HWLM_ENGINE_FDR);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, start, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(db, keys.data(), keys.size(), cb, scratch, groups,
                      floods_for(db, buf, len, start, ev));
}

hwlm_error_t noodExec(const struct noodTable *n, const uint8_t *buf, size_t len, size_t start,
                      HWLMCallback cb, struct hs_scratch *scratch) {
    if (!n) return HWLM_ERROR_UNKNOWN;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(n, HWLM_ENGINE_NOOD);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, start, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    return replay_nood(keys.data(), ids.data(), keys.size(), cb, scratch);
}

/* ------------------------------------------------ drop-in streaming -- */

/* fdrExecStreaming fdr.c:827-855.  len_history 0 scans as block mode (the
 * reference then applies fdr->start and never confirms into history). */
hwlm_error_t fdrExecStreaming(const struct FDR *fdr, const uint8_t *hbuf, size_t hlen,
                              const uint8_t *buf, size_t len, size_t start, HWLMCallback cb,
                              struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!fdr) return HWLM_ERROR_UNKNOWN;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(fdr, HWLM_ENGINE_FDR);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, start, keys, ids, hlen ? hbuf + hlen : nullptr, hlen) != VSA_OK)
        return HWLM_ERROR_UNKNOWN;
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(db, keys.data(), keys.size(), cb, scratch, groups,
                      floods_for(db, buf, len, start, ev));
}

/* noodExecStreaming noodle_engine.cpp:136-185 */
hwlm_error_t noodExecStreaming(const struct noodTable *n, const uint8_t *hbuf, size_t hlen,
                               const uint8_t *buf, size_t len, HWLMCallback cb,
                               struct hs_scratch *scratch) {
    if (!n) return HWLM_ERROR_UNKNOWN;
    if (len + hlen < n->msk_len || !len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(n, HWLM_ENGINE_NOOD);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, 0, keys, ids, hlen ? hbuf + hlen : nullptr, hlen) != VSA_OK)
        return HWLM_ERROR_UNKNOWN;
    return replay_nood(keys.data(), ids.data(), keys.size(), cb, scratch);
}

/* hwlmExecStreaming hwlm.c:207-247: buffers from scratch->core_info */
hwlm_error_t hwlmExecStreaming(const struct HWLM *tab, size_t len, size_t start,
                               HWLMCallback cb, struct hs_scratch *scratch,
                               hwlm_group_t groups) {
    if (!tab || !scratch) return HWLM_ERROR_UNKNOWN;
    if (!groups) return HWLM_SUCCESS;
    const char *sc = (const char *)scratch;
    const uint8_t *buf, *hbuf;
    size_t hlen;
    memcpy(&buf, sc + g_core_buf_off.load(), sizeof(buf));
    memcpy(&hbuf, sc + g_core_hbuf_off.load(), sizeof(hbuf));
    memcpy(&hlen, sc + g_core_hlen_off.load(), sizeof(hlen));
    const HWLM *h = (const HWLM *)tab;
    const uint8_t *eng = (const uint8_t *)tab + VSA_ROUNDUP_CL(sizeof(HWLM));
    if (h->type == HWLM_ENGINE_NOOD) {
        if (start) return noodExec((const noodTable *)eng, buf, len, start, cb, scratch);
        return noodExecStreaming((const noodTable *)eng, hbuf, hlen, buf, len, cb, scratch);
    }
    const union AccelAux *aa = &h->accel0;
    if ((groups & ~h->accel1_groups) == 0) aa = &h->accel1;
    start = hwlm_accel_stream(aa, hbuf, hlen, buf, len, start);
    return fdrExecStreaming((const FDR *)eng, hbuf, hlen, buf, len, start, cb, scratch, groups);
}

/* The same entry points under vsa_gpu_* names, for an integration that
 * keeps the reference's own definitions and routes each call by length
 * (the CPU below the measured break-even, the GPU
 * above it). */
hwlm_error_t vsa_gpu_hwlmExec(const struct HWLM *tab, const uint8_t *buf, size_t len,
                              size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                              hwlm_group_t groups) {
    return hwlmExec(tab, buf, len, start, cb, scratch, groups);
}
hwlm_error_t vsa_gpu_hwlmExecStreaming(const struct HWLM *tab, size_t len, size_t start,
                                       HWLMCallback cb, struct hs_scratch *scratch,
                                       hwlm_group_t groups) {
    return hwlmExecStreaming(tab, len, start, cb, scratch, groups);
}
hwlm_error_t vsa_gpu_fdrExec(const struct FDR *fdr, const uint8_t *buf, size_t len,
                             size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                             hwlm_group_t groups) {
    return fdrExec(fdr, buf, len, start, cb, scratch, groups);
}
hwlm_error_t vsa_gpu_noodExec(const struct noodTable *n, const uint8_t *buf, size_t len,
                              size_t start, HWLMCallback cb, struct hs_scratch *scratch) {
    return noodExec(n, buf, len, start, cb, scratch);
}

} // extern "C"

/* ------------------------------------------------- batching service --- */

/* Concurrent drop-in calls (many host threads scanning blocks, each through
 * its Rose floating table: rose/block.c:259, hsbench -T) share launches: a
 * worker thread with its own context takes the calls queued within a short
 * window, stages all their buffers into pinned memory, sends them in one
 * DMA, scans them as the blocks of ONE launch (vsa_scan_blocks, starts per
 * block) and hands each caller its records (rebased to its buffer); the
 * caller replays them through its own callback on its own thread, exactly as
 * hwlmExec does (groups, NOREPEAT, squash, flood events).  A call pays one
 * launch shared by the batch instead of one of its own.  The accel pre-skip
 * is not applied on this path (it only moves `start` past positions where no
 * literal can match). */
struct vsa_batcher {
    struct Req {
        const void *tab;
        const uint8_t *buf;
        size_t len, start;
        vsa_db *db = nullptr;
        std::vector<uint64_t> keys;
        std::vector<uint32_t> ids;
        int rc = VSA_OK;
        bool done = false;
    };
    int device = 0;
    uint32_t max_batch = 256;
    uint32_t window_us = 20;
    size_t max_bytes = 64u << 20;
    std::mutex m;
    std::condition_variable cv_req, cv_done;
    std::deque<Req *> q;
    bool stop = false;
    /* callers inside vsa_batcher_hwlmExec that still hold m or will re-lock
     * it (counted under m); destroy waits for zero before freeing m / cv */
    uint32_t inflight = 0;
    std::condition_variable cv_idle;
    std::thread worker;
    uint64_t batches = 0, calls = 0;

    void run() {
        vsa_ctx *c = nullptr;
        if (vsa_ctx_create(device, &c) != VSA_OK) c = nullptr;
        t_ctx = c; /* registry_get loads the tables on this context */
        std::vector<Req *> batch;
        std::vector<uint64_t> offs, lens, starts;
        std::vector<uint64_t> keys;
        std::vector<uint32_t> ids;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m);
                cv_req.wait(lk, [&] { return stop || !q.empty(); });
                if (stop && q.empty()) break;
                /* a short window for more callers to join the launch */
                if (q.size() < max_batch && window_us)
                    cv_req.wait_for(lk, std::chrono::microseconds(window_us),
                                    [&] { return stop || q.size() >= max_batch; });
                batch.clear();
                size_t bytes = 0;
                while (!q.empty() && batch.size() < max_batch &&
                       (batch.empty() || bytes + q.front()->len <= max_bytes)) {
                    bytes += q.front()->len;
                    batch.push_back(q.front());
                    q.pop_front();
                }
            }
            /* one launch per table in the batch */
            std::stable_sort(batch.begin(), batch.end(),
                             [](const Req *a, const Req *b) { return a->tab < b->tab; });
            for (size_t i = 0; i < batch.size();) {
                size_t j = i;
                while (j < batch.size() && batch[j]->tab == batch[i]->tab) j++;
                const int rc = c ? scan_group(c, batch.data() + i, j - i, offs, lens, starts,
                                              keys, ids)
                                 : VSA_E_DEVICE;
                for (size_t k = i; k < j; k++)
                    if (rc != VSA_OK) batch[k]->rc = rc;
                i = j;
            }
            {
                std::lock_guard<std::mutex> lk(m);
                for (Req *r : batch) r->done = true;
                batches++;
                calls += batch.size();
            }
            cv_done.notify_all();
        }
        if (c) {
            while (!t_registry.empty()) vsa_db_free(t_registry.begin()->second);
            vsa_ctx_destroy(c);
        }
        t_ctx = nullptr;
    }

    static int scan_group(vsa_ctx *c, Req **rq, size_t n, std::vector<uint64_t> &offs,
                          std::vector<uint64_t> &lens, std::vector<uint64_t> &starts,
                          std::vector<uint64_t> &keys, std::vector<uint32_t> &ids) {
        vsa_db *db = registry_get(rq[0]->tab, -1);
        if (!db) return VSA_E_INVALID;
        size_t total = 0;
        offs.resize(n);
        lens.resize(n);
        starts.resize(n);
        for (size_t k = 0; k < n; k++) {
            offs[k] = total;
            lens[k] = rq[k]->len;
            starts[k] = rq[k]->start;
            total += rq[k]->len;
        }
        int r;
        if ((r = ensure_in(c, total + 16)) != VSA_OK) return r;
        if ((r = ensure_hin(c, total)) != VSA_OK) return r;
        for (size_t k = 0; k < n; k++) memcpy(c->ws.h_in + offs[k], rq[k]->buf, rq[k]->len);
        c->res_host = nullptr;
        VSA_CHECK(hipMemcpyAsync(c->ws.d_in, c->ws.h_in, total, hipMemcpyHostToDevice, c->stream));
        uint64_t nm = 0;
        if ((r = scan_blocks_impl(c, db, c->ws.d_in, offs.data(), lens.data(), starts.data(),
                                  (uint32_t)n, 0, &nm)) != VSA_OK)
            return r;
        if ((r = fetch_records(c, nm, keys, ids)) != VSA_OK) return r;
        /* the records are in end order: each caller's are one run */
        uint64_t k0 = 0;
        for (size_t k = 0; k < n; k++) {
            const uint64_t hi = (offs[k] + lens[k]) << VSA_KEY_END_SHIFT;
            uint64_t k1 = k0;
            while (k1 < nm && keys[k1] < hi) k1++;
            Req *q = rq[k];
            q->db = db;
            q->keys.resize(k1 - k0);
            q->ids.assign(ids.begin() + (ptrdiff_t)k0, ids.begin() + (ptrdiff_t)k1);
            const uint64_t base = offs[k] << VSA_KEY_END_SHIFT;
            for (uint64_t i = k0; i < k1; i++) q->keys[i - k0] = keys[i] - base;
            k0 = k1;
        }
        return VSA_OK;
    }
};

extern "C" {

int vsa_batcher_create(int device, uint32_t max_batch, uint32_t window_us, vsa_batcher_t **out) {
    if (!out || !max_batch || max_batch > VSA_MAX_BLOCKS) return VSA_E_INVALID;
    vsa_batcher *b = new (std::nothrow) vsa_batcher;
    if (!b) return VSA_E_NOMEM;
    b->device = device;
    b->max_batch = max_batch;
    b->window_us = window_us;
    b->worker = std::thread([b] { b->run(); });
    *out = b;
    return VSA_OK;
}

int vsa_batcher_destroy(vsa_batcher_t *b) {
    if (!b) return VSA_E_INVALID;
    {
        std::lock_guard<std::mutex> lk(b->m);
        b->stop = true;
    }
    b->cv_req.notify_all();
    b->worker.join();
    {
        /* the worker finished every queued call before exiting; wait for
         * their callers to leave the mutex (a woken caller re-locks it) */
        std::unique_lock<std::mutex> lk(b->m);
        b->cv_idle.wait(lk, [&] { return b->inflight == 0; });
    }
    delete b;
    return VSA_OK;
}

int vsa_batcher_stats(vsa_batcher_t *b, uint64_t *batches, uint64_t *calls) {
    if (!b) return VSA_E_INVALID;
    std::lock_guard<std::mutex> lk(b->m);
    if (batches) *batches = b->batches;
    if (calls) *calls = b->calls;
    return VSA_OK;
}

hwlm_error_t vsa_batcher_hwlmExec(vsa_batcher_t *b, const struct HWLM *tab, const uint8_t *buf,
                                  size_t len, size_t start, HWLMCallback cb,
                                  struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!b || !tab) return HWLM_ERROR_UNKNOWN;
    if (!groups || start >= len) return HWLM_SUCCESS;
    /* a buffer that would fill a batch on its own goes alone */
    if (len > b->max_bytes / 4) return hwlmExec(tab, buf, len, start, cb, scratch, groups);
    vsa_batcher::Req r;
    r.tab = tab;
    r.buf = buf;
    r.len = len;
    r.start = start;
    {
        /* destroy may run concurrently: a call that finds it stopping is
         * refused; one already queued is served (the worker drains the
         * queue before it exits) and is counted until it has left m */
        std::unique_lock<std::mutex> lk(b->m);
        if (b->stop) return HWLM_ERROR_UNKNOWN;
        b->inflight++;
        b->q.push_back(&r);
        b->cv_req.notify_one();
        b->cv_done.wait(lk, [&] { return r.done; });
        if (--b->inflight == 0 && b->stop) b->cv_idle.notify_all();
    }
    if (r.rc != VSA_OK || !r.db) return HWLM_ERROR_UNKNOWN;
    if (r.db->type == HWLM_ENGINE_NOOD)
        return replay_nood(r.keys.data(), r.ids.data(), r.keys.size(), cb, scratch);
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(r.db, r.keys.data(), r.keys.size(), cb, scratch, groups,
                      floods_for(r.db, buf, len, start, ev));
}

} /* extern "C" */

/* The writes of one logical stream (hs_scan: one block-mode write;
 * hs_scan_vector: all pieces) scanned in ONE launch: the history bytes and
 * the writes laid end to end in the context's input buffer, each write a
 * block whose history is what precedes it (<= 16 bytes, enough for the
 * 8-byte HWLM literals); then each write's records replayed in order with
 * its own flood events and ends relative to it.  cbctx is an opaque
 * callback context (no Rose scratch: no INCLUDED_JUMP squash). */
namespace vsa {
/* the host copy of a loaded database's HWLM blob (vsa_internal.h) */
int ctxDevice(const struct vsa_ctx *c) { return c ? c->device : 0; }
int dbHostBlob(const struct vsa_db *db, const uint8_t **blob, size_t *size) {
    if (!db || !blob || !size) return VSA_E_INVALID;
    *blob = db->hblob;
    *size = db->size;
    return VSA_OK;
}
hwlm_error_t exec_pieces(vsa_ctx *c, const vsa_db *db, const u8 *hist, size_t hist_len,
                         const u8 *const *bufs, const size_t *lens, size_t n,
                         LitCallback cb, void *cbctx, void (*on_piece)(void *, size_t)) {
    if (!c || !db) return HWLM_ERROR_UNKNOWN;
    size_t total = 0;
    for (size_t i = 0; i < n; i++) total += lens[i];
    if (!total) return HWLM_SUCCESS;
    const size_t pre = 16, hl0 = std::min<size_t>(hist_len, 16);
    if (ensure_in(c, pre + total + 16) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    /* the history and every piece staged in pinned memory, one DMA (past
     * PIN_STAGE_MAX: a copy per piece) */
    const bool staged = pre + total <= PIN_STAGE_MAX && ensure_hin(c, pre + total) == VSA_OK;
    if (staged) {
        if (hl0) memcpy(c->ws.h_in + pre - hl0, hist + hist_len - hl0, hl0);
    } else if (hl0 && hipMemcpyAsync(c->ws.d_in + pre - hl0, hist + hist_len - hl0, hl0,
                                     hipMemcpyHostToDevice, c->stream) != hipSuccess) {
        return HWLM_ERROR_UNKNOWN;
    }
    std::vector<uint64_t> off, len, st, hl;
    std::vector<size_t> which;
    size_t pos = pre, seen = hist_len;
    for (size_t i = 0; i < n; i++) {
        if (!lens[i]) continue;
        if (staged) {
            memcpy(c->ws.h_in + pos, bufs[i], lens[i]);
        } else if (hipMemcpyAsync(c->ws.d_in + pos, bufs[i], lens[i], hipMemcpyHostToDevice,
                                  c->stream) != hipSuccess) {
            return HWLM_ERROR_UNKNOWN;
        }
        off.push_back(pos);
        len.push_back(lens[i]);
        st.push_back(0);
        hl.push_back(std::min<size_t>(seen, 16));
        which.push_back(i);
        pos += lens[i];
        seen += lens[i];
    }
    if (staged && hipMemcpyAsync(c->ws.d_in + pre - hl0, c->ws.h_in + pre - hl0,
                                 pos - (pre - hl0), hipMemcpyHostToDevice,
                                 c->stream) != hipSuccess)
        return HWLM_ERROR_UNKNOWN;
    uint64_t nm = 0;
    if (scan_blocks_impl(c, db, c->ws.d_in, off.data(), len.data(), st.data(),
                         (uint32_t)off.size(), SCAN_HOST_SORT_SMALL, &nm, hl.data()) != VSA_OK)
        return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (fetch_records(c, nm, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    hs_scratch *sc = (hs_scratch *)cbctx;
    std::vector<vsa::FloodEvent> ev;
    uint64_t k = 0;
    for (size_t b = 0; b < off.size(); b++) {
        const uint64_t hi = off[b] + len[b];
        uint64_t k2 = k;
        while (k2 < nm && (keys[k2] >> VSA_KEY_END_SHIFT) < hi) {
            keys[k2] -= off[b] << VSA_KEY_END_SHIFT; /* end relative to the write */
            k2++;
        }
        if (on_piece) on_piece(cbctx, which[b]);
        hwlm_error_t r;
        if (db->type == HWLM_ENGINE_NOOD) {
            r = replay_nood(keys.data() + k, ids.data() + k, k2 - k, cb, sc);
        } else {
            r = replay_lit(db, keys.data() + k, k2 - k, cb, sc, HWLM_ALL_GROUPS,
                           floods_for(db, bufs[which[b]], len[b], 0, ev), false);
        }
        if (r != HWLM_SUCCESS) return r;
        k = k2;
    }
    return HWLM_SUCCESS;
}
/* One launch over device-resident blocks (hlens NULL: block mode) and the
 * sorted records copied to the host (want_records) or only counted. */
int scan_records(vsa_ctx *c, const vsa_db *db, const u8 *d_data, const uint64_t *offsets,
                 const uint64_t *lens, const uint64_t *hlens, uint32_t nblocks,
                 std::vector<uint64_t> *keys, std::vector<uint32_t> *ids, uint64_t *n_out,
                 const vsa_plan *plan) {
    uint64_t nm = 0;
    int r;
    if (plan) {
        r = vsa_scan_plan(c, db, plan, 0, &nm);
    } else {
        std::vector<uint64_t> st(nblocks, 0);
        r = scan_blocks_impl(c, db, d_data, offsets, lens, st.data(), nblocks, 0, &nm, hlens);
    }
    if (r != VSA_OK) return r;
    *n_out = nm;
    if (!keys) return VSA_OK;
    keys->resize(nm);
    ids->resize(nm);
    if (nm) {
        VSA_CHECK(hipMemcpyAsync(keys->data(), c->ws.d_keys[c->cur], nm * 8,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipMemcpyAsync(ids->data(), c->ws.d_ids[c->cur], nm * 4,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipStreamSynchronize(c->stream));
    }
    return VSA_OK;
}

int records_fetch_async(vsa_ctx *c, uint64_t n, uint64_t *h_keys, uint32_t *h_ids) {
    if (!c->ev_rec) VSA_CHECK(hipEventCreateWithFlags(&c->ev_rec, hipEventDisableTiming));
    if (n) {
        VSA_CHECK(hipMemcpyAsync(h_keys, c->ws.d_keys[c->cur], n * 8, hipMemcpyDeviceToHost,
                                 c->stream));
        VSA_CHECK(hipMemcpyAsync(h_ids, c->ws.d_ids[c->cur], n * 4, hipMemcpyDeviceToHost,
                                 c->stream));
    }
    VSA_CHECK(hipEventRecord(c->ev_rec, c->stream));
    return VSA_OK;
}

int records_wait(vsa_ctx *c) {
    if (c->ev_rec) VSA_CHECK(hipEventSynchronize(c->ev_rec));
    return VSA_OK;
}

void *host_pinned_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault) != hipSuccess)
        return nullptr;
    return p;
}

void host_pinned_free(void *p) {
    if (p) (void)hipHostFree(p);
}

/* The records of one call (ends relative to that call's buffer) through
 * the callback, without flood emulation (no host buffer address) */
int replay_records(const vsa_db *db, const uint64_t *keys, const uint32_t *ids, uint64_t n,
                   LitCallback cb, void *cbctx) {
    hs_scratch *sc = (hs_scratch *)cbctx;
    if (db->type == HWLM_ENGINE_NOOD) return replay_nood(keys, ids, n, cb, sc);
    return replay_lit(db, keys, n, cb, sc, HWLM_ALL_GROUPS, nullptr, false);
}
} // namespace vsa

extern "C" {

int vsa_scan_blocks_ex(vsa_ctx_t *c, const vsa_db_t *db, const uint8_t *d_data,
                       const uint64_t *offsets, const uint64_t *lens, const uint64_t *starts,
                       const uint64_t *report_lo, uint32_t nblocks, uint32_t flags,
                       uint64_t *n_matches) {
    uint64_t dummy;
    return scan_blocks_impl(c, db, d_data, offsets, lens, starts, nblocks, flags,
                            n_matches ? n_matches : &dummy, nullptr, report_lo);
}

int vsa_scan_blocks_stream(vsa_ctx_t *c, const vsa_db_t *db, const uint8_t *d_data,
                           const uint64_t *offsets, const uint64_t *lens,
                           const uint64_t *starts, const uint64_t *hlens, uint32_t nblocks,
                           uint32_t flags, uint64_t *n_matches) {
    uint64_t dummy;
    return scan_blocks_impl(c, db, d_data, offsets, lens, starts, nblocks, flags,
                            n_matches ? n_matches : &dummy, hlens);
}


/* Host-only view of the schedule build_plan makes for a batch (no GPU
 * needed; tests/test_plan.py checks its invariants): the segment
 * descriptors (4 words each) and, for per-workgroup lists, the grid + 1
 * list bounds after them.  `words` receives up to cap words; returns the
 * word count (or a negative error), *nsegs / *grid the segment count and
 * the workgroups (0: region tickets).  waves / ns as a launch on num_cus
 * CUs with ns scanning waves each would use; d_data only sets the
 * alignment. */
int vsa_plan_describe(const uint8_t *d_data, const uint64_t *offsets, const uint64_t *lens,
                      const uint64_t *starts, const uint64_t *hlens, const uint64_t *report_lo,
                      uint32_t nblocks, uint32_t num_cus, uint32_t ns, uint32_t *words,
                      uint64_t cap, uint64_t *nsegs, uint32_t *grid, const float *wg_weights) {
    if (!offsets || !lens || !nblocks || !ns || !num_cus) return VSA_E_INVALID;
    BatchPlan pl;
    int r = build_plan(d_data, offsets, lens, starts, hlens, report_lo, nblocks,
                       (uint64_t)num_cus * ns, pl, nullptr, ns, wg_weights);
    if (r != VSA_OK) return r;
    if (words) memcpy(words, pl.segblk.data(), std::min<uint64_t>(cap, pl.segblk.size()) * 4);
    if (nsegs) *nsegs = pl.nsegs;
    if (grid) *grid = pl.grid;
    return (int)pl.segblk.size();
}

int vsa_plan_blocks(const uint8_t *d_data, const uint64_t *offsets, const uint64_t *lens,
                    const uint64_t *starts, const uint64_t *hlens, const uint64_t *report_lo,
                    uint32_t nblocks, void *out) {
    if (!offsets || !lens || !nblocks || !out) return VSA_E_INVALID;
    BatchPlan pl;
    int r = build_plan(d_data, offsets, lens, starts, hlens, report_lo, nblocks,
                       (uint64_t)256 * (LIT_WAVES - 1), pl);
    if (r != VSA_OK) return r;
    memcpy(out, pl.blocks.data(), (size_t)nblocks * sizeof(VsaBlock));
    return VSA_OK;
}

/* Host-only (tests): the schedule feedback's weight updates over `launches`
 * synthetic launches of `grid` workgroups (workgroup b on XCD b % 8) whose
 * XCDs stream at rate[x] (any unit; a workgroup's time = its share / its
 * XCD's rate, plus noise x jitter), each workgroup's share in proportion to
 * the applied weights.  Writes the applied weights to w_out[8]; returns how
 * many times they changed (plan rebuilds). */
int vsa_feedback_simulate(const double *rate, uint32_t grid, uint32_t launches, double jitter,
                          float *w_out) {
    if (!rate || !w_out || grid < 8 || grid > 1024) return VSA_E_INVALID;
    vsa_ctx::FbSet F;
    for (int b = 0; b < 1024; b++) {
        F.xcc[b] = (uint8_t)(b & 7);
        F.wg[b] = 1.0f;
    }
    std::vector<unsigned long long> h(2 * grid);
    uint64_t rs = 0x9e3779b97f4a7c15ULL;
    auto rnd = [&]() {
        rs ^= rs << 13;
        rs ^= rs >> 7;
        rs ^= rs << 17;
        return (double)(rs >> 11) / 9007199254740992.0 * 2.0 - 1.0;
    };
    uint32_t v0 = F.version;
    for (uint32_t l = 0; l < launches; l++) {
        double tw = 0;
        for (uint32_t b = 0; b < grid; b++) tw += F.wg[b];
        for (uint32_t b = 0; b < grid; b++) {
            const double share = F.wg[b] / tw;
            const double t = share / rate[b & 7] * (1.0 + jitter * rnd());
            h[grid + b] = 1000;
            h[b] = ((unsigned long long)(b & 7) << 60) | (1000 + (unsigned long long)(t * 1e9));
        }
        (void)feedback_update(F, h.data(), grid);
    }
    memcpy(w_out, F.wa, sizeof(F.wa));
    return (int)(F.version - v0);
}

int vsa_plan_create(vsa_ctx_t *c, const uint8_t *d_data, const uint64_t *offsets,
                    const uint64_t *lens, const uint64_t *starts, const uint64_t *hlens,
                    const uint64_t *report_lo, uint32_t nblocks, vsa_plan_t **out) {
    if (!c || !d_data || !offsets || !lens || !nblocks || !out) return VSA_E_INVALID;
    BatchPlan pl;
    int r = build_plan(d_data, offsets, lens, starts, hlens, report_lo, nblocks,
                       (uint64_t)c->num_cus * (LIT_WAVES - 1), pl);
    if (r != VSA_OK) return r;
    vsa_plan *p = new (std::nothrow) vsa_plan;
    if (!p) return VSA_E_NOMEM;
    p->ctx = c;
    c->plans.push_back(p);
    p->d_data = d_data;
    p->nb = nblocks;
    p->segs = pl.nsegs;
    p->grid = pl.grid;
    p->end_bits = pl.end_bits;
    p->bytes = pl.bytes;
    const uint64_t *ins[5] = {offsets, lens, starts, hlens, report_lo};
    for (int k = 0; k < 5; k++)
        if (ins[k]) p->in[k].assign(ins[k], ins[k] + nblocks);
    /* room for a rebuilt map: weighted shares can cut a few more pieces */
    p->segblk_cap = std::max<size_t>(1, pl.segblk.size() + pl.segblk.size() / 4 + 4 * 1024);
    p->flags.resize(nblocks);
    for (uint32_t i = 0; i < nblocks; i++) p->flags[i] = pl.blocks[i].flags;
    if (hipSetDevice(c->device) != hipSuccess ||
        hipMalloc(&p->d_blocks, nblocks * sizeof(VsaBlock)) != hipSuccess ||
        hipMalloc(&p->d_segblk, p->segblk_cap * sizeof(uint32_t)) != hipSuccess ||
        upload_plan(c, pl, p->d_blocks, p->d_segblk) != VSA_OK ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        vsa_plan_free(p);
        return VSA_E_DEVICE;
    }
    *out = p;
    return VSA_OK;
}

int vsa_plan_free(vsa_plan_t *p) {
    if (!p) return VSA_OK;
    int r = VSA_OK;
    if (vsa_ctx *c = p->ctx) {
        if (c->launch.d_blocks == p->d_blocks) {
            /* a scan of this plan still in flight is completed while its
             * tables exist (an overflow rescan reads them) */
            r = finish_pending(c);
            c->launch.d_blocks = nullptr;
            c->launch.d_segblk = nullptr;
        }
        (void)hipStreamSynchronize(c->stream);
        c->plans.erase(std::remove(c->plans.begin(), c->plans.end(), p), c->plans.end());
    }
    if (p->d_blocks) (void)hipFree(p->d_blocks);
    if (p->d_segblk) (void)hipFree(p->d_segblk);
    if (p->h_stage) (void)hipHostFree(p->h_stage);
    delete p;
    return r;
}

/* A prebuilt plan follows the context's schedule feedback: when the
 * weights for this kind of scan changed since the plan's segment map was
 * built, the map is rebuilt and uploaded before the launch (the context's
 * previous scan is complete, and only this context's scans read the plan;
 * the weights move by > 1 % steps, so this happens a few times while they
 * settle).  A map that would outgrow its buffer keeps the old one. */
int refresh_plan(vsa_ctx *c, const vsa_db *db, vsa_plan *p) {
    if (!xcd_feedback_on() || p->grid < 64 || p->in[0].empty()) return VSA_OK;
    const int si = fb_set_of(db);
    if (!c->fb.set[si].known) return VSA_OK;
    const uint64_t key = fb_key_of(c, db);
    if (key == p->fb_key) return VSA_OK;
    BatchPlan pl;
    auto in = [&](int k) { return p->in[k].empty() ? nullptr : p->in[k].data(); };
    int r = build_plan(p->d_data, in(0), in(1), in(2), in(3), in(4), p->nb,
                       (uint64_t)c->num_cus * (LIT_WAVES - 1), pl, nullptr, LIT_WAVES - 1,
                       c->fb.set[si].wg);
    if (r != VSA_OK) return r;
    if (pl.blocks.size() != p->nb) return VSA_E_INVALID;
    const size_t bb = (size_t)p->nb * sizeof(VsaBlock);
    if (pl.segblk.size() > p->segblk_cap) {
        /* weighted shares cut more pieces than the map had room for: grow
         * it (the context's previous scan, the only reader, is complete) */
        const size_t cap = pl.segblk.size() + pl.segblk.size() / 4;
        uint32_t *d = nullptr;
        VSA_CHECK(hipMalloc(&d, cap * sizeof(uint32_t)));
        VSA_CHECK(hipFree(p->d_segblk));
        p->d_segblk = d;
        p->segblk_cap = cap;
        if (p->h_stage) VSA_CHECK(hipHostFree(p->h_stage));
        p->h_stage = nullptr;
    }
    /* through a pinned staging buffer, queued on the scan stream: no host
     * wait.  The staging is rewritten only at this plan's next refresh, by
     * then this context's next scan -- queued behind these copies -- has
     * completed (finish_pending), so the copies have run */
    if (!p->h_stage)
        VSA_CHECK(hipHostMalloc(&p->h_stage, bb + p->segblk_cap * sizeof(uint32_t),
                                hipHostMallocDefault));
    uint8_t *hs = (uint8_t *)p->h_stage;
    bool blocks_same = p->flags.size() == p->nb;
    for (uint32_t i = 0; blocks_same && i < p->nb; i++)
        blocks_same = p->flags[i] == pl.blocks[i].flags;
    if (!blocks_same) {
        memcpy(hs, pl.blocks.data(), bb);
        VSA_CHECK(hipMemcpyAsync(p->d_blocks, hs, bb, hipMemcpyHostToDevice, c->stream));
        p->flags.resize(p->nb);
        for (uint32_t i = 0; i < p->nb; i++) p->flags[i] = pl.blocks[i].flags;
    }
    memcpy(hs + bb, pl.segblk.data(), pl.segblk.size() * sizeof(uint32_t));
    VSA_CHECK(hipMemcpyAsync(p->d_segblk, hs + bb, pl.segblk.size() * sizeof(uint32_t),
                             hipMemcpyHostToDevice, c->stream));
    p->segs = pl.nsegs;
    p->grid = pl.grid;
    /* the weights it follows now (only once applied: a failed rebuild is
     * tried again at the next scan) */
    p->fb_key = key;
    p->rebuilds++;
    return VSA_OK;
}

uint32_t vsa_plan_rebuilds(const vsa_plan_t *p) { return p ? p->rebuilds : 0u; }

int vsa_scan_plan(vsa_ctx_t *c, const vsa_db_t *db, const vsa_plan_t *p, uint32_t flags,
                  uint64_t *n_matches) {
    if (!c || !db || !p || p->ctx != c) return VSA_E_INVALID;
    if (int r0 = finish_pending(c)) return r0;
    if (int r1 = refresh_plan(c, db, const_cast<vsa_plan *>(p))) return r1;
    uint64_t dummy;
    return launch_planned(c, db, p->d_data, p->d_blocks, p->d_segblk, p->nb, p->segs,
                          p->grid, p->end_bits, p->bytes, flags,
                          n_matches ? n_matches : &dummy);
}

int vsa_scan_plan_pack(vsa_ctx_t *c, const vsa_db_t *db, const vsa_plan_t *p, void *d_dst,
                       uint64_t cap) {
    if (!c || !db || !p || !d_dst || p->ctx != c) return VSA_E_INVALID;
    if (int r0 = finish_pending(c)) return r0;
    if (int r1 = refresh_plan(c, db, const_cast<vsa_plan *>(p))) return r1;
    c->launch.pack_dst = d_dst;
    c->launch.pack_cap = cap;
    uint64_t n = 0;
    int r = launch_planned(c, db, p->d_data, p->d_blocks, p->d_segblk, p->nb, p->segs, p->grid,
                           p->end_bits, p->bytes, VSA_SCAN_ASYNC, &n);
    /* not consumed (no segments, or a launch without the binned sort): the
     * records are packed the separate way, after the host completes it */
    const bool fused = c->launch.pack_dst == nullptr && c->pending;
    c->launch.pack_dst = nullptr;
    if (r != VSA_OK) return r;
    return fused ? VSA_OK : vsa_scan_pack(c, d_dst, cap);
}

void vsa_get_scratch_core_info(long *buf_off, long *hbuf_off, long *hlen_off) {
    *buf_off = g_core_buf_off.load();
    *hbuf_off = g_core_hbuf_off.load();
    *hlen_off = g_core_hlen_off.load();
}

void vsa_set_scratch_core_info(long buf_off, long hbuf_off, long hlen_off) {
    g_core_buf_off.store(buf_off);
    g_core_hbuf_off.store(hbuf_off);
    g_core_hlen_off.store(hlen_off);
}

/* ----------------------------------------------------- drop-in accel -- */

int64_t vsa_shufti_find(const uint8_t lo[16], const uint8_t hi[16], const uint8_t *buf,
                        size_t len, int reverse) {
    uint8_t cls[32];
    cls_from_shufti(lo, hi, cls);
    uint64_t f = len, l = 0;
    if (class_host(cls, nullptr, buf, len, &f, &l) != VSA_OK) return -2;
    return reverse ? (int64_t)l - 1 : (int64_t)f;
}

int64_t vsa_truffle_find(const uint8_t m1[16], const uint8_t m2[16], const uint8_t *buf,
                         size_t len, int reverse) {
    uint8_t cls[32];
    cls_from_truffle(m1, m2, cls);
    uint64_t f = len, l = 0;
    if (class_host(cls, nullptr, buf, len, &f, &l) != VSA_OK) return -2;
    return reverse ? (int64_t)l - 1 : (int64_t)f;
}

int64_t vsa_verm_find(int mode, uint8_t c1, uint8_t c2, uint8_t m1, uint8_t m2, int nocase,
                      const uint8_t *buf, size_t len) {
    uint8_t cls[32], cls2[32];
    uint8_t cm = nocase ? 0xdf : 0xff;
    uint64_t f = len, l = 0;
    switch (mode) {
    case 0: /* vermicelliExec */
    case 2: /* rvermicelliExec */
        cls_from_masked(c1, cm, false, cls);
        break;
    case 1: /* nvermicelliExec */
    case 3: /* rnvermicelliExec */
        cls_from_masked(c1, cm, true, cls);
        break;
    case 4: /* vermicelliDoubleExec */
        cls_from_masked(c1, cm, false, cls);
        cls_from_masked(c2, cm, false, cls2);
        break;
    case 5: /* vermicelliDoubleMaskedExec */
        cls_from_masked(c1, m1, false, cls);
        cls_from_masked(c2, m2, false, cls2);
        break;
    case 6: /* rvermicelliDoubleExec */
        cls_from_masked(c1, cm, false, cls);
        cls_from_masked(c2, cm, false, cls2);
        break;
    default:
        return -2;
    }
    bool pair = mode >= 4;
    if (class_host(cls, pair ? cls2 : nullptr, buf, len, &f, &l) != VSA_OK) return -2;
    if (mode == 2 || mode == 3) return (int64_t)l - 1;
    if (mode == 6) {
        /* vermicelli_simd.cpp:360-423: position of c2 in the last pair (the
         * pair bitmap marks c1's position, so that is `last`); a c2 at
         * buf[0] is a partial pair; else buf - 1 */
        if (l) return (int64_t)l;
        if (len && cls_has(cls2, buf[0])) return 0;
        return -1;
    }
    if (pair && f == len && len && cls_has(cls, buf[len - 1])) {
        /* partial match at the end (vermicelli_simd.cpp:349-355) */
        return (int64_t)len - 1;
    }
    return (int64_t)f;
}

static void m128_bytes(vsa_m128_t m, uint8_t out[16]) { memcpy(out, &m, 16); }

/* The pointer-returning drop-ins have no error channel in the reference
 * ABI.  A device failure (the vsa_*_find helpers return -2) is recorded for
 * vsa_last_error() and answered with the no-skip pointer: buf for forward
 * scans, buf_end - 1 for reverse ones (every accel caller, hwlm.c:48-105 and
 * accel.c:35-180, then scans from there), never buf + (-2). */
static thread_local int t_last_error = VSA_OK;

static void note_error(const char *who) {
    t_last_error = VSA_E_DEVICE;
    if (getenv("VSA_DEBUG")) fprintf(stderr, "vsa: %s: device failure\n", who);
}

static const uint8_t *fwd_result(int64_t r, const uint8_t *buf, const uint8_t *buf_end,
                                 const char *who) {
    if (r == -2) {
        note_error(who);
        return buf;
    }
    return r < 0 ? buf_end : buf + r;
}

static const uint8_t *rev_result(int64_t r, const uint8_t *buf, const uint8_t *buf_end,
                                 const char *who) {
    if (r == -2) {
        note_error(who);
        return buf_end - 1;
    }
    return buf + r; /* -1: buf - 1, "not found" */
}

int vsa_last_error(void) {
    const int e = t_last_error;
    t_last_error = VSA_OK;
    return e;
}

const uint8_t *shuftiExec(vsa_m128_t mask_lo, vsa_m128_t mask_hi, const uint8_t *buf,
                          const uint8_t *buf_end) {
    uint8_t lo[16], hi[16];
    m128_bytes(mask_lo, lo);
    m128_bytes(mask_hi, hi);
    return fwd_result(vsa_shufti_find(lo, hi, buf, (size_t)(buf_end - buf), 0), buf, buf_end,
                      "shuftiExec");
}

void vsa_set_wave_log(void *d_log) { g_wave_log = (unsigned long long *)d_log; }

void vsa_set_accel_vector_size(uint32_t vsize) {
    if (vsize == 16 || vsize == 32 || vsize == 64) g_vector_size = vsize;
}

int64_t vsa_shufti_double_find(const uint8_t lo1[16], const uint8_t hi1[16],
                               const uint8_t lo2[16], const uint8_t hi2[16],
                               const uint8_t *buf, size_t len) {
    return pair_host(lo1, hi1, lo2, hi2, buf, len, g_vector_size);
}

const uint8_t *shuftiDoubleExec(vsa_m128_t mask1_lo, vsa_m128_t mask1_hi, vsa_m128_t mask2_lo,
                                vsa_m128_t mask2_hi, const uint8_t *buf,
                                const uint8_t *buf_end) {
    uint8_t lo1[16], hi1[16], lo2[16], hi2[16];
    m128_bytes(mask1_lo, lo1);
    m128_bytes(mask1_hi, hi1);
    m128_bytes(mask2_lo, lo2);
    m128_bytes(mask2_hi, hi2);
    return fwd_result(vsa_shufti_double_find(lo1, hi1, lo2, hi2, buf, (size_t)(buf_end - buf)),
                      buf, buf_end, "shuftiDoubleExec");
}

int vsa_shufti_build_double_masks(const uint8_t onechar[32], const uint8_t *pairs,
                                  size_t npairs, uint8_t lo1[16], uint8_t hi1[16],
                                  uint8_t lo2[16], uint8_t hi2[16]) {
    return vsa::shuftiDoubleMasks(onechar, pairs, npairs, lo1, hi1, lo2, hi2) ? 0 : -1;
}

const uint8_t *rshuftiExec(vsa_m128_t mask_lo, vsa_m128_t mask_hi, const uint8_t *buf,
                           const uint8_t *buf_end) {
    uint8_t lo[16], hi[16];
    m128_bytes(mask_lo, lo);
    m128_bytes(mask_hi, hi);
    return rev_result(vsa_shufti_find(lo, hi, buf, (size_t)(buf_end - buf), 1), buf, buf_end,
                      "rshuftiExec");
}

const uint8_t *truffleExec(vsa_m128_t mask1, vsa_m128_t mask2, const uint8_t *buf,
                           const uint8_t *buf_end) {
    uint8_t a[16], b[16];
    m128_bytes(mask1, a);
    m128_bytes(mask2, b);
    return fwd_result(vsa_truffle_find(a, b, buf, (size_t)(buf_end - buf), 0), buf, buf_end,
                      "truffleExec");
}

const uint8_t *rtruffleExec(vsa_m128_t mask1, vsa_m128_t mask2, const uint8_t *buf,
                            const uint8_t *buf_end) {
    uint8_t a[16], b[16];
    m128_bytes(mask1, a);
    m128_bytes(mask2, b);
    return rev_result(vsa_truffle_find(a, b, buf, (size_t)(buf_end - buf), 1), buf, buf_end,
                      "rtruffleExec");
}

static const uint8_t *verm_fwd(int mode, char c1, char c2, char m1, char m2, char nocase,
                               const uint8_t *buf, const uint8_t *buf_end, const char *who) {
    return fwd_result(vsa_verm_find(mode, (uint8_t)c1, (uint8_t)c2, (uint8_t)m1, (uint8_t)m2,
                                    nocase, buf, (size_t)(buf_end - buf)),
                      buf, buf_end, who);
}

static const uint8_t *verm_rev(int mode, char c1, char c2, char nocase, const uint8_t *buf,
                               const uint8_t *buf_end, const char *who) {
    return rev_result(vsa_verm_find(mode, (uint8_t)c1, (uint8_t)c2, 0, 0, nocase, buf,
                                    (size_t)(buf_end - buf)),
                      buf, buf_end, who);
}

const uint8_t *vermicelliExec(char c, char nocase, const uint8_t *buf, const uint8_t *buf_end) {
    return verm_fwd(0, c, 0, 0, 0, nocase, buf, buf_end, "vermicelliExec");
}
const uint8_t *nvermicelliExec(char c, char nocase, const uint8_t *buf, const uint8_t *buf_end) {
    return verm_fwd(1, c, 0, 0, 0, nocase, buf, buf_end, "nvermicelliExec");
}
const uint8_t *rvermicelliExec(char c, char nocase, const uint8_t *buf, const uint8_t *buf_end) {
    return verm_rev(2, c, 0, nocase, buf, buf_end, "rvermicelliExec");
}
const uint8_t *rnvermicelliExec(char c, char nocase, const uint8_t *buf,
                                const uint8_t *buf_end) {
    return verm_rev(3, c, 0, nocase, buf, buf_end, "rnvermicelliExec");
}
const uint8_t *vermicelliDoubleExec(char c1, char c2, char nocase, const uint8_t *buf,
                                    const uint8_t *buf_end) {
    return verm_fwd(4, c1, c2, 0, 0, nocase, buf, buf_end, "vermicelliDoubleExec");
}
const uint8_t *rvermicelliDoubleExec(char c1, char c2, char nocase, const uint8_t *buf,
                                     const uint8_t *buf_end) {
    return verm_rev(6, c1, c2, nocase, buf, buf_end, "rvermicelliDoubleExec");
}

const uint8_t *vermicelliDoubleMaskedExec(char c1, char c2, char m1, char m2,
                                          const uint8_t *buf, const uint8_t *buf_end) {
    return verm_fwd(5, c1, c2, m1, m2, 0, buf, buf_end, "vermicelliDoubleMaskedExec");
}

/* accel.c:35-180 dispatch for the forward schemes HWLM and NFAs use */
/* accel.c:36-183: minimum lengths (16, 17 for the double forms, which stop
 * one byte early), then rv = MAX(c + offset, rv) - offset. */
const uint8_t *run_accel(const union AccelAux *accel, const uint8_t *c, const uint8_t *c_end) {
    const size_t len = (size_t)(c_end - c);
    int64_t r;
    switch (accel->accel_type) {
    case ACCEL_NONE:
        return c;
    case ACCEL_VERM:
    case ACCEL_VERM_NOCASE:
        if (c + 15 >= c_end) return c;
        r = vsa_verm_find(0, accel->verm.c, 0, 0, 0, accel->accel_type == ACCEL_VERM_NOCASE, c,
                          len);
        break;
    case ACCEL_DVERM:
    case ACCEL_DVERM_NOCASE:
        if (c + 16 + 1 >= c_end) return c;
        r = vsa_verm_find(4, accel->dverm.c1, accel->dverm.c2, 0, 0,
                          accel->accel_type == ACCEL_DVERM_NOCASE, c, len - 1);
        break;
    case ACCEL_DVERM_MASKED:
        if (c + 16 + 1 >= c_end) return c;
        r = vsa_verm_find(5, accel->dverm.c1, accel->dverm.c2, accel->dverm.m1, accel->dverm.m2,
                          0, c, len - 1);
        break;
    case ACCEL_SHUFTI:
        if (c + 15 >= c_end) return c;
        r = vsa_shufti_find(accel->shufti.lo.b, accel->shufti.hi.b, c, len, 0);
        break;
    case ACCEL_TRUFFLE:
        if (c + 15 >= c_end) return c;
        r = vsa_truffle_find(accel->truffle.mask1.b, accel->truffle.mask2.b, c, len, 0);
        break;
    case ACCEL_DSHUFTI:
        if (c + 15 + 1 >= c_end) return c;
        r = vsa_shufti_double_find(accel->dshufti.lo1.b, accel->dshufti.hi1.b,
                                   accel->dshufti.lo2.b, accel->dshufti.hi2.b, c, len - 1);
        break;
    case ACCEL_RED_TAPE:
        r = (int64_t)len;
        break;
    default:
        return c;
    }
    if (r < 0) { /* device failure: no acceleration (see fwd_result) */
        note_error("run_accel");
        return c;
    }
    const uint8_t *rv = c + r;
    rv = std::max(c + accel->generic.offset, rv);
    return rv - accel->generic.offset;
}

int vsa_hwlm_register(const void *blob, int bare_type) {
    if (!blob) return VSA_E_INVALID;
    const uint8_t *p = (const uint8_t *)blob;
    size_t size;
    if (bare_type < 0) {
        size = VSA_ROUNDUP_CL(sizeof(HWLM)) +
               engine_size(p + VSA_ROUNDUP_CL(sizeof(HWLM)), p[0]);
    } else {
        if (bare_type != HWLM_ENGINE_NOOD && bare_type != HWLM_ENGINE_FDR) return VSA_E_INVALID;
        size = engine_size(p, bare_type);
    }
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_registered[blob] = size;
    return VSA_OK;
}

int vsa_hwlm_unregister(const void *blob) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    return g_registered.erase(blob) ? VSA_OK : VSA_E_INVALID;
}

void vsa_set_scratch_layout(long fdr_conf_off, long fdr_conf_offset_off) {
    g_fdr_conf_off.store(fdr_conf_off);
    g_fdr_conf_offset_off.store(fdr_conf_offset_off);
}

void vsa_get_scratch_layout(long *fdr_conf_off, long *fdr_conf_offset_off) {
    *fdr_conf_off = g_fdr_conf_off.load();
    *fdr_conf_offset_off = g_fdr_conf_offset_off.load();
}

/* ---------------------------------------------------------- builder --- */

void vsa_build_opts_default(vsa_build_opts_t *o) {
    o->engine_hint = -1;
    o->allow_noodle = 1;
    o->allow_teddy = 1;
    o->allow_fat_teddy = 1;
    o->allow_flood = 1; /* the reference Grey default (grey.cpp:68) */
}

int vsa_hwlm_build(const vsa_literal_t *lits, size_t n, const vsa_build_opts_t *opts,
                   void **blob, size_t *size) {
    if (!lits || !n || !blob || !size) return VSA_E_INVALID;
    vsa::BuildOptions bo;
    if (opts) {
        bo.engine_hint = opts->engine_hint;
        bo.allow_noodle = opts->allow_noodle;
        bo.allow_teddy = opts->allow_teddy;
        bo.allow_fat_teddy = opts->allow_fat_teddy;
        bo.allow_flood = opts->allow_flood;
    }
    std::vector<vsa::Literal> v;
    v.reserve(n);
    for (size_t i = 0; i < n; i++) {
        const vsa_literal_t &l = lits[i];
        if (!l.s || !l.len) return VSA_E_INVALID;
        v.push_back(vsa::makeLiteral(l.s, l.len, l.nocase, l.noruns, l.id, l.groups, l.msk,
                                     l.cmp, l.msk_len));
    }
    uint8_t *out = nullptr;
    int r = vsa::buildHwlm(std::move(v), bo, &out, size);
    if (r != VSA_OK) return r;
    *blob = out;
    return VSA_OK;
}

void vsa_blob_free(void *blob) { free(blob); }

int vsa_hwlm_set_accel(void *blob, const union AccelAux *a0, const union AccelAux *a1,
                       uint64_t g1) {
    if (!blob) return VSA_E_INVALID;
    HWLM *h = (HWLM *)blob;
    if (a0) memcpy(&h->accel0, a0, sizeof(*a0));
    if (a1) memcpy(&h->accel1, a1, sizeof(*a1));
    h->accel1_groups = g1;
    return VSA_OK;
}

int vsa_shufti_build_masks(const uint8_t cls[32], uint8_t lo[16], uint8_t hi[16]) {
    return vsa::shuftiMasks(cls, lo, hi);
}

void vsa_truffle_build_masks(const uint8_t cls[32], uint8_t m1[16], uint8_t m2[16]) {
    vsa::truffleMasks(cls, m1, m2);
}

} /* extern "C" */
