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
#include <hipcub/hipcub.hpp>

#include "runtime_internal.h"

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

namespace vsa_rt {

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

int ensure_tables(vsa_ctx *c, uint32_t nb, uint64_t nsegs, bool keep_blocks) {
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

/* the least gain (us of kernel time) that applies new weights;
 * VSA_FB_GAIN_US=-1 restores the earlier rule (any weight moved by 2 %) */
int fb_gain_us() {
    static const int v = env_int("VSA_FB_GAIN_US", 4);
    return v;
}

/* Dynamic shares (kernels.hip dyn_bounds): an option (VSA_DYN_SHARES=1, or
 * vsa_ctx_set_dyn_shares per context) for the FDR launches of at least
 * VSA_DYN_MIN_MIB (default 2048) MiB over eligible plans (build_plan: >=
 * 256 MiB of parts of blocks in address order).  Off by default: measured
 *  it takes the XCDs' spread at 4 GiB from 8-17 to 5
 * us, but the kernel and the pipelined bench step come out even or 0.3 %
 * slower on two of three boxes (791 -> 773 us synchronous on the third);
 * the streaming scans (noodle, Teddy), whose XCDs share HBM bandwidth,
 * were 3-4 % slower at 1 GiB, so they never take it. */
bool dyn_shares_on() {
    static const bool v = env_int("VSA_DYN_SHARES", 0) != 0;
    return v;
}

uint64_t dyn_min_bytes() {
    static const uint64_t v = (uint64_t)std::max(0, env_int("VSA_DYN_MIN_MIB", 2048)) << 20;
    return v;
}

static bool fb_trace() {
    static const bool v = env_int("VSA_FB_TRACE", 0) != 0;
    return v;
}

/* arm the feedback record of the next launch (set: FbSet kind) */
void arm_feedback(vsa_ctx *c, int set, uint32_t grid, uint64_t bytes, bool small) {
    c->fb.armed = xcd_feedback_on() && c->fb.h && grid >= 64 && grid <= 1024 &&
                  bytes >= (256u << 20) && !small ? set : -1;
    c->fb.grid = grid;
    /* a scan whose counters vsa_bin_finish publishes records in device
     * memory and rides on the publish; otherwise (and under the fused
     * finish, whose publish would wait for them) host stores, a record
     * not yet complete when the host reads it being skipped
     * (feedback_update) */
    c->fb.dev = c->fb.armed >= 0 && c->fb.d_rec && c->launch.bins && !small &&
                !c->launch.fused;
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
    if (const int gus = fb_gain_us(); gus >= 0) {
        /* the rule in time: with shares wa an XCD ends in proportion to
         * wa / nw (nw estimates its rate), with nw all together, so the
         * launch would end (max r / mean r - 1) of its length earlier.
         * The 2 % rule above left XCDs up to 11-20 us apart on a 4 GiB
         * scan (1.4 % moves, never applied: profiles/r06/r06w_wg_spread.jsonl,
         * whose per-XCD spread is all of the workgroups' persistent spread);
         * apply when the gain is worth the refresh (~10-20 us, at most once
         * per 16 launches) */
        double rmax = 0, rsum = 0, rn = 0;
        for (int x = 0; x < 8; x++)
            if (cnt[x]) {
                const double r = F.wa[x] / nw[x];
                rmax = std::max(rmax, r);
                rsum += r;
                rn += 1;
            }
        moved = (rmax * rn / rsum - 1.0) * tm / 100.0 > (double)gus;
    }
    if (fb_trace()) {
        /* diagnostic (VSA_FB_TRACE=1): one line per record to stderr */
        fprintf(stderr, "fb v%u tm_us %.1f", F.version, tm / 100.0);
        for (int x = 0; x < 8; x++)
            fprintf(stderr, " x%d %+.2f/%.4f/%.4f", x,
                    cnt[x] ? (sum[x] / cnt[x] - tm) / 100.0 : 0.0, F.wa[x], nw[x]);
        fprintf(stderr, " moved %d\n", (int)moved);
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

unsigned long long *g_wave_log = nullptr;

/* the fused finish's default for new contexts: VSA_FUSED_FINISH=1 turns
 * it on (vsa_ctx_set_fused_finish per context).  Off by default: measured
 * against the vsa_bin_finish launch it shortens the pipelined step by 0.4-
 * 2.5 us (0.3-0.8 %) but lengthens the scan kernel by 5-6 us
 * (profiles/r06/r06q_fused_publish_ab.jsonl) */
bool fused_finish_default() {
    static const bool v = env_int("VSA_FUSED_FINISH", 0) != 0;
    return v;
}

/* the fused finish's buffers: local-bin staging for `grid` workgroups
 * (grown, never shrunk) and the totals (zero: no epoch matches) */
int ensure_fstage(vsa_ctx *c, uint32_t grid) {
    Workspace &w = c->ws;
    if (grid > VSA_FIN_MAX_GRID) return VSA_E_INVALID;
    if (!w.d_fagg) {
        VSA_CHECK(hipMalloc(&w.d_fagg, 2 * VSA_FIN_MAX_GRID * sizeof(unsigned long long)));
        VSA_CHECK(hipMemsetAsync(w.d_fagg, 0, 2 * VSA_FIN_MAX_GRID * sizeof(unsigned long long),
                                 c->stream));
    }
    if (grid > w.fstage_grid) {
        if (w.d_fstage) {
            /* the previous launch may still read the old staging */
            VSA_CHECK(hipStreamSynchronize(c->stream));
            VSA_CHECK(hipFree(w.d_fstage));
            w.d_fstage = nullptr;
            w.fstage_grid = 0;
        }
        VSA_CHECK(hipMalloc(&w.d_fstage, (size_t)grid * VSA_LBINS * VSA_SORT_BIN_MAX *
                                             (sizeof(uint64_t) + sizeof(uint32_t))));
        w.fstage_grid = grid;
    }
    return VSA_OK;
}

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
    /* the fused finish: the scan sorts its records itself (kernels.hip
     * fused_finish) when the plan's local bins allow it (plan_fused) */
    c->launch.fused = c->launch.bins && c->launch.fin_ok && c->launch.db &&
                      !c->launch.db->split && c->launch.db->mode != VSA_MODE_FAT &&
                      c->fused_finish;
    if (c->launch.fused) {
        if (int r = ensure_fstage(c, c->launch.grid)) return r;
    } else {
        if (c->launch.bins && !c->ws.d_bstage)
            VSA_CHECK(hipMalloc(&c->ws.d_bstage, (size_t)VSA_SORT_BINS * VSA_SORT_BIN_MAX *
                                                     (sizeof(uint64_t) + sizeof(uint32_t))));
        const uint32_t par = c->bin_par;
        if (c->launch.bins && !c->bins_clean[par])
            VSA_CHECK(hipMemsetAsync(bin_counts_of(c, par), 0, VSA_SORT_BINS * sizeof(uint32_t),
                                     c->stream));
        c->bins_clean[par] = false;
    }
    /* drop-in calls (a few records, sorted by the host) skip the kernel
     * timing and get their counters and records published (no copies) */
    const bool small = (c->launch.flags & SCAN_HOST_SORT_SMALL) != 0;
    /* the timing events ride on every timing_every-th dispatch only
     * (vsa_ctx_set_timing: they cost ~4 us per step at 512 MiB,
     * profiles/r06/r06n_gap_knobs.jsonl) */
    c->launch.timed = !small && c->timing_every &&
                      (c->lit_launches % (uint64_t)c->timing_every) == 0;
    c->launch.ev_start = c->launch.timed ? c->ev0 : nullptr;
    c->launch.ev_stop = c->launch.timed ? c->ev1 : nullptr;
    /* dynamic shares: the launch balances its XCDs itself (its records go
     * to the stream's state, not to the host feedback) */
    c->launch.dyn = c->launch.dyn_kib && c->dyn_shares && !c->launch.fused && !small &&
                    db->mode == VSA_MODE_FDR4 && c->launch.bytes >= c->dyn_min &&
                    c->launch.grid >= 64 && c->launch.grid <= 256 && c->dyn;
    if (c->launch.dyn) arm_feedback(c, 0, 0, 0, true); /* disarmed */
    else arm_feedback(c, fb_set_of(db), c->launch.grid, c->launch.bytes, small);
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
    if (c->launch.fused) {
        /* sorted, packed and published by the scan itself */
        c->launch.pack_dst = nullptr;
        c->launch.dev_sort = true;
        c->launch.published = true;
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
    if (c->launch.dyn) {
        /* dynamic shares (kernels.hip dyn_bounds): this launch's records and
         * weights in buffer epoch & 1, the previous dynamic launch's (same
         * grid and mode, complete by stream order) in the other */
        DynState &D = *c->dyn;
        constexpr size_t REC = 512, WTS = 8;
        if (!D.d) {
            VSA_CHECK(hipMalloc(&D.d, (2 * REC + WTS) * sizeof(unsigned long long)));
            VSA_CHECK(hipMemsetAsync(D.d, 0, (2 * REC + WTS) * sizeof(unsigned long long),
                                     c->stream));
        }
        const uint64_t e = ++D.epoch;
        c->launch.dyn_epoch = e;
        const bool prev = D.grid == c->launch.grid && D.kind == db->mode;
        uint32_t *wts = (uint32_t *)(D.d + 2 * REC);
        P.wg_time = D.d + (e & 1) * REC;
        P.dyn_prev = prev ? D.d + ((e - 1) & 1) * REC : nullptr;
        P.dyn_wprev = prev ? wts + ((e - 1) & 1) * WTS : nullptr;
        P.dyn_wout = wts + (e & 1) * WTS;
        P.dyn_kib = c->launch.dyn_kib;
        P.dyn_margin = c->launch.dyn_margin;
        /* the plan's owned bins of the sure ranges (plan_wg_bins: after the
         * static table and the fused finish's) */
        P.wg_bins = c->launch.d_segblk + 4 * nsegs + 7 * (size_t)c->launch.grid + 1;
        D.grid = c->launch.grid;
        D.kind = db->mode;
    }
    P.wave_log = g_wave_log;
    if (c->launch.fused) {
        /* the fused finish (kernels.hip fused_finish): local bins in the
         * fused staging, the plan's local-bin table after its owned bins,
         * sorted records into buffer 1 (as vsa_bin_finish), published by the
         * last workgroup out with this launch's sequence */
        const uint32_t G = c->launch.grid;
        P.bin_keys = (uint64_t *)w.d_fstage;
        P.bin_ids = (uint32_t *)(w.d_fstage + (size_t)w.fstage_grid * VSA_LBINS *
                                                  VSA_SORT_BIN_MAX * sizeof(uint64_t));
        P.bin_counts = nullptr;
        P.fin_wg = c->launch.d_segblk + 4 * nsegs + G + 1 + 2 * (size_t)G;
        P.fin_keys = w.d_keys[1];
        P.fin_ids = w.d_ids[1];
        P.fin_agg = w.d_fagg;
        P.fin_seq = ++c->pub_seq;
        P.fin_epoch = (uint32_t)(P.fin_seq % 0xfffffffeULL) + 1u;
        P.fin_pub = w.d_pub;
        P.fin_pk = (uint64_t *)c->launch.pack_dst;
        P.fin_pk_cap = c->launch.pack_cap;
    }
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
    if (fb_trace() && c->launch.dyn) {
        /* diagnostic (VSA_FB_TRACE=1): the dynamic shares' weights and the
         * per-XCD end deviations of this launch (us), to stderr */
        /* (the launch is complete; a later one writes the other buffer) */
        const DynState &D = *c->dyn;
        const uint64_t ep = c->launch.dyn_epoch;
        unsigned long long rec[512 + 4];
        const uint32_t G = c->launch.grid;
        if (hipMemcpy(rec, D.d + (ep & 1) * 512, 2 * G * 8, hipMemcpyDeviceToHost) ==
                hipSuccess &&
            hipMemcpy(rec + 512, D.d + 1024 + (ep & 1) * 4, 32, hipMemcpyDeviceToHost) ==
                hipSuccess) {
            const uint32_t *wq = (const uint32_t *)(rec + 512);
            double s[8] = {0}, k[8] = {0}, t0 = 1e300;
            for (uint32_t b = 0; b < G; b++) t0 = std::min(t0, (double)rec[G + b]);
            for (uint32_t b = 0; b < G; b++) {
                const uint32_t x = (uint32_t)(rec[b] >> 60) & 7u;
                s[x] += (double)(rec[b] & ((1ULL << 60) - 1)) - t0;
                k[x] += 1;
            }
            double tm = 0, nx = 0;
            for (int x = 0; x < 8; x++)
                if (k[x]) tm += s[x] / k[x], nx += 1;
            tm /= nx;
            fprintf(stderr, "dyn e%llu tm_us %.1f", (unsigned long long)ep, tm / 100.0);
            for (int x = 0; x < 8; x++)
                fprintf(stderr, " x%d %+.2f/%.4f", x, k[x] ? (s[x] / k[x] - tm) / 100.0 : 0.0,
                        wq[x] / 65536.0);
            fprintf(stderr, "\n");
        }
    }
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
    if (!c->launch.timed) {
        c->kms_stale = false;
        if (!(flags & SCAN_HOST_SORT_SMALL)) c->last_kernel_ms = -1.0; /* untimed */
    } else if (c->launch.fused) {
        /* the scan published from inside itself: its end event may not be
         * written yet, so the kernel time is read when asked for
         * (vsa_scan_kernel_ms) */
        c->kms_stale = true;
    } else if (!(flags & SCAN_HOST_SORT_SMALL)) {
        c->kms_stale = false;
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


/* launch a planned batch whose tables are on the device */
int launch_planned(vsa_ctx *c, const vsa_db *db, const uint8_t *d_data, const VsaBlock *d_blocks,
                   const uint32_t *d_segblk, uint32_t nb, uint64_t segs,
                   uint32_t grid, int end_bits, uint64_t bytes, uint32_t flags, uint64_t *n_out,
                   bool fin_ok, uint32_t dyn_kib, uint32_t dyn_margin) {
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
    c->launch.fin_ok = fin_ok;
    c->launch.dyn_kib = dyn_kib;
    c->launch.dyn_margin = dyn_margin;
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
                     const uint64_t *hlens, const uint64_t *rlos) {
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
    const uint64_t waves = (uint64_t)c->plan_cus() * ns_plan;
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
                          pl.grid, pl.end_bits, pl.bytes, flags, n_out, pl.fin_ok, pl.dyn_kib,
                          pl.dyn_margin);
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

} // namespace vsa_rt

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
    c->fused_finish = fused_finish_default();
    c->dyn_shares = dyn_shares_on();
    c->dyn_min = dyn_min_bytes();
    VSA_CHECK(hipSetDevice(device));
    int cus = 0;
    VSA_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    c->num_cus = cus > 0 ? cus : 256;
    VSA_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->stream_ref.reset((void *)c->stream, [](void *st) { (void)hipStreamDestroy((hipStream_t)st); });
    c->dyn = std::make_shared<DynState>();
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
    if (w.d_fstage) (void)hipFree(w.d_fstage);
    if (w.d_fagg) (void)hipFree(w.d_fagg);
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
    if (c->ev_mark) (void)hipEventDestroy(c->ev_mark);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
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
    c->dyn = base->dyn;               /* one dynamic-share state per stream */
    c->reserved_cus = base->reserved_cus;
    c->fused_finish = base->fused_finish;
    c->timing_every = base->timing_every;
    c->dyn_shares = base->dyn_shares;
    c->dyn_min = base->dyn_min;
    c->stream = base->stream;
    *out = c;
    return VSA_OK;
}

void *vsa_ctx_stream(vsa_ctx_t *c) { return c ? (void *)c->stream : nullptr; }

int vsa_ctx_set_reserved_cus(vsa_ctx_t *c, int n) {
    if (!c || n < 0 || n >= c->num_cus) return VSA_E_INVALID;
    c->reserved_cus = n;
    c->memo.valid = false; /* per-call plans are rebuilt for the new grid */
    return VSA_OK;
}

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

double vsa_scan_kernel_ms(vsa_ctx_t *c) {
    if (!c) return 0.0;
    if (c->kms_stale) {
        /* the end event of a fused-finish scan: polled, as wait_stream (a
         * blocking wait wakes late and would hold up the caller's next
         * launch) */
        c->kms_stale = false;
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e;
        while ((e = hipEventQuery(c->ev1)) == hipErrorNotReady) {
            (void)hipGetLastError();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
                e = hipEventSynchronize(c->ev1);
                break;
            }
        }
        float ms = 0.f;
        if (e == hipSuccess && hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess)
            c->last_kernel_ms = ms;
        (void)hipGetLastError();
    }
    return c->last_kernel_ms;
}

uint64_t vsa_scan_launches(vsa_ctx_t *c) { return c ? c->lit_launches : 0; }

int vsa_scan_last_fused(vsa_ctx_t *c) { return c && c->launch.fused ? 1 : 0; }

int vsa_scan_last_dyn(vsa_ctx_t *c) { return c && c->launch.dyn ? 1 : 0; }

int vsa_ctx_set_dyn_shares(vsa_ctx_t *c, int on, uint64_t min_bytes) {
    if (!c) return VSA_E_INVALID;
    c->dyn_shares = on != 0;
    c->dyn_min = min_bytes;
    return VSA_OK;
}

int vsa_ctx_set_timing(vsa_ctx_t *c, uint32_t every) {
    if (!c) return VSA_E_INVALID;
    c->timing_every = every;
    return VSA_OK;
}

int vsa_ctx_set_fused_finish(vsa_ctx_t *c, int on) {
    if (!c) return VSA_E_INVALID;
    c->fused_finish = on != 0;
    return VSA_OK;
}

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
        c->kms_stale = false;
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

void vsa_set_wave_log(void *d_log) { g_wave_log = (unsigned long long *)d_log; }

} /* extern "C" */
