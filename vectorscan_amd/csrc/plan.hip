/*
 * plan.hip -- launch plans of the literal scan (host side): the block table,
 * the per-workgroup segment lists (equal or feedback-weighted shares of the
 * bytes; large blocks cut into one segment per wave, small ones packed into
 * groups and runs) and the sort bins each workgroup owns alone
 * (build_plan, plan_wg_bins), and the prebuilt-plan API (vsa_plan_create /
 * vsa_scan_plan / vsa_scan_plan_pack; refresh_plan follows the schedule
 * feedback).  tests/test_plan.py checks the plans on the CPU through
 * vsa_plan_describe.
 */
#include "runtime_internal.h"

namespace vsa_rt {

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
 * workgroup, the bins [lo, hi) (hi - lo <= VSA_LBINS; 0, 0 = none); a
 * dynamic-share plan appends a second such table after the fused finish's,
 * for its dynamic launches. */
void plan_fused(BatchPlan &pl, const VsaBlock *blocks, int64_t mis);

static void owned_bins(BatchPlan &pl, const VsaBlock *blocks, int64_t mis, bool dyn) {
    const uint32_t G = pl.grid;
    const uint64_t base = 4 * pl.nsegs;
    std::vector<int64_t> hlo(G, INT64_MAX), hhi(G, INT64_MIN);
    /* dynamic shares: workgroup b's range moves within dyn_margin KiB of
     * the equal-share boundaries, so it owns bins only inside its sure range
     * [nom_b + margin, nom_b+1 - margin) of the live KiB (the first and last
     * boundaries are fixed) */
    const uint64_t TK = dyn ? pl.dyn_kib : 0, MK = pl.dyn_margin;
    auto sure = [&](uint32_t i, bool upper) -> uint64_t {
        if (i == 0) return 0;
        if (i >= G) return TK;
        const uint64_t nom = TK * i / G;
        return upper ? (nom > MK ? nom - MK : 0) : std::min(nom + MK, TK);
    };
    for (uint32_t b = 0; b < G; b++) {
        uint32_t s0g = pl.segblk[base + b], s1g = pl.segblk[base + b + 1];
        uint64_t klo = 0, khi = 0;
        if (TK) {
            klo = sure(b, false);
            khi = sure(b + 1, true);
            /* the segments overlapping [klo, khi): word 3 ascends */
            s0g = s1g = 0;
            if (khi > klo) {
                uint32_t a = 0, e = (uint32_t)pl.nsegs;
                while (a < e) { /* first segment ending after klo */
                    const uint32_t m = (a + e) / 2;
                    const uint64_t end = (uint64_t)pl.segblk[4 * (uint64_t)m + 3] +
                                         pl.segblk[4 * (uint64_t)m + 2];
                    if (end > klo) e = m;
                    else a = m + 1;
                }
                s0g = s1g = a;
                while (s1g < pl.nsegs && pl.segblk[4 * (uint64_t)s1g + 3] < khi) s1g++;
            }
        }
        for (uint32_t sg = s0g; sg < s1g; sg++) {
            const uint32_t *d = &pl.segblk[4 * (uint64_t)sg];
            const uint32_t first = d[0] & 0xffffffu, cnt = d[0] >> 24;
            int64_t lo, hi;
            if (cnt == 0) {
                const VsaBlock &B = blocks[first];
                uint64_t off = d[1], len = d[2];
                if (TK) {
                    /* the part inside the sure range (kernels.hip's clip) */
                    const uint64_t a = std::max<uint64_t>(d[3], klo);
                    const uint64_t e = std::min<uint64_t>((uint64_t)d[3] + d[2], khi);
                    off += a - d[3];
                    len = e - a;
                }
                const int64_t s0 = B.org - mis + ((int64_t)off << 10);
                lo = std::max<int64_t>((int64_t)B.base, s0);
                hi = std::min<int64_t>((int64_t)(B.base + B.len), s0 + ((int64_t)len << 10));
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

/* the owned bins of the static lists, the fused finish's local bins, then
 * (dynamic-share plans) the owned bins of the sure ranges */
void plan_wg_bins(BatchPlan &pl, const VsaBlock *blocks, int64_t mis) {
    owned_bins(pl, blocks, mis, false);
    plan_fused(pl, blocks, mis);
    if (pl.dyn_kib) owned_bins(pl, blocks, mis, true);
}

/* The fused finish's local bins (kernels.hip fused_finish), appended to
 * segblk after the owned bins: 4 words per workgroup -- the lowest end it
 * can report (lo, hi word), the local bin shift, the local bins (<=
 * VSA_LBINS) -- over the ends its segments report: [base + max(start, rlo),
 * base + len) of each block, cut to a part's KiB range: 256 local bins
 * per workgroup, 4x finer than the global bins at 256 workgroups (fewer
 * crowds; a wave sorts its 16 bins in one pass when they are sparse).
 * Eligible (fin_ok)
 * when these hulls are disjoint and ascend with the workgroup index -- then
 * every record's bin is its own workgroup's, the workgroups' records follow
 * each other in workgroup order in the sorted output, and a workgroup's
 * look-back waits only for workgroups dispatched before it -- and the grid
 * has >= 64 workgroups (local bins then at least as fine as the global
 * ones). */
void plan_fused(BatchPlan &pl, const VsaBlock *blocks, int64_t mis) {
    const uint32_t G = pl.grid;
    const uint64_t base = 4 * pl.nsegs;
    pl.fin_ok = G >= 64 && G <= VSA_FIN_MAX_GRID;
    int64_t prev_hi = INT64_MIN;
    for (uint32_t b = 0; b < G; b++) {
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        auto add = [&](const VsaBlock &B, int64_t l, int64_t h) {
            l = std::max<int64_t>(l, (int64_t)(B.base + std::max<uint64_t>(B.start, (uint64_t)B.rlo)));
            h = std::min<int64_t>(h, (int64_t)(B.base + B.len));
            if (h > l) {
                lo = std::min(lo, l);
                hi = std::max(hi, h);
            }
        };
        for (uint32_t sg = pl.segblk[base + b]; sg < pl.segblk[base + b + 1]; sg++) {
            const uint32_t *d = &pl.segblk[4 * (uint64_t)sg];
            const uint32_t first = d[0] & 0xffffffu, cnt = d[0] >> 24;
            if (cnt == 0) {
                const VsaBlock &B = blocks[first];
                const int64_t s0 = B.org - mis + ((int64_t)d[1] << 10);
                add(B, s0, s0 + ((int64_t)d[2] << 10));
            } else {
                for (uint32_t k = 0; k < cnt; k++) {
                    const VsaBlock &B = blocks[first + k];
                    add(B, INT64_MIN, INT64_MAX);
                }
            }
        }
        uint32_t w[4] = {0, 0, 0, 0};
        if (hi > lo) {
            if (lo < prev_hi) pl.fin_ok = false;
            prev_hi = hi;
            const uint64_t span = (uint64_t)(hi - lo);
            uint32_t s = 0;
            while (((span - 1) >> s) + 1 > VSA_LBINS) s++;
            w[0] = (uint32_t)(uint64_t)lo;
            w[1] = (uint32_t)((uint64_t)lo >> 32);
            w[2] = s;
            w[3] = (uint32_t)(((span - 1) >> s) + 1);
        }
        pl.segblk.insert(pl.segblk.end(), w, w + 4);
    }
}

int build_plan(const uint8_t *d_data, const uint64_t *offs, const uint64_t *lens,
               const uint64_t *starts, const uint64_t *hlens, const uint64_t *rlos,
               uint32_t nb, uint64_t waves, BatchPlan &pl, VsaBlock *out,
               uint64_t ns, const float *wg_w) {
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
    /* one 16-byte descriptor per segment (kernels.h VsaLitParams.seg_desc);
     * word 3: the segment's position in the plan's live KiB (dynamic
     * shares) */
    uint64_t kib_pos = 0;
    auto push_desc = [&](uint32_t info, uint64_t off, uint64_t len) {
        pl.segblk.push_back(info);
        pl.segblk.push_back((uint32_t)(off >> 10));
        pl.segblk.push_back((uint32_t)((len + 1023) >> 10));
        pl.segblk.push_back((uint32_t)kib_pos);
        kib_pos += (len + 1023) >> 10;
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
    /* dynamic shares (kernels.hip dyn_bounds): large launches whose
     * segments are all parts of blocks, the blocks in ascending,
     * non-overlapping order (so the live KiB ascend with the addresses and
     * a bin inside one workgroup's sure range is its own) */
    pl.dyn_kib = pl.dyn_margin = 0;
    if (G >= 64 && G <= 256 && pl.bytes >= (256ull << 20) &&
        kib_pos < (1ull << 32) && kib_pos >= 16 * G) {
        bool ok = true;
        for (uint64_t s = 0; s < pl.nsegs && ok; s++) ok = (pl.segblk[4 * s] >> 24) == 0;
        int64_t prev_end = INT64_MIN;
        for (uint32_t i = 0; i < nb && ok; i++) {
            if (spans[i] < 0) continue;
            ok = (int64_t)out[i].base >= prev_end;
            prev_end = (int64_t)(out[i].base + out[i].len);
        }
        if (ok) {
            pl.dyn_kib = (uint32_t)kib_pos;
            /* a boundary moves at most 1/6 of a share: per-XCD weights in
             * 0.9-1.1 move the b % 8 interleave's boundaries less, and the
             * owned bins keep 2/3 of each share */
            pl.dyn_margin = (uint32_t)(kib_pos / G / 6);
        }
    }
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

} // namespace vsa_rt

extern "C" {

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

int vsa_plan_dyn(const uint8_t *d_data, const uint64_t *offsets, const uint64_t *lens,
                 const uint64_t *starts, const uint64_t *hlens, const uint64_t *report_lo,
                 uint32_t nblocks, uint32_t num_cus, uint32_t ns, uint32_t *out) {
    if (!offsets || !lens || !nblocks || !ns || !num_cus || !out) return VSA_E_INVALID;
    BatchPlan pl;
    int r = build_plan(d_data, offsets, lens, starts, hlens, report_lo, nblocks,
                       (uint64_t)num_cus * ns, pl, nullptr, ns);
    if (r != VSA_OK) return r;
    out[0] = pl.dyn_kib;
    out[1] = pl.dyn_margin;
    return VSA_OK;
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
            /* ~800 us launches (100 MHz ticks): a 4 GiB scan's length, which
             * the gain rule (fb_gain_us) weighs */
            h[b] = ((unsigned long long)(b & 7) << 60) |
                   (1000 + (unsigned long long)(t * 8e4 * grid));
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
                       (uint64_t)c->plan_cus() * (LIT_WAVES - 1), pl);
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
    p->fin_ok = pl.fin_ok;
    p->dyn_kib = pl.dyn_kib;
    p->dyn_margin = pl.dyn_margin;
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
                       (uint64_t)c->plan_cus() * (LIT_WAVES - 1), pl, nullptr, LIT_WAVES - 1,
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
    p->fin_ok = pl.fin_ok;
    p->dyn_kib = pl.dyn_kib;
    p->dyn_margin = pl.dyn_margin;
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
                          n_matches ? n_matches : &dummy, p->fin_ok, p->dyn_kib, p->dyn_margin);
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
                           p->end_bits, p->bytes, VSA_SCAN_ASYNC, &n, p->fin_ok, p->dyn_kib,
                           p->dyn_margin);
    /* not consumed (no segments, or a launch without the binned sort): the
     * records are packed the separate way, after the host completes it */
    const bool fused = c->launch.pack_dst == nullptr && c->pending;
    c->launch.pack_dst = nullptr;
    if (r != VSA_OK) return r;
    return fused ? VSA_OK : vsa_scan_pack(c, d_dst, cap);
}

} /* extern "C" */
