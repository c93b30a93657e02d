"""Per-wave log of the cfg-4 scan (VSA_DEBUG_FLAGS=4096, vsa_set_wave_log):
when each scanning wave started and ended, how much it scanned, and where it
ran (XCC, HW_ID), to find what sets the schedule's tail."""
import ctypes
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(4096 | 16384 | int(os.environ.get("EXTRA_DBG", "0")))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
# WORKLOAD=noodle: cfg 1's single literal (noodle engine); else cfg 4's set
# WORKLOAD=teddy: cfg 3's 48 literals (seed 55, Teddy), planted every 4 KiB
plant = 64 << 10
hint = -1
if os.environ.get("WORKLOAD") == "noodle":
    lits = [vsa.HwlmLiteral(b"abcde", False, 1)]
elif os.environ.get("WORKLOAD") == "teddy":
    import tools.bench_configs as bc
    lits = bc.lits_printable(48, 55)
    plant = 4 << 10
else:
    lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctx, vsa.hwlm_build(lits, engine_hint=hint))
total = int(float(os.environ.get("GIB", "4")) * (1 << 30))
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, plant, dev)
log = torch.zeros(1024 * 16 * 8, dtype=torch.int64, device=dev)
vsa.lib.vsa_set_wave_log.argtypes = [ctypes.c_void_p]
vsa.lib.vsa_set_wave_log(log.data_ptr())
torch.cuda.synchronize()
offs = [i * bl for i in range(4)]
per_launch = []
for i in range(22):
    log.zero_()
    ctx.scan_blocks(db, data.data_ptr(), offs, [bl] * 4)
    if i >= 0:
        # per-XCD workgroup done time (us from the first wave start) of
        # this launch: is the XCD order stable launch to launch?
        LL = log[:65536].view(-1, 8).cpu().numpy().astype(np.int64)
        LL = LL[(LL[:, 0] != 0) & (LL[:, 1] != 0)]
        tz = LL[:, 0].min()
        xd = {}
        for w, x, e in zip(LL[:, 4].tolist(), (LL[:, 6] & 0xf).tolist(), ((LL[:, 1] - tz) / 100.0).tolist()):
            xd.setdefault(x, {}).setdefault(w, 0)
            xd[x][w] = max(xd[x][w], e)
        bx = {w: x for w, x in zip(LL[:, 4].tolist(), (LL[:, 6] & 0xf).tolist())}
        rr = sum(1 for w, x in bx.items() if w % 8 == x)
        per_launch.append("launch %d kernel %.4f ms; xcd p50 done: %s; wg%%8==xcc %d/%d" % (
            i, ctx.kernel_ms(), " ".join("%d:%.1f" % (x, np.median(list(v.values())))
                                        for x, v in sorted(xd.items())), rr, len(bx)))
LA = log.cpu().numpy().astype(np.int64)
L = LA[:65536].reshape(-1, 8)
nev = int(LA[65535])
EV = LA[65536:65536 + 4 * min(nev, 16000)].reshape(-1, 4)
for line in per_launch:
    print(line)
L = L[L[:, 0] != 0]
L = L[L[:, 1] != 0] if len(L) else L
t0 = L[:, 0].min()
st, en = (L[:, 0] - t0) / 100.0, (L[:, 1] - t0) / 100.0
it = L[:, 3]
rate = it / np.maximum(en - st, 1e-3)  # KiB per us
print("kernel %.4f ms, %d scanning waves" % (ctx.kernel_ms(), len(L)))
print("start us: min %.1f p50 %.1f p99 %.1f max %.1f" % (st.min(), np.median(st), np.percentile(st, 99), st.max()))
print("end   us: min %.1f p1 %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f" %
      (en.min(), *np.percentile(en, [1, 10, 50, 90, 99]), en.max()))
print("KiB/us per wave: p1 %.3f p50 %.3f p99 %.3f" % tuple(np.percentile(rate, [1, 50, 99])))
print("segments per wave: min %d max %d; KiB per wave min %d p50 %d max %d" %
      (L[:, 2].min(), L[:, 2].max(), it.min(), np.median(it), it.max()))
xcc = L[:, 6] & 0xf
for x in sorted(set(xcc.tolist())):
    m = xcc == x
    print("xcc %d: waves %d, end p50 %.1f max %.1f, KiB/us p50 %.3f, KiB total %d" %
          (x, m.sum(), np.median(en[m]), en[m].max(), np.median(rate[m]), it[m].sum()))
wv = L[:, 5]
print("KiB/us p50 by wave: " + " ".join("%d:%.2f" % (w, np.median(rate[wv == w]))
                                        for w in sorted(set(wv.tolist()))))
wg = L[:, 4]
wg_end = {}
for w, e in zip(wg.tolist(), en.tolist()):
    wg_end[w] = max(wg_end.get(w, 0), e)
we = np.array(sorted(wg_end.values()))
print("workgroup done us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f" %
      (we.min(), *np.percentile(we, [10, 50, 90]), we.max()))
# per workgroup: bytes scanned and the rate over its busy span
wk, wkib = {}, {}
for w, k, s0, e0 in zip(wg.tolist(), it.tolist(), st.tolist(), en.tolist()):
    wkib[w] = wkib.get(w, 0) + k
wr = np.array([wkib[w] / max(wg_end[w], 1e-3) for w in sorted(wg_end)])
print("workgroup KiB: min %d p50 %d max %d; KiB/us (share / done): min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f" %
      (min(wkib.values()), np.median(list(wkib.values())), max(wkib.values()),
       wr.min(), *np.percentile(wr, [10, 50, 90]), wr.max()))
wxcc = {}
for w, x in zip(wg.tolist(), xcc.tolist()):
    wxcc[w] = x
for x in sorted(set(wxcc.values())):
    ends = [wg_end[w] for w in wg_end if wxcc[w] == x]
    print("xcc %d workgroups done us: min %.1f p50 %.1f max %.1f" % (x, min(ends), np.median(ends), max(ends)))
order = np.argsort(-en)[:12]
print("latest waves: end, start, segs, KiB, wg, wave, xcc, rate")
for k in order:
    print("  %.1f %.1f %d %d %d %d %d %.3f" % (en[k], st[k], L[k, 2], it[k], L[k, 4], L[k, 5], xcc[k], rate[k]))

# pool takes: when each workgroup took its pool segments
if len(EV):
    et = (EV[:, 0] - t0) / 100.0
    print("pool takes %d: first %.1f p10 %.1f p50 %.1f p90 %.1f last %.1f us" %
          (len(EV), et.min(), *np.percentile(et, [10, 50, 90]), et.max()))
    pw = {}
    for w, t in zip(EV[:, 1].tolist(), et.tolist()):
        pw.setdefault(w, []).append(t)
    firsts = np.array([min(v) for v in pw.values()])
    print("workgroups taking pool: %d; first take p10 %.1f p50 %.1f p90 %.1f; takes per wg p50 %d max %d" %
          (len(pw), *np.percentile(firsts, [10, 50, 90]), np.median([len(v) for v in pw.values()]),
           max(len(v) for v in pw.values())))
    late = sorted(wg_end, key=lambda w: -wg_end[w])[:6]
    early = sorted(wg_end, key=lambda w: wg_end[w])[:6]
    for tag, ws in (("latest", late), ("earliest", early)):
        for w in ws:
            v = sorted(pw.get(w, []))
            print("  %s wg %d done %.1f KiB %d pool takes %d at %s" %
                  (tag, w, wg_end[w], wkib[w], len(v), " ".join("%.0f" % x for x in v[:12])))
