"""Per-wave log of the cfg-4 scan (VSA_DEBUG_FLAGS=4096, vsa_set_wave_log):
when each scanning wave started and ended, how much it scanned, and where it
ran (XCC, HW_ID), to find what sets the schedule's tail."""
import ctypes
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(4096 | int(os.environ.get("EXTRA_DBG", "0")))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
total = 4 << 30
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
log = torch.zeros(1024 * 16 * 8, dtype=torch.int64, device=dev)
vsa.lib.vsa_set_wave_log.argtypes = [ctypes.c_void_p]
vsa.lib.vsa_set_wave_log(log.data_ptr())
torch.cuda.synchronize()
offs = [i * bl for i in range(4)]
for i in range(22):
    log.zero_()
    ctx.scan_blocks(db, data.data_ptr(), offs, [bl] * 4)
L = log.view(-1, 8).cpu().numpy().astype(np.int64)
L = L[L[:, 0] != 0]
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
order = np.argsort(-en)[:12]
print("latest waves: end, start, segs, KiB, wg, wave, xcc, rate")
for k in order:
    print("  %.1f %.1f %d %d %d %d %d %.3f" % (en[k], st[k], L[k, 2], it[k], L[k, 4], L[k, 5], xcc[k], rate[k]))
