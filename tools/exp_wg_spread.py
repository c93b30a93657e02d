"""Is the workgroups' end-time spread persistent?  Per-workgroup done times
(diagnostic build's wave log: the last scanning wave's end per workgroup)
over repeated 4 GiB / 512 MiB FDR scans with equal shares
(VSA_XCD_FEEDBACK=0): the spread within a launch, and the correlation of
the per-workgroup deviations between launches (persistent -> per-workgroup
shares could absorb it; random -> only dynamic balancing can).
Needs VSA_LIB_VARIANT=libvsa_diag.so (-DVSA_DIAG).
  python tools/exp_wg_spread.py"""
import ctypes
import json
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(4096 | 8192)
os.environ.setdefault("VSA_XCD_FEEDBACK", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
log = torch.zeros(1024 * 16 * 8, dtype=torch.int64, device=dev)
vsa.lib.vsa_set_wave_log.argtypes = [ctypes.c_void_p]
vsa.lib.vsa_set_wave_log(log.data_ptr())
total = 4 << 30
lits = bench.make_literals(5000, seed=12)
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
torch.cuda.synchronize()
for mib, nb in ((512, 1), (4096, 4)):
    bl = (mib << 20) // nb
    offs = [i * bl for i in range(nb)]
    plan = ctx.plan(data.data_ptr(), offs, [bl] * nb)
    for _ in range(40):
        ctx.scan_plan(db, plan)
    devs, xccs = [], None
    for _ in range(12):
        log.zero_()
        ctx.scan_plan(db, plan)
        L = log[:65536].view(-1, 8).cpu().numpy().astype(np.int64)
        sc = L[(L[:, 0] != 0) & (L[:, 1] != 0) & (L[:, 7] != 0)]
        wg = sc[:, 4]
        G = int(wg.max()) + 1
        t0 = sc[:, 7].min()
        done = np.zeros(G)
        start = np.full(G, np.inf)
        for w, e, s in zip(wg.tolist(), sc[:, 1].tolist(), sc[:, 0].tolist()):
            done[w] = max(done[w], (e - t0) / 100.0)
            start[w] = min(start[w], (s - t0) / 100.0)
        xcc = np.zeros(G, np.int64)
        for w, x in zip(wg.tolist(), sc[:, 6].tolist()):
            xcc[w] = x
        xccs = xcc
        devs.append(done - np.median(done))
    D = np.array(devs)
    c = np.corrcoef(D)
    off = c[~np.eye(len(D), dtype=bool)]
    per_xcd = [round(float(np.mean(D[:, xccs == x])), 2) for x in range(8)]
    print(json.dumps({"mib": mib, "grid": int(D.shape[1]),
                      "spread_us_p90_minus_p10": round(float(np.mean(np.percentile(D, 90, axis=1) -
                                                                     np.percentile(D, 10, axis=1))), 2),
                      "max_minus_median_us": round(float(np.mean(D.max(axis=1))), 2),
                      "launch_to_launch_corr_mean": round(float(off.mean()), 3),
                      "mean_dev_us_per_xcd": per_xcd,
                      "persistent_part_us_std": round(float(np.std(D.mean(axis=0))), 2),
                      "random_part_us_std": round(float(np.mean(np.std(D - D.mean(axis=0), axis=1))), 2)}),
          flush=True)
    plan.close()
