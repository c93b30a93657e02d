"""Cost of a crowded sort bin: a binned scan's records
live only in their bins, so a bin past VSA_SORT_BIN_MAX records makes the
launch run again without bins, and the context then skips bins for
bin_backoff launches (16, x4 per repeated crowd, up to 4,096).  Workloads:
256 MiB printable (seed 5), noodle "abcde" / FDR 5k literals (bench.py's),
one literal planted per 4 KiB ("sparse"), and the same plus a burst every
1 MiB -- a 1 KiB window of one literal repeated, ~200 records in one
16 KiB bin ("bursty").  Per workload: CALLS synchronous plan scans, the
mean / p50 / p99 wall time per call, the scan kernel time, launches per
call and the calls that ran twice (the crowds).  The bursty steady state
is the unbinned path (output + library sort); bursty minus sparse is what a
crowd costs per call.
  python tools/exp_dense.py [calls]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n = 256 << 20
rng = np.random.default_rng(5)
base = rng.integers(0x20, 0x7F, n, dtype=np.uint8)
settle = vsa.Context(0)
for name, lits in (("noodle", [vsa.HwlmLiteral(b"abcde", False, 1)]),
                   ("fdr5k", bench.make_literals(5000, seed=12))):
    text = lits[0].s
    for kind in ("sparse", "bursty"):
        buf = base.copy()
        pl = np.frombuffer(text, np.uint8)
        for o in range(0, n - 4096, 4096):
            buf[o + 100:o + 100 + len(pl)] = pl
        if kind == "bursty":
            rep = np.frombuffer(text * (1000 // len(text)), np.uint8)
            for o in range(0, n - 4096, 1 << 20):
                buf[o + 2048:o + 2048 + len(rep)] = rep
        ctx = vsa.Context(0)  # fresh: no backoff carried over
        d = ctx.malloc(n)
        ctx.h2d(d, buf)
        db = vsa.Database(ctx, vsa.hwlm_build(lits))
        plan = ctx.plan(d, [0], [n])
        # clock settle on another context (its crowds are not this one's)
        sdb = vsa.Database(settle, vsa.hwlm_build(lits))
        splan = settle.plan(d, [0], [n])
        for _ in range(60):
            settle.scan_plan(sdb, splan)
        splan.close()
        sdb.close()
        walls, ks, twice, cnt = [], [], [], set()
        for i in range(calls):
            l0 = ctx.launches()
            t0 = time.perf_counter()
            cnt.add(ctx.scan_plan(db, plan))
            walls.append((time.perf_counter() - t0) * 1e3)
            ks.append(ctx.kernel_ms())
            if ctx.launches() - l0 > 1:
                twice.append(i)
        w = np.array(walls)
        print(json.dumps({"db": name, "corpus": kind, "calls": calls, "matches": sorted(cnt),
                          "wall_ms_mean": round(float(w.mean()), 4),
                          "wall_ms_p50": round(float(np.median(w)), 4),
                          "wall_ms_p99": round(float(np.percentile(w, 99)), 4),
                          "kernel_ms_mean": round(float(np.mean(ks)), 4),
                          "first_call_ms": round(walls[0], 4),
                          "rerun_calls": twice[:12], "reruns": len(twice)}), flush=True)
        plan.close()
        db.close()
        ctx.free(d)
        ctx.close()
settle.close()
