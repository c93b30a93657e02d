"""One GPU, the per-rank step of bench.py at N = 1, 2, 4, 8 (verdict r02
item 4): rank 0's windows of plan_corpus_stripes over the 4 GiB cfg-4
corpus (4 / 2 / 1 / 0.5 GiB), scanned exactly as a rank's step does
(vsa_scan_blocks_ex with report_lo, count read back), warm, then K timed
steps.  Prints one JSON line per N: step ms, kernel ms, step - kernel.
The collective is not part of this (one GPU); it is what an N-rank run adds.
  python tools/exp_stripes.py [steps] [warmup]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402
from vectorscan_amd import stripe  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
total = 4 << 30
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
torch.cuda.synchronize()
dptr = data.data_ptr()
for n in (1, 2, 4, 8):
    cuts, plan = stripe.plan_corpus_stripes(total, bl, n)
    wins = plan[0]
    offs = [w.wlo for w in wins]
    lens = [w.wlen for w in wins]
    rlos = [w.rlo for w in wins]
    plan = ctx.plan(dptr, offs, lens, None, None, rlos)
    for _ in range(warm):
        ctx.scan_plan(db, plan)
    ks = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m = ctx.scan_plan(db, plan)
        ks.append(ctx.kernel_ms())
    torch.cuda.synchronize()
    st = (time.perf_counter() - t0) / steps * 1e3
    k = sum(ks) / len(ks)
    plan.close()
    print(json.dumps({"ranks": n, "rank_bytes": cuts[1] - cuts[0], "windows": len(wins),
                      "step_ms": round(st, 4), "kernel_ms": round(k, 4),
                      "overhead_us": round((st - k) * 1e3, 1), "matches": m}), flush=True)
