"""Schedule feedback over time: VSA_FB_TRACE=1 makes feedback_update print
each record's per-XCD deviation from the mean end (us), the applied and the
estimated weights; this runs N synchronous 4 GiB FDR 5k plan scans (one
process, the product library) and prints each launch's kernel time, so the
trace shows whether the weights settle and the XCDs end together.
EXP_MIB sets the size (4096), EXP_LITS the database (fdr: FDR 5k, teddy:
48 literals, nood: one literal).
  VSA_FB_TRACE=1 python tools/exp_fb_trace.py [launches] 2> trace.txt"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
mib = int(os.environ.get("EXP_MIB", "4096"))
dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
total = mib << 20
kind = os.environ.get("EXP_LITS", "fdr")
lits = (bench.make_literals(5000, seed=12) if kind == "fdr" else
        bench.make_literals(48, seed=55) if kind == "teddy" else
        [vsa.HwlmLiteral(b"abcde", False, 1)])
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
torch.cuda.synchronize()
nb = 4 if mib >= 1024 else 1
bl = total // nb
plan = ctx.plan(data.data_ptr(), [i * bl for i in range(nb)], [bl] * nb)
ks = []
for i in range(n):
    ctx.scan_plan(db, plan)
    ks.append(round(ctx.kernel_ms() * 1e3, 1))
    print("launch %d kernel_us %.1f" % (i, ks[-1]), file=sys.stderr, flush=True)
print(json.dumps({"mib": mib, "lits": kind, "launches": n, "kernel_us": ks}), flush=True)
plan.close()
