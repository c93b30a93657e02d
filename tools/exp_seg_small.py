"""Kernel time of the cfg-4 scan at per-rank stripe sizes (strong scaling:
4 GiB / N per GPU) against the segment size (VSA_SEG_KB; 0 = the planner's
choice; the plan is memoized per context, so one size per process).
Usage: [VSA_SEG_KB=k] exp_seg_small.py MIB"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

mib = int(sys.argv[1])
dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
total = mib << 20
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
offs = [i * bl for i in range(4)]
torch.cuda.synchronize()
ks = []
settle = int(os.environ.get("SETTLE", "20"))  # untimed launches (GPU clock ramp)
for i in range(settle + 40):
    n = ctx.scan_blocks(db, data.data_ptr(), offs, [bl] * 4)
    if i >= settle:
        ks.append(ctx.kernel_ms())
print("MiB %d seg_kb %s steal %s steal_w %s kernel median %.4f ms min %.4f matches %d" % (
    mib, os.environ.get("VSA_SEG_KB", "auto"), os.environ.get("VSA_STEAL", "-"),
    os.environ.get("VSA_STEAL_W", "-"), float(np.median(ks)), min(ks), n),
    flush=True)
