"""Median kernel time (hipEvents, clock-settled) of the cfg-4 FDR scan at
several sizes: 512 MiB (the N = 8 rank stripe), 1 GiB, 4 GiB as 4 blocks.
One JSON line; the library is the one VSA_LIB_VARIANT names (A/B builds,
tools/archive/build_variant.sh)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
total = 4 << 30
lits = bench.make_literals(int(os.environ.get("LITS", "5000")), seed=12)
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
torch.cuda.synchronize()
base = data.data_ptr()
res = {"variant": os.environ.get("VSA_LIB_VARIANT", "default")}
for mib, nb in ((512, 1), (1024, 1), (4096, 4)):
    bl = (mib << 20) // nb
    offs = [i * bl for i in range(nb)]
    plan = ctx.plan(base, offs, [bl] * nb)
    for _ in range(60):
        ctx.scan_plan(db, plan)
    ks, n = [], 0
    for _ in range(40):
        n = ctx.scan_plan(db, plan)
        ks.append(ctx.kernel_ms() * 1000.0)
    res["us_%d" % mib] = round(float(np.median(ks)), 1)
    res["n_%d" % mib] = int(n)
print(json.dumps(res), flush=True)
