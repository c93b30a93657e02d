"""cfg-4 scan kernel time and the confirm-wave phase counters
(VSA_DEBUG_FLAGS=64: [4] gather [5] expand [6] confirm [7] idle cycles,
[8] gathers [9] chunk entries [10] expansion rounds [11] confirm batches)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

ctx = vsa.Context(0)
lits = bench.make_literals(int(os.environ.get("LITS", "5000")), seed=12)
blob = vsa.hwlm_build(lits)
db = vsa.Database(ctx, blob)
n = 4 << 30
bl = n // 4
data = bench.make_corpus_device(torch, 0, n, n, lits, 5, 64 << 10, torch.device("cuda", 0))
torch.cuda.synchronize()
ks = []
for i in range(30):
    ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)
    ks.append(ctx.kernel_ms())
c = ctx.debug_counters()
ncu = 256
print("lits %d kernel ms %.4f matches %d cand %d" % (len(lits), np.mean(ks[10:]), c[0], c[2]))
print("per CU: gather %.0f expand %.0f confirm %.0f idle %.0f cycles; gathers %.0f entries %.0f "
      "rounds %.0f batches %.0f" % tuple(x / ncu for x in c[4:12]))
