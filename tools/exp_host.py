"""Host-side cost of a per-call vsa_scan_blocks plan (1 GiB resident, cfg-4
literal set, blocks of 2 KiB / 16 KiB / 256 MiB): run with VSA_HOST_TIMING=1
for the library's build / copy / launch+wait split per call."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

lits = bench.make_literals(5000, seed=12)
ctx = vsa.Context(0)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
total = 1 << 30
data = bench.make_corpus(total, lits, seed=5, plant_every=64 << 10)
d = ctx.malloc(total)
ctx.h2d(d, data)
for chunk in [2 << 10, 16 << 10, 256 << 20]:
    n = total // chunk
    offs = np.arange(n, dtype=np.uint64) * chunk
    lens = np.full(n, chunk, np.uint64)
    for i in range(4):
        t0 = time.perf_counter()
        ctx.scan_blocks(db, d, offs, lens)
        t1 = time.perf_counter()
        print("chunk", chunk, "wall %.3f ms" % ((t1 - t0) * 1e3), flush=True)
