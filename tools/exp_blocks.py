"""Per-block overhead of the batch scan: 1 GiB cut into blocks of 2 KiB ..
1 MiB, wall time of vsa_scan_blocks (tables built per call) and of
vsa_scan_plan (tables built once) vs the kernel time (cfg-4 FDR set).
The blocks are back to back, so packed segments scan as runs; run with
VSA_NO_RUNS=1 for the per-block path.
  python tools/exp_blocks.py [TOTAL_MIB [CHUNK_KIB ...]]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
ctx = vsa.Context(0)
db = vsa.Database(ctx, blob)
total = (int(sys.argv[1]) << 20) if len(sys.argv) > 1 else 1 << 30
data = bench.make_corpus(total, lits, seed=5, plant_every=64 << 10)
d = ctx.malloc(total)
ctx.h2d(d, data)
for _ in range(40):  # clock settle (profiles/r03_ramp.jsonl)
    ctx.scan_blocks(db, d, [0], [total])
chunks = [int(x) << 10 for x in sys.argv[2:]] or [2 << 10, 4 << 10, 16 << 10, 64 << 10, 1 << 20, 256 << 20]
for chunk in chunks:
    n = total // chunk
    offs = np.arange(n, dtype=np.uint64) * chunk
    lens = np.full(n, chunk, np.uint64)
    for _ in range(3):
        ctx.scan_blocks(db, d, offs, lens)
    walls, ks = [], []
    for _ in range(10):
        t0 = time.perf_counter()
        m = ctx.scan_blocks(db, d, offs, lens)
        walls.append(time.perf_counter() - t0)
        ks.append(ctx.kernel_ms())
    plan = ctx.plan(d, offs, lens)
    pw = []
    for _ in range(10):
        t0 = time.perf_counter()
        m2 = ctx.scan_plan(db, plan)
        pw.append(time.perf_counter() - t0)
    plan.close()
    assert m2 == m
    print("chunk %8d blocks %7d matches %6d wall %.3f ms plan wall %.3f ms kernel %.3f ms" %
          (chunk, n, m, min(walls) * 1e3, min(pw) * 1e3, min(ks)), flush=True)
