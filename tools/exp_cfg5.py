"""cfg-5-shaped set (bench.make_mixed_set: 10k mixed-flag literals) on 1 GiB
of 16 KiB chunks, block mode, corpus resident in HBM: per-pass wall time of
vsa_hs_corpus_scan (scan + record copy, then the host replay) one pass at a
time and pipelined (vsa_hs_corpus_scan_repeats), per replay thread count.
Run with VSA_HOST_TIMING=1 for the library's per-phase split on stderr.
  python tools/exp_cfg5.py [repeats] [plant_every_kib] [shared_ids 0/1]
(hsbench's cfg-5 corpus, tools/make_hsbench_corpus.py --mixed: 64, 0)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402
from vectorscan_amd import hs, hsbench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
plant = (int(sys.argv[2]) if len(sys.argv) > 2 else 64) << 10
shared = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
exprs, flags, ids = bench.make_mixed_set(10000, shared_ids=shared)
lits = [vsa.HwlmLiteral(e, False, i) for i, e in enumerate(exprs)]
nbytes, chunk = 1 << 30, 16 << 10
data = bench.make_corpus(nbytes, lits, seed=5, plant_every=plant)
blocks = [(i, i % 64, data[o:o + chunk].tobytes()) for i, o in enumerate(range(0, nbytes, chunk))]
del data
g = hsbench.GpuCorpus(exprs, ids, flags, blocks, hs.MODE_BLOCK)
del blocks
for _ in range(30):  # clock settle
    g.scan()
for threads in [int(t) for t in os.environ.get("EXP_THREADS", "16,8,4").split(",")]:
    t0 = time.perf_counter()
    tots, each = [], []
    for _ in range(reps):
        t1 = time.perf_counter()
        tots.append(g.scan(threads=threads)[0])
        each.append(time.perf_counter() - t1)
    one = (time.perf_counter() - t0) / reps
    g.scan_repeats(reps, threads)  # untimed: the first call sets up its second context
    t0 = time.perf_counter()
    pt = g.scan_repeats(reps, threads)
    pipe = (time.perf_counter() - t0) / reps
    print(json.dumps({"plant_every": plant, "shared_ids": shared, "threads": threads,
                      "repeats": reps, "one_ms_per_gib": round(one * 1e3, 3),
                      "one_best_ms": round(min(each) * 1e3, 3),
                      "one_median_ms": round(sorted(each)[len(each) // 2] * 1e3, 3),
                      "pipelined_ms_per_gib": round(pipe * 1e3, 3), "matches": tots[0],
                      "totals_equal": len(set(tots) | set(pt)) == 1}), flush=True)
g.close()
