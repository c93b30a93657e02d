"""CPU baseline thread sweep (verdict r03 item 8): the SSE2 port of the
reference FDR main loop (oracle.c, bench.py's cpu_baseline engine) over a
1 GiB sample of the cfg-4 corpus at 16 / 32 / 64 / all-allowed threads,
pinned one per physical core (then wrapping onto the core list), beside the
cgroup CPU quota.  CPU only; run on the GPU box for its host numbers.
  python tools/exp_cpu_threads.py [GiB]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import oracle  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
n = int(gib * (1 << 30))
lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
eng = vsa.engine_blob(blob)
data = bench.make_corpus(n, lits, seed=5, plant_every=64 << 10)
pins, quota, visible, phys = bench.host_cpu_share()
oracle.set_pin(pins)
want = None
for t in sorted({16, 32, 64, len(pins), len(os.sched_getaffinity(0))}):
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        d = oracle.digest_mt(eng, data, t, simd=True)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    want = want or d
    print(json.dumps({"threads": t, "GBps": round(n / best / 1e9, 3), "s": round(best, 4),
                      "match_set_equal": d == want, "cpu_quota": quota,
                      "physical_cores": phys, "cpus_visible": visible,
                      "cpu": bench._cpu_model()}), flush=True)
