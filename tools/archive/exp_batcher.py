"""Concurrent drop-in calls, plain hwlmExec (each thread its own context,
one launch per call) against the batching service (vsa_batcher: calls of
all threads that arrive together share one launch), cfg-4 literal set:
aggregate calls/s and GB/s and the mean per-call latency, per buffer size
and thread count.  One JSON line per configuration.
  python tools/exp_batcher.py [calls_per_thread]"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

per = int(sys.argv[1]) if len(sys.argv) > 1 else 200
lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
vsa.hwlm_register(blob)
data = bench.make_corpus(64 << 20, lits, seed=5, plant_every=64 << 10)


def run(threads, size, fn):
    bufs = [data[(t * per * size) % (len(data) - size):][:size].tobytes() for t in range(threads)]
    counts = [0] * threads
    lat = [0.0] * threads

    def work(t):
        n = 0
        t0 = time.perf_counter()
        for _ in range(per):
            rc, m = fn(bufs[t])
            n += len(m)
        lat[t] = (time.perf_counter() - t0) / per
        counts[t] = n

    for t in range(threads):  # warm every thread's context / tables
        fn(bufs[t])
    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    return {"calls_per_s": round(threads * per / el), "GBps": round(threads * per * size / el / 1e9, 3),
            "mean_call_us": round(sum(lat) / threads * 1e6, 1), "matches": sum(counts)}


b = vsa.Batcher(0, max_batch=256, window_us=30)
for size in (4 << 10, 16 << 10, 64 << 10):
    for threads in (1, 8, 16):
        plain = run(threads, size, lambda d: vsa.hwlm_exec(blob, d))
        l0, c0 = b.stats()
        bat = run(threads, size, lambda d: b.hwlm_exec(blob, d))
        l1, c1 = b.stats()
        print(json.dumps({"bytes": size, "threads": threads, "plain": plain, "batcher": bat,
                          "calls_per_launch": round((c1 - c0) / max(1, l1 - l0), 1),
                          "matches_equal": plain["matches"] == bat["matches"]}), flush=True)
b.close()
