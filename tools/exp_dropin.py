"""Per-call cost of the drop-in hwlmExec (host buffer -> pinned staging ->
one DMA -> scan -> published count + records -> host sort -> replay through a
C callback) against the CPU path for the same call, per buffer size, for the
cfg-4 literal set: the break-even size of INTEGRATION.md's length threshold.

  GPU  unregistered blob (the whole blob compared with the cached copy per
       call) and registered (vsa_hwlm_register: no compare);
  CPU  the oracle's SSE2 port of the reference FDR loop (fdr.c:145-333), one
       thread, the same bytes and literal set (the reference SIMD build is
       not buildable here; SURVEY §6 measured it at 1.77 GB/s per core).

One JSON line per size; the last line names the break-even size."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import oracle  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
eng = vsa.engine_blob(blob)
data = bench.make_corpus(64 << 20, lits, seed=5, plant_every=64 << 10)
lib = vsa.lib
count = ctypes.c_uint64(0)


@vsa.HWLMCallback
def cb(end, id_, scratch):
    count.value += 1
    return vsa.HWLM_ALL_GROUPS


def per_call(fn, reps):
    for _ in range(3):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


rows = []
for size in [1 << 10, 4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20,
             64 << 20]:
    buf = np.ascontiguousarray(data[:size])
    ptr = buf.ctypes.data
    reps = max(5, min(300, (64 << 20) // size))

    def gpu():
        count.value = 0
        assert lib.hwlmExec(blob.ptr, ptr, size, 0, cb, None, vsa.HWLM_ALL_GROUPS) == 0

    t_unreg = per_call(gpu, reps)
    n_gpu = count.value
    vsa.hwlm_register(blob)
    t_reg = per_call(gpu, reps)
    vsa.hwlm_unregister(blob)
    creps = max(3, min(300, (16 << 20) // size))
    t_cpu = per_call(lambda: oracle.fdr_exec_simd(eng, buf), creps)
    st, m = oracle.fdr_exec_simd(eng, buf)
    row = {"bytes": size, "gpu_us": round(t_unreg * 1e6, 1),
           "gpu_registered_us": round(t_reg * 1e6, 1), "cpu_sse2_1t_us": round(t_cpu * 1e6, 1),
           "gpu_registered_GBps": round(size / t_reg / 1e9, 3),
           "cpu_GBps": round(size / t_cpu / 1e9, 3), "matches": n_gpu,
           "matches_equal": n_gpu == len(m)}
    rows.append(row)
    print(json.dumps(row), flush=True)
even = next((r["bytes"] for r in rows if r["gpu_registered_us"] <= r["cpu_sse2_1t_us"]), None)
print(json.dumps({"break_even_bytes": even,
                  "rule": "smallest size where the registered GPU call is no slower than "
                          "one CPU thread"}), flush=True)
