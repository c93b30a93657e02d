"""PCIe-inclusive rate of the drop-in hwlmExec (host buffer -> H2D -> scan ->
sort -> D2H -> replay through a C callback): latency and GB/s per buffer
size for the cfg-4 literal set, and the device-resident batch rate beside
it.  Writes one JSON line per size."""
import ctypes
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
data = bench.make_corpus(64 << 20, lits, seed=5, plant_every=64 << 10)
lib = vsa.lib
count = ctypes.c_uint64(0)


@vsa.HWLMCallback
def cb(end, id_, scratch):
    count.value += 1
    return vsa.HWLM_ALL_GROUPS


for size in [1 << 10, 4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20,
             64 << 20]:
    buf = np.ascontiguousarray(data[:size])
    ptr = buf.ctypes.data
    for _ in range(3):
        lib.hwlmExec(blob.ptr, ptr, size, 0, cb, None, vsa.HWLM_ALL_GROUPS)
    reps = max(5, min(200, (64 << 20) // size))
    t0 = time.perf_counter()
    for _ in range(reps):
        count.value = 0
        rc = lib.hwlmExec(blob.ptr, ptr, size, 0, cb, None, vsa.HWLM_ALL_GROUPS)
        assert rc == 0
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"bytes": size, "calls": reps, "us_per_call": round(dt * 1e6, 1),
                      "GBps": round(size / dt / 1e9, 3), "matches": count.value}), flush=True)
