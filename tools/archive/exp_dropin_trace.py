"""Drop-in hwlmExec calls of one size, repeated, for a rocprofv3 trace of what
one call issues (copies, kernels, HIP API calls).  Usage:
  rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --stats -d DIR -- \
      python tools/exp_dropin_trace.py [bytes] [calls]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 10
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
data = bench.make_corpus(1 << 20, lits, seed=5, plant_every=64 << 10)
buf = np.ascontiguousarray(data[:size])
count = ctypes.c_uint64(0)


@vsa.HWLMCallback
def cb(end, id_, scratch):
    count.value += 1
    return vsa.HWLM_ALL_GROUPS


vsa.hwlm_register(blob)
for _ in range(20):
    assert vsa.lib.hwlmExec(blob.ptr, buf.ctypes.data, size, 0, cb, None,
                            vsa.HWLM_ALL_GROUPS) == 0
t0 = time.perf_counter()
for _ in range(calls):
    assert vsa.lib.hwlmExec(blob.ptr, buf.ctypes.data, size, 0, cb, None,
                            vsa.HWLM_ALL_GROUPS) == 0
dt = (time.perf_counter() - t0) / calls
vsa.hwlm_unregister(blob)
print(f"bytes {size} calls {calls} per call {dt * 1e6:.1f} us matches/call "
      f"{count.value / (calls + 20):.1f}", flush=True)
