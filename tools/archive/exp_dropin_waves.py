"""Where one small drop-in scan's time goes: the wave log (VSA_DEBUG_FLAGS
4096 | 8192) of a hwlmExec call on `bytes` of the cfg-4 corpus: kernel entry
(before the table staging), each scanning wave's start / end, the confirm
wave's end, in us from the kernel entry.  Usage: exp_dropin_waves.py [bytes]"""
import ctypes
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(4096 | 8192)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 10
lits = bench.make_literals(5000, seed=12)
blob = vsa.hwlm_build(lits)
data = bench.make_corpus(1 << 20, lits, seed=5, plant_every=64 << 10)
buf = np.ascontiguousarray(data[:size])
log = torch.zeros(1024 * 16 * 8, dtype=torch.int64, device="cuda")
vsa.lib.vsa_set_wave_log.argtypes = [ctypes.c_void_p]
vsa.lib.vsa_set_wave_log(log.data_ptr())
torch.cuda.synchronize()


@vsa.HWLMCallback
def cb(end, id_, scratch):
    return vsa.HWLM_ALL_GROUPS


vsa.hwlm_register(blob)
for rep in range(6):
    log.zero_()
    torch.cuda.synchronize()
    assert vsa.lib.hwlmExec(blob.ptr, buf.ctypes.data, size, 0, cb, None,
                            vsa.HWLM_ALL_GROUPS) == 0
    torch.cuda.synchronize()
    L = log.view(-1, 8).cpu().numpy().astype(np.int64)
    L = L[L[:, 0] != 0]
    conf = (L[:, 2] == 1) & (L[:, 3] == 0) & (L[:, 4] == 0) & (L[:, 7] == 0)
    scan = ~conf
    entries = np.concatenate([L[scan, 7], L[conf, 0]])
    t0 = entries.min()

    def us(v):
        return (v - t0) / 100.0

    line = "bytes %d: scanning waves %d" % (size, scan.sum())
    if scan.any():
        line += "; entry spread %.2f us; first scan start %.2f us; scan ends %.2f-%.2f us; " \
                "segs %s" % (us(entries).max(), us(L[scan, 0]).min(), us(L[scan, 1]).min(),
                             us(L[scan, 1]).max(), list(L[scan, 2]))
    if conf.any():
        line += "; confirm end %.2f us" % us(L[conf, 1]).max()
    print(line, flush=True)
vsa.hwlm_unregister(blob)
