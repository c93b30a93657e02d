"""Host simulation of the FDR4 sweep's level-1 position pattern (no GPU):
with the engine's own 4-field table (vsa.derive_fdr4_table) over 8 MiB of
cfg-4 text, the share of ends still live after level 1 alone, of conf dwords
with a live end, and of (lane, dword) pairs the level-2 gate passes
(kernels.hip fdr4_conf: dword w or w + 1 live).  Usage:
python tools/sim_level1.py [literals]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

nl = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
lits = bench.make_literals(nl, seed=12)
T = vsa.derive_fdr4_table(vsa.hwlm_build(lits), 15).astype(np.uint64)
n = 8 << 20
b = bench.make_corpus(n, lits, seed=5, plant_every=64 << 10).astype(np.uint64)
p1 = np.concatenate([np.zeros(1, np.uint64), b[:-1]])
p2 = np.concatenate([np.zeros(2, np.uint64), b[:-2]])
key = ((p1 & np.uint64(0x7F)) | ((p2 & np.uint64(1)) << np.uint64(7)) |
       ((b & np.uint64(0x7F)) << np.uint64(8)))
X = T[key.astype(np.int64)]
pos = np.arange(n)


def conf_of(sel):
    conf = np.zeros(n, np.uint64)
    xs = np.where(sel, X, np.uint64(0))
    for f in range(4):
        conf[f:] |= (xs[:n - f] >> np.uint64(8 * f)) & np.uint64(0xFF)
    return conf


live_all = ((~conf_of(np.ones(n, bool))) & np.uint64(0xFF)) != 0
print("%d literals, all 16 positions: live ends %.3e" % (nl, live_all.mean()))
for name, pp in (("even", [0, 2]), ("01", [0, 1]), ("03", [0, 3]), ("12", [1, 2]), ("23", [2, 3])):
    live1 = ((~conf_of(np.isin(pos % 4, pp))) & np.uint64(0xFF)) != 0
    lw = live1.reshape(-1, 4).any(axis=1)
    gate = lw | np.concatenate([lw[1:], [True]])
    print("level 1 = positions %-4s mod 4: live ends %.4f, live dwords %.3f, level-2 gate %.3f"
          % (name, live1.mean(), lw.mean(), gate.mean()))
