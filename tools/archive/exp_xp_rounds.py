"""Host count (no GPU) of scanner-expansion work per 1 KiB iteration: the
FDR4 first stage restated in numpy (tests/test_cpu_oracle.py
_fdr4_candidates logic, per end and bucket) over 8 MiB of the cfg-4 corpus;
per 64-lane iteration the candidate bits and R = the most bits any lane
holds (the rounds of one-bit-per-lane extraction).  Split pass 0 shown for
50k.  python tools/exp_xp_rounds.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

for nl in (20000, 50000):
    lits = bench.make_literals(nl, seed=12)
    blob = vsa.hwlm_build(lits)
    data = bench.make_corpus(8 << 20, lits, seed=5, plant_every=64 << 10)
    for par in ([-1] if nl == 20000 else [-1, 0]):
        T, _ = vsa.derive_fdr4_pass(blob, par)
        b = np.frombuffer(bytes(data), np.uint8).astype(np.uint64)
        n = len(b)
        p1 = np.concatenate([np.zeros(1, np.uint64), b[:-1]])
        p2 = np.concatenate([np.zeros(2, np.uint64), b[:-2]])
        key = ((p1 & np.uint64(0x7f)) | ((b & np.uint64(0x7f)) << np.uint64(7)) |
               ((p2 & np.uint64(1)) << np.uint64(14)))
        x = T[key.astype(np.int64)].astype(np.uint64)
        conf = np.zeros(n, np.uint64)
        for f in range(4):
            conf[f:] |= (x[:n - f] >> np.uint64(8 * f)) & np.uint64(0xff)
        cand = (~conf) & np.uint64(0xff)
        if par >= 0:
            cand[(b & np.uint64(1)) != np.uint64(par)] = 0
        bits = np.unpackbits(cand.astype(np.uint8)[:, None], axis=1).sum(axis=1)
        it = bits.reshape(-1, 16).sum(axis=1).reshape(-1, 64)
        R = it.max(axis=1)
        print("lits %d pass %d: %.2e bits/B, %.1f bits per iteration, mean R %.2f, R histogram %s"
              % (nl, par, bits.sum() / n, it.sum(axis=1).mean(), R.mean(),
                 np.bincount(R)[:8].tolist()))
