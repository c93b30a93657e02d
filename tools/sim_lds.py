#!/usr/bin/env python3
"""Host model of the FDR filter's LDS cost (no GPU): LDS-array cycles per
1 KiB wave iteration for the derived stride-1 table (runtime.hip
derive_fdr_table) under lookup schedules.

Layout as in kernels.hip lit_iter: lane l of a 1 KiB chunk looks up
positions p = 16 l + j - 1 (j = 0..15), key = vsa_fdr_key(b[p], b[p + 1]),
entry field k -> end p + k.  A ds_read_b64 is served per half-wave (32
lanes) over 32 bank pairs (entry index mod 32); its cost is the largest
number of distinct addresses on one bank pair among the ACTIVE lanes
(identical addresses broadcast; MI355X_MICROARCH.md §LDS), 0 when no lane
of the half is active.

Schedules: `all` (today: 16 lookups, every lane); `lvl2` (the 8 even j,
then the 8 odd j only in lanes where some end the lookup reaches is still
alive); `lvl3` (even j, then j = 1 mod 4, then j = 3 mod 4, each masked).
The filter result is the same for every schedule (a masked lookup only
touches dead ends).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def conf_from(E, pos_mask, n):
    """OR of field k of E[p] into end p + k for the lookups in pos_mask"""
    conf = np.zeros(n + 8, np.uint64)
    ps = np.nonzero(pos_mask)[0]
    for k in range(8):
        f = (E[ps] >> np.uint64(8 * k)) & np.uint64(0xFF)
        conf[ps + k] |= f  # ps + k distinct for fixed k
    return conf[:n]


def alive_of(conf):
    return ((~conf) & np.uint64(0xFF)) != 0


def reach_any(alive, n):
    """r[p] = any(alive[p .. p + 7])"""
    a = np.zeros(n + 8, bool)
    a[:n] = alive
    r = np.zeros(n, bool)
    for k in range(8):
        r |= a[k:k + n]
    return r


def half_cost(keys, active):
    """keys, active: (rows, 32) -> per-row max distinct addresses per bank pair"""
    k = np.where(active, keys, -1)
    k.sort(axis=1)
    uniq = (k >= 0) & np.concatenate([np.ones((k.shape[0], 1), bool), k[:, 1:] != k[:, :-1]],
                                     axis=1)
    bank = np.where(uniq, k & 31, 32)
    cnt = np.zeros((k.shape[0], 33), np.int32)
    rows = np.repeat(np.arange(k.shape[0]), 32)
    np.add.at(cnt, (rows, bank.ravel()), 1)
    return cnt[:, :32].max(axis=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=4)
    ap.add_argument("--lits", type=int, default=5000)
    args = ap.parse_args()
    import bench
    import vectorscan_amd as vsa
    lits = bench.make_literals(args.lits, seed=12)
    blob = vsa.hwlm_build(lits)
    T, kb, fb = vsa.derive_first_stage(blob)
    n = int(args.mib * (1 << 20)) & ~1023
    data = bench.make_corpus(n + 16, lits, seed=5, plant_every=64 << 10).astype(np.int64)
    # positions p = -1 .. n - 2 map to index p + 1
    b = np.concatenate([[0], data])
    K = (b[:n] & 0x7F) | ((b[1:n + 1] & 0x7F) << 7)  # key of position p = i - 1
    E = T[K]
    # end index: end e = p + k -> index p + 1 + k (ends shifted by one like p)
    j = np.arange(n) % 16
    even = (j % 2) == 0
    m1 = (j % 4) == 1
    m3 = (j % 4) == 3
    full = conf_from(E, np.ones(n, bool), n)
    c1 = conf_from(E, even, n)
    a1 = reach_any(alive_of(c1), n)
    c2 = c1 | conf_from(E, m1, n)
    a2 = reach_any(alive_of(c2), n)
    print("alive ends: after even %.4f, after +1mod4 %.4f, final %.6f" %
          (alive_of(c1).mean(), alive_of(c2).mean(), alive_of(full).mean()))
    sched = {
        "all": np.ones(n, bool),
        "lvl2": np.where(even, True, a1),
        "lvl3": np.where(even, True, np.where(m1, a1, a2)),
    }
    # rows: (kib, half, j): lanes 32 per half
    keys = K.reshape(-1, 2, 32, 16).transpose(0, 1, 3, 2).reshape(-1, 32)
    for name, act in sched.items():
        a = act.reshape(-1, 2, 32, 16).transpose(0, 1, 3, 2).reshape(-1, 32)
        cost = half_cost(keys, a)
        per_kib = cost.reshape(-1, 32).sum(axis=1)
        frac = a.mean()
        print("%-5s LDS cycles / KiB %.1f (min-2 model %.1f), active lanes %.3f" %
              (name, per_kib.mean(), np.maximum(cost, 1).reshape(-1, 32).sum(axis=1).mean(),
               frac))


if __name__ == "__main__":
    main()
