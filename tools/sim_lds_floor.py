"""Host model (no GPU) of the FDR sweep's LDS-array cycles per 1 KiB wave
iteration for the shipped two-level FDR4 schedule and the alternatives the
round-5 verdict named, priced with the issue probe's measured random-read
costs (profiles/r05/probe_issue.jsonl, LDS cycles per wave instruction per
CU at a given share of active lanes):

    ds_read_b32: 2.344 (0 %), 4.149 (28 %), 5.413 (50 %), 7.066 (100 %)
    ds_read_b64: 2.393 (0 %), 4.238 (28 %), 5.451 (50 %), 7.023 (100 %)

(interpolated linearly between the measured shares).  Lane l of a wave
holds bytes [16 l, 16 l + 16) of the 1 KiB chunk and looks up its 16
positions j; a lookup at position p ORs field f of its entry into end
p + f.  A later level looks a position up only in lanes where a 4-end conf
dword its fields reach still has a live end (the shipped gate, kernels.hip
fdr4_conf); a gated-off lane costs no bank but its instruction still
issues.  Designs:

  A  shipped: FDR4 u32 (15-bit key b[p-2] bit 0 + 7 + 7, 4 fields), level 1
     = even j (8 reads), level 2 = odd j gated (8 EXEC-masked reads)
  B  FDR4 u32, level 1 = j = 0 mod 4, level 2 = j = 2 mod 4, level 3 = odd j
  C  8-field u64 (14-bit key 7 + 7 of b[p-1], b[p]: the 128 KiB that fits),
     level 1 = j = 0 mod 4, level 2 = j = 2 mod 4, level 3 = odd j
  D  8-field u64, level 1 = even j, level 2 = odd j
  E  A with level 2 split per slot (exact per-position gate; more VALU,
     measured slower in round 5: r05zg)

Prints, per design, modeled LDS cycles per KiB iteration (the shipped
kernel's PMC gives 97 per KiB per CU for all LDS instructions, 16 of 17.2
of them lookups), the reads per lane, and the final first-stage candidate
ends per byte (what reaches the confirm).  python tools/sim_lds_floor.py
[literals] [MiB]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

PROBE = {4: ([0.0, 0.28, 0.5, 1.0], [2.344, 4.149, 5.413, 7.066]),
         8: ([0.0, 0.28, 0.5, 1.0], [2.393, 4.238, 5.451, 7.023])}

nl = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
mib = float(sys.argv[2]) if len(sys.argv) > 2 else 8
lits = bench.make_literals(nl, seed=12)
blob = vsa.hwlm_build(lits)
n = int(mib * (1 << 20)) & ~1023
b = bench.make_corpus(n, lits, seed=5, plant_every=64 << 10).astype(np.int64)
p1 = np.concatenate([[0], b[:-1]])
p2 = np.concatenate([[0, 0], b[:-2]])
T4 = vsa.derive_fdr4_table(blob, 15).astype(np.uint64)
X4 = T4[(p1 & 0x7F) | ((p2 & 1) << 7) | ((b & 0x7F) << 8)]      # vsa_fdr4_key


def derive_fdr8(blob):
    """the 8-field table of rounds 1-2 (u64: 8 ends x 8 buckets keyed by 7 +
    7 bits of b[p-1], b[p]), derived like runtime.hip derive_fdr4_table from
    the blob's own LitInfo records (fdr_confirm.h:57-83: FDRConfirm 32 B,
    litIndex u32[1 << nBits], LitInfo {v, msk, groups, id, size, flags,
    next} 32 B); bit f * 8 + b clear = bucket b may end f bytes later"""
    import ctypes
    eng = vsa.engine_blob(blob)
    rd = lambda a, n: int.from_bytes(ctypes.string_at(a, n), "little")  # noqa: E731
    cbase = eng + rd(eng + 16, 4)
    T = np.full(1 << 14, (1 << 64) - 1, np.uint64)
    always = 0
    for bk in range(8):
        off = rd(cbase + 4 * bk, 4)
        if not off:
            continue
        fc = cbase + off
        nbits = rd(fc + 16, 4)
        li = np.frombuffer(ctypes.string_at(fc + 32, 4 << nbits), np.uint32)
        offs = set()
        for o in li[li != 0].tolist():
            while True:
                offs.add(o)
                if not rd(fc + o + 30, 1):
                    break
                o += 32
        for o in offs:
            v, m = rd(fc + o, 8), rd(fc + o + 8, 8)

            def cand(back):
                mm = (m >> (8 * (7 - back))) & 0xFF
                vv = (v >> (8 * (7 - back))) & mm
                return np.unique(np.array([x & 0x7F for x in range(256) if x & mm == vv]))
            for f in range(8):
                bit = 1 << (f * 8 + bk)
                c0, c1 = cand(f), cand(f + 1) if f < 7 else np.arange(128)
                if len(c0) * len(c1) >= 1 << 14:
                    always |= bit
                    continue
                keys = (c1[:, None] | (c0[None, :] << 7)).ravel()
                T[keys] &= np.uint64(~bit & ((1 << 64) - 1))
    return T & np.uint64(~always & ((1 << 64) - 1))


T8 = derive_fdr8(blob)
X8 = T8[(p1 & 0x7F) | ((b & 0x7F) << 7)]                           # key (b[p-1], b[p])
j = np.arange(n) % 16
FULL = 0xFF


def conf_add(conf, X, sel, F):
    ps = np.nonzero(sel)[0]
    for f in range(F):
        e = ps + f
        ok = e < n
        conf[e[ok]] |= (X[ps[ok]] >> np.uint64(8 * f)) & np.uint64(FULL)


def alive(conf):
    return ((~conf) & np.uint64(FULL)) != 0


def gate(al, F):
    """position p may still matter: a live end in a conf dword p's fields
    reach (dwords floor(p / 4) .. floor((p + F - 1) / 4))"""
    dw = al.reshape(-1, 4).any(axis=1)
    nd = len(dw)
    g = np.zeros(n, bool)
    d0 = np.arange(n) // 4
    for k in range((F + 6) // 4 + 1):
        dk = d0 + k
        lim = (np.arange(n) + F - 1) // 4
        use = (dk <= lim) & (dk < nd)
        g[use] |= dw[dk[use]]
    return g


def cost(active, sel, width):
    """LDS cycles per KiB iteration of one wave: each position j of the
    level (sel) is one wave instruction over 64 lanes, priced by its share
    of active lanes (an instruction with every lane gated off still issues)"""
    a = active.reshape(-1, 64, 16)            # (chunk, lane, j)
    share = a.mean(axis=1)                     # (chunk, j)
    xs, ys = PROBE[width]
    c = np.interp(share, xs, ys)
    issued = sel[:16]                          # the level's j (periodic in 16)
    return float(c[:, issued].sum(axis=1).mean()), float(a.sum(axis=2).mean())


def run(name, X, F, width, levels):
    conf = np.zeros(n, np.uint64)
    tot, reads = 0.0, 0.0
    act = None
    for li, sel in enumerate(levels):
        if li == 0:
            act = sel.copy()
        else:
            act = sel & gate(alive(conf), F)
        c, r = cost(act, sel, width)
        tot += c
        reads += r
        conf_add(conf, X, act, F)
    cand = np.unpackbits((~conf & np.uint64(FULL)).astype(np.uint8)).sum() / n
    print("%s  LDS cycles/KiB %5.1f  reads/lane %5.2f  candidate bits/byte %.2e"
          % (name, tot, reads, cand), flush=True)
    return tot


even, odd = j % 2 == 0, j % 2 == 1
m0, m2 = j % 4 == 0, j % 4 == 2
print("%d literals, %.0f MiB of cfg-4 text" % (nl, mib))
a = run("A shipped FDR4 even|odd      ", X4, 4, 4, [even, odd])
run("B FDR4 0mod4|2mod4|odd       ", X4, 4, 4, [m0, m2, odd])
run("C 8-field 0mod4|2mod4|odd    ", X8, 8, 8, [m0, m2, odd])
run("D 8-field even|odd           ", X8, 8, 8, [even, odd])
# E: the exact per-slot gate (each odd position gated by its own 4 ends)
conf = np.zeros(n, np.uint64)
conf_add(conf, X4, even, 4)
al = alive(conf)
ex = np.zeros(n, bool)
for f in range(4):
    ex[:n - f] |= al[f:]
c1, r1 = cost(even, even, 4)
c2, r2 = cost(odd & ex, odd, 4)
print("E FDR4 even|odd exact gate   LDS cycles/KiB %5.1f  reads/lane %5.2f  (A: %5.1f)"
      % (c1 + c2, r1 + r2, a))
# F: a conflict-free level 0 in front of A -- the only table small enough
# for 32 bank-private copies beside the 128 KiB one (<= 160 entries x 4 B x
# 32 copies <= 20 KiB): 7 bits of b[p] alone, buckets merged per field.
# Its ends live, and A's level-1 lanes it could gate off:
T0 = np.zeros(128, np.uint64)
for x in range(128):
    sel = (b & 0x7F) == x
    if sel.any():
        merged = np.bitwise_and.reduce(X4[sel])   # fields live for some key of byte x
        T0[x] = merged
conf0 = np.zeros(n, np.uint64)
conf_add(conf0, T0[b & 0x7F], np.ones(n, bool), 4)
al0 = alive(conf0)
print("F level-0 byte filter (conflict-free, 16 reads at 2.342): ends live %.3f, "
      "A's level-1 lanes it gates off %.3f" % (al0.mean(),
      1 - gate(al0, 4).reshape(-1, 64, 16)[:, :, ::2].any(axis=2).mean()))
