#!/usr/bin/env python3
"""Host simulation of FDR first-stage designs (no GPU): candidate rates of a
derived first stage on the cfg-4 literal set over a synthetic corpus sample.

A design is: lookups at positions p with p % stride == phase; the key of a
lookup is a bit-field fold of the bytes at p + o for o in `key_offs`
(`key_bits[i]` low bits of each byte); the entry holds one 8-bucket field
per end offset d in `ends` (end e = p + d).  End e, bucket b is a candidate
when every lookup reaching it has bit b clear (the table is derived from the
blob's own LitInfo records, like runtime.hip derive_fdr_table, so it is a
no-false-negative filter for any design).

Usage: python tools/sim_filter.py [--mib 16] [--lits 5000]
"""
import argparse
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lit_records(blob_bytes):
    """(v, msk, bucket) of every LitInfo of an FDR blob (fdr_confirm.h:57-83)"""
    eng = 192
    conf = eng + struct.unpack_from("<I", blob_bytes, eng + 16)[0]
    out = []
    for b in range(8):
        off = struct.unpack_from("<I", blob_bytes, conf + 4 * b)[0]
        if not off:
            continue
        fc = conf + off
        nbits = struct.unpack_from("<I", blob_bytes, fc + 16)[0]
        seen = set()
        for h in range(1 << nbits):
            o = struct.unpack_from("<I", blob_bytes, fc + 32 + 4 * h)[0]
            while o and o not in seen:
                seen.add(o)
                v, msk = struct.unpack_from("<QQ", blob_bytes, fc + o)
                nxt = blob_bytes[fc + o + 30]
                out.append((v, msk, b))
                if not nxt:
                    break
                o += 32
    return out


def byte_sets(v, m, bits):
    """values of the low `bits` bits of a byte consistent with (x & m) == v"""
    mask = (1 << bits) - 1
    xs = np.arange(256)
    ok = (xs & m) == (v & m)
    return np.unique(xs[ok] & mask)


def build_table(recs, key_offs, key_bits, ends):
    nbits = sum(key_bits)
    T = np.full(1 << nbits, np.uint64(0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    shifts = np.cumsum([0] + list(key_bits[:-1]))
    for v, msk, b in recs:
        for fi, d in enumerate(ends):
            bit = np.uint64(1 << (fi * 8 + b))
            # key byte i sits at p + o = e - d + o: literal byte index
            # 7 - (d - o) counted from the start of the 8-byte window
            keys = np.zeros(1, dtype=np.int64)
            for o, kb, sh in zip(key_offs, key_bits, shifts):
                back = d - o  # bytes before the end
                if 0 <= back <= 7:
                    mb = (msk >> (8 * (7 - back))) & 0xFF
                    vb = (v >> (8 * (7 - back))) & 0xFF
                else:
                    mb, vb = 0, 0
                vals = byte_sets(vb, mb, kb).astype(np.int64) << int(sh)
                keys = (keys[:, None] | vals[None, :]).ravel()
            T[keys] &= ~bit
    return T


def conf_of(data, T, key_offs, key_bits, ends, stride, phase):
    """per-end 8-bucket dead bits of one table design"""
    n = len(data)
    shifts = np.cumsum([0] + list(key_bits[:-1]))
    pad = 16
    buf = np.zeros(n + 2 * pad, dtype=np.int64)
    buf[pad:pad + n] = data
    pos = np.arange(n)
    lk = pos[(pos % stride) == phase]
    key = np.zeros(len(lk), dtype=np.int64)
    for o, kb, sh in zip(key_offs, key_bits, shifts):
        key |= (buf[lk + o + pad] & ((1 << kb) - 1)) << int(sh)
    E = T[key]
    conf = np.zeros(n + 16, dtype=np.uint64)
    for fi, d in enumerate(ends):
        f = (E >> np.uint64(8 * fi)) & np.uint64(0xFF)
        e = lk + d
        ok = (e >= 0) & (e < n)
        conf[e[ok]] |= f[ok]
    return conf[:n]


def simulate(data, T, key_offs, key_bits, ends, stride, phase):
    n = len(data)
    shifts = np.cumsum([0] + list(key_bits[:-1]))
    pad = 16
    buf = np.zeros(n + 2 * pad, dtype=np.int64)
    buf[pad:pad + n] = data
    pos = np.arange(n)
    lk = pos[(pos % stride) == phase]
    key = np.zeros(len(lk), dtype=np.int64)
    for o, kb, sh in zip(key_offs, key_bits, shifts):
        key |= (buf[lk + o + pad] & ((1 << kb) - 1)) << int(sh)
    E = T[key]
    conf = np.zeros(n + 16, dtype=np.uint64)
    for fi, d in enumerate(ends):
        f = (E >> np.uint64(8 * fi)) & np.uint64(0xFF)
        e = lk + d
        ok = (e >= 0) & (e < n)
        conf[e[ok]] |= f[ok]
    conf = conf[:n]
    # ends below 8 see fewer lookups; drop them from the count
    cand = (~conf) & np.uint64(0xFF)
    cand[:16] = 0
    bits = np.unpackbits(cand.astype(np.uint8)[:, None], axis=1).sum()
    lanes = (cand.reshape(-1, 16).max(axis=1) != 0).sum() if n % 16 == 0 else None
    return int(bits), int(np.count_nonzero(cand)), lanes


DESIGNS = {
    # current: stride 1, pair (p-1, p) 7+7 bits, ends p .. p+7
    "s1_pair77": dict(key_offs=(-1, 0), key_bits=(7, 7), ends=range(0, 8), stride=1),
    "s1_pair76": dict(key_offs=(-1, 0), key_bits=(7, 6), ends=range(0, 8), stride=1),
    "s1_pair67": dict(key_offs=(-1, 0), key_bits=(6, 7), ends=range(0, 8), stride=1),
    "s1_tri455": dict(key_offs=(-2, -1, 0), key_bits=(4, 5, 5), ends=range(0, 8), stride=1),
    "s1_tri545": dict(key_offs=(-2, -1, 0), key_bits=(5, 4, 5), ends=range(0, 8), stride=1),
    "s1_tri554": dict(key_offs=(-2, -1, 0), key_bits=(5, 5, 4), ends=range(0, 8), stride=1),
    "s1_skip77": dict(key_offs=(-2, 0), key_bits=(7, 7), ends=range(0, 8), stride=1),
    "s1_skip76": dict(key_offs=(-2, 0), key_bits=(7, 6), ends=range(0, 8), stride=1),
    "s1_gap377": dict(key_offs=(-3, 0), key_bits=(7, 7), ends=range(0, 8), stride=1),
    "s2_pair77": dict(key_offs=(-1, 0), key_bits=(7, 7), ends=range(0, 8), stride=2),
    "s2_tri554_back": dict(key_offs=(-2, -1, 0), key_bits=(5, 5, 4), ends=range(0, 8), stride=2),
    "s2_tri455_back": dict(key_offs=(-2, -1, 0), key_bits=(4, 5, 5), ends=range(0, 8), stride=2),
    "s2_tri554_ctr": dict(key_offs=(-1, 0, 1), key_bits=(5, 5, 4), ends=range(-1, 7), stride=2),
    "s2_tri455_ctr": dict(key_offs=(-1, 0, 1), key_bits=(4, 5, 5), ends=range(-1, 7), stride=2),
    "s2_tri545_ctr": dict(key_offs=(-1, 0, 1), key_bits=(5, 4, 5), ends=range(-1, 7), stride=2),
    "s2_tri664_ctr13": dict(key_offs=(-1, 0, 1), key_bits=(5, 5, 3), ends=range(-1, 7), stride=2),
    # 4-field (u32) entries with trigram keys: 2^15 x 4 B = 128 KiB
    "s1_tri555_f4": dict(key_offs=(-2, -1, 0), key_bits=(5, 5, 5), ends=range(0, 4), stride=1),
    "s1_tri465_f4": dict(key_offs=(-2, -1, 0), key_bits=(4, 6, 5), ends=range(0, 4), stride=1),
    "s1_tri564_f4": dict(key_offs=(-2, -1, 0), key_bits=(5, 6, 4), ends=range(0, 4), stride=1),
    "s1_tri456_f4": dict(key_offs=(-2, -1, 0), key_bits=(4, 5, 6), ends=range(0, 4), stride=1),
    "s1_pair78_f4": dict(key_offs=(-1, 0), key_bits=(7, 8), ends=range(0, 4), stride=1),
    "s1_tri177_f4": dict(key_offs=(-2, -1, 0), key_bits=(1, 7, 7), ends=range(0, 4), stride=1),
    "s1_tri276_f4": dict(key_offs=(-2, -1, 0), key_bits=(2, 7, 6), ends=range(0, 4), stride=1),
    "s1_tri366_f4": dict(key_offs=(-2, -1, 0), key_bits=(3, 6, 6), ends=range(0, 4), stride=1),
    "s1_tri375_f4": dict(key_offs=(-2, -1, 0), key_bits=(3, 7, 5), ends=range(0, 4), stride=1),
    "s1_tri555_f5": dict(key_offs=(-2, -1, 0), key_bits=(5, 5, 5), ends=range(0, 5), stride=1),
    # level 1 alone (even positions) of the two-level sweeps
    "s2_tri555_f4": dict(key_offs=(-2, -1, 0), key_bits=(5, 5, 5), ends=range(0, 4), stride=2),
    "s2_tri465_f4": dict(key_offs=(-2, -1, 0), key_bits=(4, 6, 5), ends=range(0, 4), stride=2),
    "s2_tri177_f4": dict(key_offs=(-2, -1, 0), key_bits=(1, 7, 7), ends=range(0, 4), stride=2),
    "s2_tri276_f4": dict(key_offs=(-2, -1, 0), key_bits=(2, 7, 6), ends=range(0, 4), stride=2),
    "s1_tri177_f3": dict(key_offs=(-2, -1, 0), key_bits=(1, 7, 7), ends=range(0, 3), stride=1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=16)
    ap.add_argument("--lits", type=int, default=5000)
    ap.add_argument("--designs", default=",".join(DESIGNS))
    args = ap.parse_args()
    import bench
    import vectorscan_amd as vsa
    lits = bench.make_literals(args.lits, seed=12)
    blob = vsa.hwlm_build(lits)
    recs = lit_records(blob.tobytes())
    n = int(args.mib * (1 << 20)) & ~15
    data = bench.make_corpus(n, lits, seed=5, plant_every=64 << 10).astype(np.int64)
    print("records %d, engine %d, %d bytes" % (len(recs), blob.engine_id, n))
    for name in args.designs.split(","):
        if "+" in name:
            # two tables AND-ed: an end is a candidate only if both pass it
            conf = np.zeros(n, dtype=np.uint64)
            for part in name.split("+"):
                d = DESIGNS[part]
                T = build_table(recs, d["key_offs"], d["key_bits"], list(d["ends"]))
                conf |= conf_of(data, T, d["key_offs"], d["key_bits"], list(d["ends"]),
                                d["stride"], 0)
            cand = (~conf) & np.uint64(0xFF)
            cand[:16] = 0
            bits = int(np.unpackbits(cand.astype(np.uint8)[:, None], axis=1).sum())
            lanes = int((cand.reshape(-1, 16).max(axis=1) != 0).sum())
            print("%-18s cand bits %9d (%.2e/B)  lanes %7s" % (name, bits, bits / n, lanes),
                  flush=True)
            continue
        d = DESIGNS[name]
        T = build_table(recs, d["key_offs"], d["key_bits"], list(d["ends"]))
        bits, ends, lanes = simulate(data, T, d["key_offs"], d["key_bits"], list(d["ends"]),
                                     d["stride"], 0)
        occ = 1.0 - np.mean([bin(int(x)).count("1") for x in T[:4096]]) / 64
        print("%-18s cand bits %9d (%.2e/B)  ends %8d  lanes %7s  occ %.3f" %
              (name, bits, bits / n, ends, lanes, occ), flush=True)


if __name__ == "__main__":
    main()
