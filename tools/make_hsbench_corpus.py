"""Synthetic hsbench inputs: an expression file of N pure literals (the
bench cfg-4 generator: printable, length 4-8, 2% caseless) and a corpus in
the CorpusBuilder.py sqlite schema (uniform printable bytes with planted
literals, cut into chunks, round-robin over streams).

    python tools/make_hsbench_corpus.py --out DIR --lits 5000 --bytes 1G \
        --chunk 16K --streams 64
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402
from vectorscan_amd import hsbench  # noqa: E402


def size(s):
    m = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(s[:-1]) * m[s[-1]] if s[-1] in m else int(s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--lits", type=int, default=5000)
    ap.add_argument("--bytes", default="256M")
    ap.add_argument("--chunk", default="16K")
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--mixed", action="store_true",
                    help="cfg-5-shaped set (bench.make_mixed_set): length 4-16, "
                         "flags i / H / L mixed, shared ids")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    if a.mixed:
        from vectorscan_amd import hs
        exprs, flags, ids = bench.make_mixed_set(a.lits, shared_ids=False)
        lits = [vsa.HwlmLiteral(e, False, i) for i, e in enumerate(exprs)]
        with open(os.path.join(a.out, "sigs"), "wb") as f:
            for e, fl, i in zip(exprs, flags, ids):
                fc = b"".join(c for c, bit in ((b"i", hs.FLAG_CASELESS),
                                               (b"H", hs.FLAG_SINGLEMATCH),
                                               (b"L", hs.FLAG_SOM_LEFTMOST)) if fl & bit)
                f.write(b"%d:/%s/%s\n" % (i, e, fc))
    else:
        lits = bench.make_literals(a.lits, seed=12)
        with open(os.path.join(a.out, "sigs"), "wb") as f:
            for l in lits:
                f.write(b"%d:/%s/%s\n" % (l.id, l.s, b"i" if l.nocase else b""))
    total, chunk = size(a.bytes), size(a.chunk)
    data = bench.make_corpus(total, lits, seed=a.seed, plant_every=64 << 10)
    chunks = [(k % a.streams, data[o:o + chunk].tobytes())
              for k, o in enumerate(range(0, total, chunk))]
    hsbench.write_corpus(os.path.join(a.out, "corpus.db"), chunks)
    print("wrote %d literals, %d chunks (%d bytes)" % (len(lits), len(chunks), total))


if __name__ == "__main__":
    main()
