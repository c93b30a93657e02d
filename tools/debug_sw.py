"""Debug helper: ShortWritings (fdr.cpp:594) through the batch API, report
the first mismatching block per engine hint."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import vectorscan_amd as vsa
import oracle
from test_gpu_parity import batch_run
from test_cpu_oracle import load, build_or_none

ctx = vsa.Context(0)
spec = load("fdr_shortwritings.json")[0]
bufs = [bytes.fromhex(x) for x in spec["bufs"]]
pats = [bytes.fromhex(x) for x in spec["pats"]]
for hint in (0, 11, 17, 3, 9):
    bad = 0
    for g in range(0, len(pats), 32):
        group = pats[g:g + 32]
        lits = [vsa.HwlmLiteral(p, False, g + i) for i, p in enumerate(group)]
        blob = build_or_none(lits, hint)
        if blob is None:
            continue
        got = batch_run(ctx, blob, bufs)
        for bi, (b, m) in enumerate(zip(bufs, got)):
            st, mo = oracle.fdr_exec(vsa.engine_blob(blob), b)
            if m != mo:
                bad += 1
                if bad <= 3:
                    print("hint", hint, "group", g, "block", bi, "len", len(b), "data", b.hex())
                    print("   gpu   ", m)
                    print("   oracle", mo)
    print("hint", hint, "bad blocks", bad, flush=True)
