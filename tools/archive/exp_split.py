"""Split passes A/B (VSA_SPLIT=0 / 1 at database load, runtime.hip
split_passes) over large literal sets: cfg-4-shaped 4 GiB corpus (4 x 1 GiB
blocks), kernel ms = mean of the last 2/3 of the launches per setting (after
one launch that sets the confirm-wave count), settings interleaved twice;
the match count must agree.  EXTRA="VSA_NCONF=3,VSA_XP=1" adds a setting
(split on) with those variables.  One JSON line per (lits, setting, round).
  python tools/exp_split.py [lits ...]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

ctx = vsa.Context(0)
n = 4 << 30
bl = n // 4
sizes = [int(x) for x in (sys.argv[1:] or ["20000", "30000", "50000"])]
settings = [{"VSA_SPLIT": "0"}, {"VSA_SPLIT": "1"}]
for ex in [x for x in os.environ.get("EXTRA", "").split(";") if x]:
    d = {"VSA_SPLIT": "1"}
    d.update(dict(kv.split("=") for kv in ex.split(",")))
    settings.append(d)
for nl in sizes:
    lits = bench.make_literals(nl, seed=12)
    blob = vsa.hwlm_build(lits)
    data = bench.make_corpus_device(torch, 0, n, n, lits, 5, 64 << 10, torch.device("cuda", 0))
    torch.cuda.synchronize()
    counts = set()
    for rnd in range(2):
        for st in settings:
            for k, v in st.items():
                os.environ[k] = v
            db = vsa.Database(ctx, blob)
            ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)
            ks = []
            launches = 24 if nl < 50000 else 9
            for i in range(launches):
                m = ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)
                ks.append(ctx.kernel_ms())
            counts.add(m)
            print(json.dumps({"lits": nl, "setting": st, "split": db.split, "round": rnd,
                              "kernel_ms": round(float(np.mean(ks[launches // 3:])), 4),
                              "candidates": int(ctx.candidates()), "matches": int(m)}),
                  flush=True)
            db.close()
            for k in st:
                os.environ.pop(k)
    assert len(counts) == 1, counts
    del data
    torch.cuda.empty_cache()
