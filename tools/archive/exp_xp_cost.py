"""Where a large set's time goes (scanner expansion, runtime.hip use_xp):
cfg-4-shaped 4 GiB corpus (4 x 1 GiB blocks), kernel ms per setting, each
on a fresh database (settings are read at load / launch): the default;
VSA_DEBUG_FLAGS=8 (candidates found, none expanded or pushed: the scan's
own cost); 1 / 2 / 3 confirm waves with expansion on; expansion off.
  python tools/exp_xp_cost.py [lits ...]"""
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
sizes = [int(x) for x in (sys.argv[1:] or ["20000"])]
settings = [{}, {"VSA_DEBUG_FLAGS": "8", "VSA_NCONF": "2", "VSA_XP": "1"},
            {"VSA_NCONF": "1", "VSA_XP": "1"}, {"VSA_NCONF": "2", "VSA_XP": "1"},
            {"VSA_NCONF": "3", "VSA_XP": "1"}, {"VSA_NCONF": "2", "VSA_XP": "0"}]
rounds = 2
if os.environ.get("XP_COST_QUICK"):  # the default setting only, one round (library A/B)
    settings, rounds = [{}], 1
for nl in sizes:
    lits = bench.make_literals(nl, seed=12)
    blob = vsa.hwlm_build(lits)
    data = bench.make_corpus_device(torch, 0, n, n, lits, 5, 64 << 10, torch.device("cuda", 0))
    torch.cuda.synchronize()
    for rnd in range(rounds):
        for st in settings:
            for k, v in st.items():
                os.environ[k] = v
            db = vsa.Database(ctx, blob)
            ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)
            ks = []
            for i in range(12):
                m = ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)
                ks.append(ctx.kernel_ms())
            print(json.dumps({"lits": nl, "lib": os.environ.get("VSA_LIB_VARIANT", "default"),
                              "setting": st, "split": db.split, "round": rnd,
                              "kernel_ms": round(float(np.mean(ks[4:])), 4),
                              "candidates": int(ctx.candidates()), "matches": int(m)}),
                  flush=True)
            db.close()
            for k in st:
                os.environ.pop(k)
    del data
    torch.cuda.empty_cache()
