"""Scanner expansion A/B (VSA_XP=0 / 1, runtime.hip use_xp) over literal-set
sizes: cfg-4-shaped 4 GiB corpus (4 x 1 GiB blocks), kernel ms = mean of the
last 20 of 30 launches per setting, settings interleaved twice; the match
count must agree between settings.  One JSON line per (lits, xp, round)."""
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
sizes = [int(x) for x in (sys.argv[1:] or ["5000", "10000", "20000", "50000"])]
# NCONFS=1,2,3,4: scanner expansion on, one line per confirm-wave count
nconfs = [x for x in os.environ.get("NCONFS", "").split(",") if x]
for nl in sizes:
    lits = bench.make_literals(nl, seed=12)
    blob = vsa.hwlm_build(lits)
    db = vsa.Database(ctx, blob)
    data = bench.make_corpus_device(torch, 0, n, n, lits, 5, 64 << 10, torch.device("cuda", 0))
    torch.cuda.synchronize()
    ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)  # rate -> nconf
    counts = set()
    settings = [("1", nc) for nc in nconfs] if nconfs else [("0", None), ("1", None)]
    for rnd in range(2):
        for xp, nc in settings:
            os.environ["VSA_XP"] = xp
            if nc:
                os.environ["VSA_NCONF"] = nc
            ks = []
            launches = 30 if nl < 50000 else 8
            for i in range(launches):
                m = ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2 * bl, 3 * bl], [bl] * 4)
                ks.append(ctx.kernel_ms())
            counts.add(m)
            print(json.dumps({"lits": nl, "xp": int(xp), "nconf": nc, "round": rnd,
                              "kernel_ms": round(float(np.mean(ks[launches // 3:])), 4),
                              "matches": int(m)}), flush=True)
    os.environ.pop("VSA_XP")
    os.environ.pop("VSA_NCONF", None)
    assert len(counts) == 1, counts
    db.close()
    del data
    torch.cuda.empty_cache()
