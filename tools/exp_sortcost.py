"""Step-cost split for the cfg-4 bench workload (experiment, GPU box):
wall ms per scan_blocks call with and without the device match sort, next to
the scan kernel's own hipEvent time.  Quantifies the step-vs-kernel gap noted
in DESIGN.md section 5."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402
from bench import make_literals, make_corpus_device  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = vsa.Context(0)
    lits = make_literals(5000, seed=12)
    blob = vsa.hwlm_build(lits)
    db = vsa.Database(ctx, blob)
    n = 4 << 30
    data = make_corpus_device(torch, n, lits, seed=5, plant_every=64 << 10, device=dev)
    torch.cuda.synchronize()
    bl = n // 4
    offs = [i * bl for i in range(4)]
    lens = [bl] * 4
    out = {}
    for sort in (True, False, True, False):
        for _ in range(2):
            ctx.scan_blocks(db, data.data_ptr(), offs, lens, sort=sort)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        km = []
        for _ in range(10):
            nm = ctx.scan_blocks(db, data.data_ptr(), offs, lens, sort=sort)
            km.append(ctx.kernel_ms())
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / 10 * 1e3
        out.setdefault("sorted" if sort else "unsorted", []).append(
            {"wall_ms": round(el, 4), "kernel_ms": round(sum(km) / len(km), 4), "matches": nm})
    print(json.dumps(out), flush=True)
    db.close()
    ctx.close()


if __name__ == "__main__":
    main()
