"""Warm-up ramp of the cfg-4 scan (verdict r02 item 3): kernel time of every
launch from the first, for the FDR scan and for the class scan (a plain
HBM stream through another kernel) in one process, in the order given:
  python tools/exp_ramp.py lit,class,lit   -> one JSON line per phase
Each phase runs N back-to-back launches over the same 4 GiB corpus; a
ramp that both kernels show from process start is the platform (clocks),
one that only the literal scan shows is the scan's own state."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

phases = (sys.argv[1] if len(sys.argv) > 1 else "lit,class,lit").split(",")
n = int(os.environ.get("RAMP_N", "40"))
dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
total = 4 << 30
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
bm = torch.empty(total // 8, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
offs = [i * bl for i in range(4)]
cls = vsa.class_bitmap(b"<>\"'")
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t_start = time.perf_counter()
for ph in phases:
    ks = []
    for i in range(n):
        if ph == "lit":
            ctx.scan_blocks_ex(db, data.data_ptr(), offs, [bl] * 4)
            ks.append(round(ctx.kernel_ms(), 4))
        elif ph == "class":
            t0 = time.perf_counter()
            ctx.class_scan(cls, data.data_ptr(), total, bm.data_ptr())
            ks.append(round((time.perf_counter() - t0) * 1e3, 4))
        elif ph == "idle":
            time.sleep(0.5)
            break
    print(json.dumps({"phase": ph, "t_s": round(time.perf_counter() - t_start, 3),
                      "ms": ks}), flush=True)
