"""Schedule tail of the cfg-4 scan (VSA_DEBUG_FLAGS=2048 timestamps, 100 MHz):
first scanning-wave start, earliest and latest scanning-wave end, per launch."""
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(2048 | int(os.environ.get("EXTRA_DBG", "0")))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
seg = os.environ.get("VSA_SEG_MAX_KIB", "default")
dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctx, vsa.hwlm_build(lits))
total = int(gib * (1 << 30))
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
torch.cuda.synchronize()
offs = [i * bl for i in range(4)]
for i in range(25):
    ctx.scan_blocks(db, data.data_ptr(), offs, [bl] * 4)
    if i >= 20:
        c = ctx.debug_counters()
        t0, e0, e1 = (~c[8]) & (2**64 - 1), (~c[9]) & (2**64 - 1), c[10]
        w0 = (~c[11]) & (2**64 - 1)
        print("seg %s: kernel %.4f ms, waves end %.1f .. %.1f us after the first start "
              "(tail %.1f us), first workgroup done at %.1f us" %
              (seg, ctx.kernel_ms(), (e0 - t0) / 100, (e1 - t0) / 100, (e1 - e0) / 100,
               (w0 - t0) / 100), flush=True)
