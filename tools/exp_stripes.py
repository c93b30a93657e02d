"""One GPU, the per-rank step of bench.py at N = 1, 2, 4, 8 (verdict r02
item 4): rank 0's windows of plan_corpus_stripes over the 4 GiB cfg-4
corpus (4 / 2 / 1 / 0.5 GiB), scanned as a rank's step does (a plan,
report_lo, sorted records, count read back), after a clock settle, then K
timed steps, both one step at a time ("sync") and pipelined over two
contexts as bench.py does ("pipe").  One JSON line per N and mode: step ms,
kernel ms, step - kernel.  The collectives are not part of this (one GPU):
they are what an N-rank run adds.  Modes pack2 / pack1: the pipelined step
with the records packed into the collective buffer by a separate vsa_pack
launch / by the sort launch itself (vsa_scan_plan_pack); "side" adds a
stand-in for the collective (a one-workgroup copy of the packed buffer's
header on another stream, after the scan) to show what the persistent grid does to it, with
EXP_RESERVE=n CUs left free (vsa_ctx_set_reserved_cus); EXP_STREAMS=2 puts
the second context on its own stream.
EXP_RANKS / EXP_MODES (comma lists) limit the rows; EXP_TIMING=n times every
n-th launch of the pipelined modes (bench.py uses 4).
  python tools/exp_stripes.py [steps] [warmup]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402
from vectorscan_amd import stripe  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
ctxs = [vsa.Context(0)]
# EXP_RESERVE=n: the grid leaves n CUs free (measured, not used by bench.py)
ctxs[0].reserve_cus(int(os.environ.get("EXP_RESERVE", "0")))
# EXP_STREAMS=2: the second context on a stream of its own, so a scan can
# start on the CUs the previous one's last workgroups leave (not bench.py's)
ctxs.append(vsa.Context(0) if os.environ.get("EXP_STREAMS") == "2"
            else vsa.Context(share_stream_with=ctxs[0]))
# EXP_TIMING=n: the pipelined modes time every n-th launch per context (as
# bench.py); their kernel_ms averages the timed ones
t_every = int(os.environ.get("EXP_TIMING", "1"))
lits = bench.make_literals(5000, seed=12)
db = vsa.Database(ctxs[0], vsa.hwlm_build(lits))
total = 4 << 30
bl = total // 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
torch.cuda.synchronize()
dptr = data.data_ptr()
ranks = [int(x) for x in os.environ.get("EXP_RANKS", "1,2,4,8").split(",")]
modes = os.environ.get("EXP_MODES", "sync,pipe,pack2,pack1,side").split(",")
for n in ranks:
    cuts, plan = stripe.plan_corpus_stripes(total, bl, n)
    wins = plan[0]
    offs = [w.wlo for w in wins]
    lens = [w.wlen for w in wins]
    rlos = [w.rlo for w in wins]
    plans = [c.plan(dptr, offs, lens, None, None, rlos) for c in ctxs]
    for _ in range(60):  # clock settle + warm
        ctxs[0].scan_plan(db, plans[0])
    cap = 1 << 16
    bufs = [torch.zeros(1 + cap + (cap + 1) // 2, dtype=torch.int64, device=dev) for _ in ctxs]
    side = torch.cuda.Stream()
    cstreams = [torch.cuda.ExternalStream(c.stream, device=dev) for c in ctxs]
    dsts = [torch.zeros_like(b) for b in bufs]
    evs = [torch.cuda.Event() for _ in ctxs]
    for mode in modes:
        ks, counts = [], []
        for c in ctxs:
            c.timing(1 if mode == "sync" else t_every)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "sync":
            for _ in range(steps):
                counts.append(ctxs[0].scan_plan(db, plans[0]))
                ks.append(ctxs[0].kernel_ms())
        elif mode == "side":
            # pack1 plus a stand-in for the collective: a copy of the packed
            # buffer on another stream that waits for the scan stream (as
            # RCCL's kernels wait on bench.py's), completed with the step;
            # with EXP_RESERVE=0 it queues behind the next scan's persistent
            # grid, with free CUs it runs beside it
            for k in range(steps):
                c, pl, bf = ctxs[k % 2], plans[k % 2], bufs[k % 2]
                c.scan_plan_pack(db, pl, bf.data_ptr(), cap)
                side.wait_stream(cstreams[k % 2])
                with torch.cuda.stream(side):
                    # one 64-byte copy: a one-workgroup kernel, the size of
                    # RCCL's small-message collective kernels
                    dsts[k % 2][:8].copy_(bf[:8])
                evs[k % 2].record(side)
                if k:
                    counts.append(ctxs[(k - 1) % 2].scan_wait())
                    evs[(k - 1) % 2].synchronize()
                    ks.append(ctxs[(k - 1) % 2].kernel_ms())
            counts.append(ctxs[(steps - 1) % 2].scan_wait())
            evs[(steps - 1) % 2].synchronize()
            ks.append(ctxs[(steps - 1) % 2].kernel_ms())
            assert int(dsts[(steps - 1) % 2][0].item()) == counts[-1]  # the header
        elif mode.startswith("pack"):
            # a rank's step as bench.py's N > 1 path queues it, minus the
            # collectives: pipelined scans whose records go into the
            # collective buffer -- pack2 by a vsa_pack launch behind the
            # sort (scan_plan + scan_pack, round 5), pack1 by the sort itself
            # (scan_plan_pack)
            for k in range(steps):
                c, pl, bf = ctxs[k % 2], plans[k % 2], bufs[k % 2]
                if mode == "pack2":
                    c.scan_plan(db, pl, asynchronous=True)
                    c.scan_pack(bf.data_ptr(), cap)
                else:
                    c.scan_plan_pack(db, pl, bf.data_ptr(), cap)
                if k:
                    counts.append(ctxs[(k - 1) % 2].scan_wait())
                    ks.append(ctxs[(k - 1) % 2].kernel_ms())
            counts.append(ctxs[(steps - 1) % 2].scan_wait())
            ks.append(ctxs[(steps - 1) % 2].kernel_ms())
            hdr = [int(b[0].item()) for b in bufs]
            assert all(h == counts[-1] for h in hdr), (hdr, counts[-1])
        else:
            for k in range(steps):
                ctxs[k % 2].scan_plan(db, plans[k % 2], asynchronous=True)
                if k:
                    counts.append(ctxs[(k - 1) % 2].scan_wait())
                    ks.append(ctxs[(k - 1) % 2].kernel_ms())
            counts.append(ctxs[(steps - 1) % 2].scan_wait())
            ks.append(ctxs[(steps - 1) % 2].kernel_ms())
        torch.cuda.synchronize()
        st = (time.perf_counter() - t0) / steps * 1e3
        ks = [x for x in ks if x >= 0] or [float("nan")]
        k = sum(ks) / len(ks)
        print(json.dumps({"lib": os.environ.get("VSA_LIB_VARIANT", ""),
                          "streams": os.environ.get("EXP_STREAMS", "1"), "ranks": n, "mode": mode, "rank_bytes": cuts[1] - cuts[0],
                          "windows": len(wins), "step_ms": round(st, 4),
                          "kernel_ms": round(k, 4), "overhead_us": round((st - k) * 1e3, 1),
                          "matches": counts[-1], "counts_equal": len(set(counts)) == 1}),
              flush=True)
    for pl in plans:
        pl.close()
