"""bench.py's N > 1 path on the GPU, in the driver's GPU suite:
two fresh rank processes (bench.py --gpus 2 spawns them with
torch.multiprocessing before anything touches the GPU; no re-exec) share
cuda:0 over gloo (VSA_BENCH_BACKEND=gloo: one-GPU boxes cannot run RCCL
between two ranks on one device).  Each rank scans its stripe of a 64 MiB
corpus (4 blocks, 7-byte halo, report_lo), packs its sorted records on the
device (vsa_scan_pack), and the PackedGather collectives bring them to rank
0, which merges them in rank order.  bench.py's own parity check then
compares every block's merged (end, id) sequence with the oracle's callback
sequence element for element.  The RCCL branch itself stays unmeasured on
hardware here (the driver's 8-GPU node runs it)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus", [2, 3])
def test_gpu_bench_stripes_gloo(gpus):
    env = dict(os.environ)
    env["VSA_BENCH_BACKEND"] = "gloo"
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus),
           "--gib", "0.0625", "--blocks", "4", "--steps", "3", "--warmup", "1", "--no-cpu",
           "--no-e2e"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == gpus
    assert d["parity"] is True, p.stderr[-4000:]
    assert d["parity_bytes"] == 64 << 20
    assert d["matches"] > 0
    assert d["config"]["parallelism"] == "stripe%d" % gpus
