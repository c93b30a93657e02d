"""bench.py's N > 1 path on the GPU, in the driver's GPU suite:
two fresh rank processes (bench.py --gpus 2 spawns them with
torch.multiprocessing before anything touches the GPU; no re-exec) share
cuda:0 over gloo (VSA_BENCH_BACKEND=gloo: one-GPU boxes cannot run RCCL
between two ranks on one device).  Each rank scans its stripe of a 64 MiB
corpus (4 blocks, 7-byte halo, report_lo), packs its sorted records on the
device (vsa_scan_pack), and the PackedGather collectives bring them to rank
0, which merges them in rank order.  bench.py's own parity check then
compares every block's merged (end, id) sequence with the oracle's callback
sequence element for element.

test_gpu_bench_rccl_world1 runs the RCCL branch itself on the one GPU:
bench.py --dist opens a world-size-1 "nccl" process group in a fresh process
(RCCL, device_id = cuda:0) and sends every step's records through the same
PackedGather all-gather + gather as the N > 1 run, on device tensors; parity
is checked on the gathered records."""
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


def test_gpu_bench_rccl_world1():
    env = dict(os.environ)
    env.pop("VSA_BENCH_BACKEND", None)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist", "--gib", "0.0625",
           "--blocks", "4", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-e2e"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["exchange"] == "rccl"
    assert d["parity"] is True, p.stderr[-4000:]
    assert d["parity_bytes"] == 64 << 20 and d["matches"] > 0
    # the read-ceiling probe ran on the same buffer
    r = d["roofline"]
    assert r["peak_measured"] and 1000 < r["peak_measured"] < 9000
