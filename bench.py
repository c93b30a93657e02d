#!/usr/bin/env python3
"""bench.py — GB/s scanned, hsbench block mode, FDR 5k-literal database
(BASELINE.json configs[3], the north star's headline workload).

One step = one device launch that scans the rank's 4 GiB corpus as 4 x 1 GiB
blocks (each block one hwlmExec: hs_scan takes a 32-bit length,
src/hs_runtime.h:479) and leaves the confirmed matches sorted in reference
callback order in HBM; the match count is read back every step.  Inputs are
resident in HBM before the timed region.

Multi-GPU: one process per GPU (torch.distributed, RCCL); every rank scans
its own 4 GiB stripe of an N x 4 GiB corpus (weak scaling, no data-path
collective in the scan); each step ends with the RCCL gather of the ranks'
sorted match records to rank 0 (where the sequential host replay runs,
vectorscan_amd/stripe.py).  The timed region is bracketed by barrier +
synchronize and the max over ranks is reported.

Extra JSON fields: roofline (kernel-only HBM GB/s from hipEvents vs the 8 TB/s
MI355X peak), cpu_baseline (the scalar oracle on a bounded sample of the
same corpus, striped over the box's 16-thread CPU share), parity (GPU ==
oracle on a 64 MiB sample).
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PRINTABLE = np.arange(0x20, 0x7F, dtype=np.uint8)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def make_literals(n, seed=12, minlen=4, maxlen=8, nocase_frac=0.02):
    """cfg 4 literal set: printable, length 4-8, 2% nocase."""
    import vectorscan_amd as vsa
    r = random.Random(seed)
    lits = []
    for i in range(n):
        ln = r.randint(minlen, maxlen)
        s = bytes(r.randint(0x20, 0x7E) for _ in range(ln))
        lits.append(vsa.HwlmLiteral(s, r.random() < nocase_frac, i))
    return lits


def plant_plan(n, lits, seed, plant_every):
    """positions + literal bytes planted once per `plant_every` bytes."""
    r = np.random.default_rng(seed + 1)
    k = n // plant_every
    which = r.integers(0, len(lits), k)
    pos = np.arange(k, dtype=np.int64) * plant_every + r.integers(0, plant_every - 8, k)
    idx, val = [], []
    for p, w in zip(pos.tolist(), which.tolist()):
        s = lits[w].s
        idx.extend(range(p, p + len(s)))
        val.extend(s)
    return np.array(idx, np.int64), np.array(val, np.uint8)


def make_corpus(n, lits, seed=5, plant_every=64 << 10):
    """numpy version (tests): uniform printable bytes + planted literals."""
    r = np.random.default_rng(seed)
    data = PRINTABLE[r.integers(0, len(PRINTABLE), n, dtype=np.int64)]
    idx, val = plant_plan(n, lits, seed, plant_every)
    data[idx] = val
    return data


def make_corpus_device(torch, n, lits, seed, plant_every, device):
    """same construction on the GPU (torch is plumbing here)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    data = torch.empty(n, dtype=torch.uint8, device=device)
    chunk = 256 << 20
    for o in range(0, n, chunk):
        m = min(chunk, n - o)
        data[o:o + m] = torch.randint(0x20, 0x7F, (m,), dtype=torch.uint8, device=device,
                                      generator=g)
    idx, val = plant_plan(n, lits, seed, plant_every)
    data[torch.from_numpy(idx).to(device)] = torch.from_numpy(val).to(device)
    return data


def cpu_baseline(blob, sample_fn, threads, budget_s=10.0, chunk=256 << 20, max_bytes=2 << 30):
    """scalar oracle (oracle/oracle.c restatement of fdrExec) on a bounded
    sample: chunks of the rank-0 corpus, each striped over `threads` host
    threads (7-byte halo, counts only), until `budget_s` of wall time."""
    import oracle
    import vectorscan_amd as vsa
    eng = vsa.engine_blob(blob)
    done, t, i = 0, 0.0, 0
    while t < budget_s and done < max_bytes:
        buf = sample_fn(i * chunk, chunk)
        if len(buf) == 0:
            break
        t0 = time.perf_counter()
        oracle.fdr_count_mt(eng, buf, threads)
        t += time.perf_counter() - t0
        done += len(buf)
        i += 1
    return done, t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--gib", type=float, default=4.0, help="corpus GiB per rank")
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--lits", type=int, default=5000)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for cpu_baseline (default min(16, cpus))")
    args = ap.parse_args()

    import torch
    import vectorscan_amd as vsa
    from vectorscan_amd import stripe

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    ctx = vsa.Context(local)
    lits = make_literals(args.lits, seed=12)
    blob = vsa.hwlm_build(lits)
    db = vsa.Database(ctx, blob)

    n = int(args.gib * (1 << 30))
    data = make_corpus_device(torch, n, lits, seed=5 + 1000 * rank, plant_every=64 << 10,
                              device=dev)
    torch.cuda.synchronize()
    bl = n // args.blocks
    offs = [i * bl for i in range(args.blocks)]
    lens = [bl] * (args.blocks - 1) + [n - bl * (args.blocks - 1)]
    dptr = data.data_ptr()

    # N > 1: the step ends with the RCCL gather of every rank's sorted match
    # records to rank 0 (device to device, over xGMI), where the host replay
    # would run; the scan itself has no data-path collective.
    gcap = 1 << 21
    gkeys = torch.zeros(gcap, dtype=torch.int64, device=dev) if dist is not None else None
    gids = torch.zeros(gcap, dtype=torch.int32, device=dev) if dist is not None else None
    gathered = [0]

    def step():
        n_local = ctx.scan_blocks(db, dptr, offs, lens)
        if dist is None:
            return n_local
        if n_local > gcap:
            raise RuntimeError("bench: %d matches exceed the gather buffer" % n_local)
        ctx.results_to_device(gkeys.data_ptr(), gids.data_ptr(), gcap)
        ctx.sync()
        got = stripe.gather_to_root(dist, gkeys, gids, n_local)
        if got is not None:
            gathered[0] = int(got[0].shape[0])
        return n_local

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()

    kms = []
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nm = 0
    for _ in range(args.steps):
        nm = step()
        kms.append(ctx.kernel_ms())
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    el = t1 - t0
    ncand = int(ctx.candidates())  # of the last timed step
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        cnt = torch.tensor([nm], dtype=torch.int64, device=dev)
        dist.all_reduce(cnt)
        total_matches = int(cnt.item())
    else:
        total_matches = nm
    ms_step = el / args.steps * 1e3
    gbs = world * n / (el / args.steps) / 1e9

    out = None
    if rank == 0:
        kavg = float(np.mean(kms))
        alg_bytes = n + 16 * nm  # input once + one 16-B record per match
        achieved = alg_bytes / (kavg * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_fdr5k_4gib.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        # parity + CPU baseline on a bounded sample of block 0
        sample = 64 << 20

        def sample_fn(off, ln):
            ln = min(ln, bl - off)
            return data[off:off + ln].cpu().numpy()

        import oracle
        host = sample_fn(0, sample)
        st, m_o = oracle.fdr_exec(vsa.engine_blob(blob), host, cap=1 << 20)
        ns = ctx.scan_blocks(db, dptr, [0], [len(host)])
        res = ctx.results(ns)
        m_g = list(zip((res["key"] >> np.uint64(24)).tolist(), res["id"].tolist()))
        parity = (m_g == m_o)
        cpu = None
        if not args.no_cpu and world == 1:
            # the GPU box's CPU share is 16 threads (os.cpu_count() shows the
            # whole host there)
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            done, t = cpu_baseline(blob, sample_fn, threads, budget_s=args.cpu_budget)
            cpu = {"value": round(done / t / 1e9, 4), "unit": "GB/s", "cores": threads,
                   "kind": "port",
                   "sample": "%d MiB of rank-0 block 0, oracle/oracle.c fdrExec restatement "
                             "(scalar), %d threads over contiguous stripes" % (done >> 20, threads)}
        out = {
            "metric": "GB/s scanned (hsbench block mode), FDR 5k literals",
            "value": round(gbs, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform printable 0x20-0x7E, 1 planted literal / 64 KiB)",
            "config": {"workload": "cfg4: FDR %d literals len 4-8 (2%% nocase), %.0f GiB per "
                                   "GPU as %d blocks, engine id %s" %
                                   (args.lits, args.gib, args.blocks, blob.engine_id),
                       "global_bytes": world * n, "parallelism": "stripe%d" % world},
            "matches": total_matches,
            "gathered_to_rank0": gathered[0] if dist is not None else None,
            "confirm_candidates": ncand,
            "parity": parity,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel_ms": round(kavg, 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    db.close()
    ctx.close()


if __name__ == "__main__":
    main()
