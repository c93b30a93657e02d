#!/usr/bin/env python3
"""Confirm-wave phase profile (VSA_DEBUG_FLAGS=64): per-CU cycles spent
gathering / expanding / confirming / idle, and gather rounds, chunk
entries, expansion rounds, confirm batches, for the cfg3 Teddy sets and the
cfg4 FDR set (1 GiB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["VSA_DEBUG_FLAGS"] = os.environ.get("VSA_DEBUG_FLAGS", "64")


def main():
    import torch
    import bench
    import vectorscan_amd as vsa
    from tools.bench_configs import lits_printable
    ctx = vsa.Context(0)
    n = 1 << 30
    sets = [("teddy48", lits_printable(48, 55), 4096, 3),
            ("teddy64", lits_printable(64, 71), 4096, 3),
            ("fdr5k", bench.make_literals(5000, seed=12), 64 << 10, 5)]
    for name, lits, pe, seed in sets:
        blob = vsa.hwlm_build(lits)
        db = vsa.Database(ctx, blob)
        data = bench.make_corpus_device(torch, n, lits, seed=seed, plant_every=pe,
                                        device=torch.device("cuda", 0))
        torch.cuda.synchronize()
        for _ in range(2):
            ctx.scan_blocks(db, data.data_ptr(), [0], [n])
        ms = ctx.kernel_ms()
        c = ctx.debug_counters()
        cus = 256
        print("%-8s %.3f ms  gather %.0fK expand %.0fK confirm %.0fK idle %.0fK cyc/CU | "
              "rounds %d entries %d exp-rounds %d batches %d (per CU) cand %d" %
              (name, ms, c[4] / cus / 1e3, c[5] / cus / 1e3, c[6] / cus / 1e3,
               c[7] / cus / 1e3, c[8] // cus, c[9] // cus, c[10] // cus, c[11] // cus, c[2]),
              flush=True)
        db.close()
        del data
    ctx.close()


if __name__ == "__main__":
    main()
