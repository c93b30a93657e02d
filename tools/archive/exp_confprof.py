"""Confirm-wave phase profile (VSA_DEBUG_FLAGS=64: s_memtime cycles spent
gathering / expanding / confirming / idle, summed over the confirm waves,
plus round counts) for match-heavy workloads: cfg-1 noodle and cfg-3 Teddy
over their 1 GiB corpora planted every 4 KiB, and the cfg-4 FDR scan.
Usage: python tools/exp_confprof.py
Needs the diagnostic build: tools/build_variant.sh diag -DVSA_DIAG, then
VSA_LIB_VARIANT=libvsa_diag.so (the product build compiles these counters
out)."""
import json
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(64 | 32768)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import tools.bench_configs as bc  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
n = 1 << 30
for name, lits, seed, plant in (("teddy48e18_p4k", bc.lits_printable(48, 55), 3, 4 << 10),
                                ("noodle_p4k", [vsa.HwlmLiteral(b"abcde", False, 1)], 3, 4 << 10),
                                ("teddy48_p4k", bc.lits_printable(48, 55), 3, 4 << 10),
                                ("fdr5k_1g", bench.make_literals(5000, seed=12), 5, 64 << 10)):
    db = vsa.Database(ctx, vsa.hwlm_build(lits, engine_hint=18 if "e18" in name else -1))
    data = bench.make_corpus_device(torch, 0, n, n, lits, seed, plant, dev)
    torch.cuda.synchronize()
    for _ in range(40):
        m = ctx.scan_blocks(db, data.data_ptr(), [0], [n])
    c = ctx.debug_counters()
    k = ctx.kernel_ms()
    cyc = k * 1e-3 * 2.1e9 * 256  # confirm-wave cycles available (one per CU, ~2.1 GHz)
    rec = {"workload": name, "kernel_ms": round(k, 4), "matches": m, "candidates": c[2],
           "share_gather": round(c[4] / cyc, 3), "share_expand": round(c[5] / cyc, 3),
           "share_confirm": round(c[6] / cyc, 3), "share_idle": round(c[7] / cyc, 3),
           "gather_rounds": c[8], "chunk_entries": c[9], "exp_rounds": c[10],
           "confirm_batches": c[11],
           # scanning waves (15 per CU): candidate-path and push cycles
           "scan_share_cand": round(c[13] / (cyc * 15), 4),
           "scan_share_push": round(c[14] / (cyc * 15), 4), "cand_iters": c[15]}
    print(json.dumps(rec), flush=True)
    del data
