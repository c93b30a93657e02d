"""Where a literal-scan launch spends its time beyond the steady sweep
(VSA_DEBUG_FLAGS=4096|8192 wave log, s_memrealtime at 100 MHz): per size,
the hipEvent kernel time against the waves' own timeline -- entry ->
first scanning-wave start (table staging), start -> median / last wave end
(the tail), and the streaming-read ceiling of the same bytes.  One JSON line
per (workload, size).  Usage: python tools/exp_overhead.py [out.jsonl]
Needs the diagnostic build: tools/build_variant.sh diag -DVSA_DIAG, then
VSA_LIB_VARIANT=libvsa_diag.so (the product build compiles these counters
out)."""
import ctypes
import json
import os
import sys

os.environ["VSA_DEBUG_FLAGS"] = str(4096 | 8192 | int(os.environ.get("EXTRA_DBG", "0")))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

dev = torch.device("cuda", 0)
ctx = vsa.Context(0)
out = open(sys.argv[1], "a") if len(sys.argv) > 1 else None
log = torch.zeros(1024 * 16 * 8, dtype=torch.int64, device=dev)
vsa.lib.vsa_set_wave_log.argtypes = [ctypes.c_void_p]
vsa.lib.vsa_set_wave_log(log.data_ptr())
total = 4 << 30
fdr_lits = bench.make_literals(5000, seed=12)
data = bench.make_corpus_device(torch, 0, total, total, fdr_lits, 5, 64 << 10, dev)
# WL: which workloads (comma list); the *_p4k ones scan their own 1 GiB
# corpus with a literal planted every 4 KiB (tools/bench_configs.py cfg 1 / 3)
WL = os.environ.get("WL", "fdr5k,noodle").split(",")
# SORT=0: unsorted output (no binned-sort staging in the scan)
SORT = os.environ.get("SORT", "1") != "0"
import tools.bench_configs as bc  # noqa: E402
sets = {"fdr5k": (fdr_lits, -1, None), "noodle": ([vsa.HwlmLiteral(b"abcde", False, 1)], -1, None),
        "noodle_p4k": ([vsa.HwlmLiteral(b"abcde", False, 1)], -1, 3),
        "teddy48_p4k": (bc.lits_printable(48, 55), -1, 3),
        "teddy48": (bc.lits_printable(48, 55), -1, None),
        "teddy48e18_p4k": (bc.lits_printable(48, 55), 18, 3),
        "teddy48e18": (bc.lits_printable(48, 55), 18, None)}
dbs = {}
for w in WL:
    ls, hint, seed = sets[w]
    dbs[w] = (vsa.Database(ctx, vsa.hwlm_build(ls, engine_hint=hint)),
              None if seed is None else
              bench.make_corpus_device(torch, 0, 1 << 30, 1 << 30, ls, seed, 4 << 10, dev))
torch.cuda.synchronize()
for name, (db, own) in dbs.items():
    base = data.data_ptr() if own is None else own.data_ptr()
    for mib, nb in (((512, 1), (1024, 1), (4096, 4)) if own is None else ((1024, 1),)):
        n = mib << 20
        bl = n // nb
        offs = [i * bl for i in range(nb)]
        for _ in range(40):  # clock ramp
            ctx.scan_blocks(db, base, offs, [bl] * nb, sort=SORT)
        rows = []
        cgap = []
        for _ in range(8):
            log.zero_()
            ctx.scan_blocks(db, base, offs, [bl] * nb, sort=SORT)
            k = ctx.kernel_ms()
            L = log[:65536].view(-1, 8).cpu().numpy().astype(np.int64)
            # scanning waves log their entry in field 7; confirm waves log
            # (entry, end, 1, 0 ...)
            rows_i = np.arange(len(L))
            scm = (L[:, 0] != 0) & (L[:, 1] != 0) & (L[:, 7] != 0)
            cfm = (L[:, 0] != 0) & (L[:, 2] == 1) & (L[:, 7] == 0)
            sc, cf = L[scm], L[cfm]
            cf_wg = rows_i[cfm] // 16
            ent = sc[:, 7]
            t0 = min(ent.min(), cf[:, 0].min()) if len(cf) else ent.min()
            st = (sc[:, 0] - t0) / 100.0
            en = (sc[:, 1] - t0) / 100.0
            wg_end = {}
            for w, e in zip(sc[:, 4].tolist(), en.tolist()):
                wg_end[w] = max(wg_end.get(w, 0.0), e)
            we = np.array(list(wg_end.values()))
            # per workgroup: its confirm wave's end after its last scanning
            # wave; all-done seen -> end; last batch start -> end
            gap, tail_done, tail_batch, nb_after = [], [], [], []
            for r, w in zip(cf, cf_wg.tolist()):
                if w not in wg_end:
                    continue
                ce = (r[1] - t0) / 100.0
                gap.append(ce - wg_end[w])
                if r[3]:
                    tail_done.append((r[1] - r[3]) / 100.0)
                if r[4]:
                    tail_batch.append((r[1] - r[4]) / 100.0)
                nb_after.append(r[5])
            cgap.append([float(np.median(gap)), float(np.max(gap)),
                         float(np.median(tail_done)) if tail_done else -1,
                         float(np.median(tail_batch)) if tail_batch else -1,
                         float(np.mean(nb_after))])
            rows.append([k * 1000.0, float(np.median(st)), float(st.max()), float(en.min()),
                         float(np.median(en)), float(en.max()), float(np.median(we)),
                         float(we.min()),
                         float((cf[:, 1].max() - t0) / 100.0) if len(cf) else 0.0])
        R = np.median(np.array(rows), axis=0)
        C = np.median(np.array(cgap), axis=0)
        _, ms, _ = ctx.read_ceiling(base, n, 5)
        rec = {"workload": name, "engine": dbs[name][0].engine, "mib": mib, "blocks": nb, "kernel_us": round(R[0], 1),
               "start_us_p50": round(R[1], 2), "start_us_max": round(R[2], 2),
               "wave_end_us_min": round(R[3], 1), "wave_end_us_p50": round(R[4], 1),
               "wave_end_us_max": round(R[5], 1), "wg_done_us_p50": round(R[6], 1),
               "wg_done_us_min": round(R[7], 1),
               "confirm_end_us_max": round(R[8], 1),
               "outside_waves_us": round(R[0] - max(R[5], R[8]), 1),
               "read_ceiling_us": round(ms * 1000.0, 1),
               "confirm_after_scan_us_p50": round(C[0], 2),
               "confirm_after_scan_us_max": round(C[1], 2),
               "confirm_end_after_all_done_us_p50": round(C[2], 2),
               "confirm_end_after_last_batch_us_p50": round(C[3], 2),
               "batches_after_all_done_mean": round(C[4], 2),
               "ideal_us_at_p50_rate": round(R[4] - R[1], 1)}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
