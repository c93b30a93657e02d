"""Summarise a tools/profile.sh run into profiles/:
  <tag>_kernel_stats.csv  (rocprofv3 --kernel-trace --stats summary)
  <tag>_pmc_lit_scan.csv  (FETCH_SIZE / WRITE_SIZE rows of the scan kernel)
  pmc_fdr5k_4gib.json     (HBM bytes per launch, read by bench.py)

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM section):
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so it is doubled; WRITE_SIZE is exact for 16-B stores.  The first
launch of each pass is the bench's parity launch on a 64 MiB sample and is
excluded (only full 4 GiB launches, > 0.5 ms, are averaged)."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
dst = os.path.join(ROOT, "profiles")
KERNEL = "vsa_lit_scan"

shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
            os.path.join(dst, tag + "_kernel_stats.csv"))
vals = {}
rows_out = []
for pass_ in ("fetch", "write"):
    rows = list(csv.DictReader(open(os.path.join(src, pass_, "run_counter_collection.csv"))))
    for r in rows:
        if KERNEL not in r["Kernel_Name"]:
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        rows_out.append([r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"],
                         r["Counter_Value"], dur])
        if dur > 500_000:  # full-size 4 GiB launches only (ns)
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
with open(os.path.join(dst, tag + "_pmc_lit_scan.csv"), "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["dispatch", "kernel", "counter", "value_kib", "duration_ns"])
    w.writerows(rows_out)
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024 * 2
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024
out = {
    "kernel": KERNEL + "<FDR>",
    "workload": "bench.py default (cfg4, 4 GiB as 4 x 1 GiB blocks)",
    "fetch_bytes_per_launch": round(fetch),
    "write_bytes_per_launch": round(write),
    "hbm_bytes_per_launch": round(fetch + write),
    "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count), WRITE_SIZE KiB x 1024",
    "source": "profiles/%s_pmc_lit_scan.csv" % tag,
}
json.dump(out, open(os.path.join(dst, "pmc_fdr5k_4gib.json"), "w"), indent=1)
print(json.dumps(out))

# per-dispatch durations of our kernels from the kernel trace
rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
with open(os.path.join(dst, tag + "_vsa_dispatches.csv"), "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["dispatch", "kernel", "grid_x", "wg_x", "lds", "vgpr", "sgpr", "scratch",
                "duration_ns"])
    full = []
    for r in rows:
        if "vsa_" not in r["Kernel_Name"]:
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        w.writerow([r["Dispatch_Id"], r["Kernel_Name"], r["Grid_Size_X"], r["Workgroup_Size_X"],
                    r["LDS_Block_Size"], r["VGPR_Count"], r["SGPR_Count"], r["Scratch_Size"], dur])
        if KERNEL in r["Kernel_Name"] and dur > 500_000:
            full.append(dur)
print("full-size %s launches: %d, avg %.1f us" % (KERNEL, len(full), sum(full) / len(full) / 1e3))

# SQ / LDS counters pass (tools/profile.sh), per full-size launch
sqf = os.path.join(src, "sq", "run_counter_collection.csv")
if os.path.exists(sqf):
    sq = {}
    for r in csv.DictReader(open(sqf)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 500_000:
            sq.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    sq = {k: sum(v) / len(v) for k, v in sq.items()}
    if sq:
        sq["lds_cycles_per_lds_instr"] = sq["SQ_LDS_IDX_ACTIVE"] / sq["SQ_INSTS_LDS"]
        sq["bank_conflict_share"] = sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"]
        json.dump(sq, open(os.path.join(dst, tag + "_sq_lds.json"), "w"), indent=1)
        print(json.dumps(sq))
# configs 1-3 / streaming lines
cl = os.path.join(src, "configs_trace.log")
if os.path.exists(cl):
    lines = [l for l in open(cl) if l.startswith("{")]
    open(os.path.join(dst, tag + "_configs.jsonl"), "w").writelines(lines)
    shutil.copy(os.path.join(src, "cfg", "run_kernel_stats.csv"),
                os.path.join(dst, tag + "_cfg_kernel_stats.csv"))
bl = [l for l in open(os.path.join(src, "bench_trace.log")) if l.startswith("{")]
if bl:
    open(os.path.join(dst, tag + "_bench.json"), "w").write(bl[-1])
