#!/usr/bin/env python3
"""Per-launch SQ / LDS counter summary of tools/exp_pmc_ab.sh runs (full
4 GiB launches only): LDS cycles per LDS instruction, bank-conflict share,
instructions per KiB, wait shares and the effective clock."""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
base = os.path.join(ROOT, "gpurun_out", "pmcab")
KIB = 4 * (1 << 30) / 1024
for v in sys.argv[1:] or ["default"]:
    vals, durs = {}, []
    for p in (1, 2):
        for f in glob.glob(os.path.join(base, "%s_p%d" % (v, p), "**", "*counter_collection.csv"),
                           recursive=True):
            for r in csv.DictReader(open(f)):
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                if dur < 500_000:
                    continue
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    durs.append(dur)
    m = {k: sum(x) / len(x) for k, x in vals.items()}
    d = sum(durs) / len(durs) if durs else float("nan")
    out = {"variant": v, "kernel_ms": round(d / 1e6, 4)}
    if "SQ_LDS_IDX_ACTIVE" in m:
        out["lds_cyc_per_instr"] = round(m["SQ_LDS_IDX_ACTIVE"] / m["SQ_INSTS_LDS"], 3)
        out["conflict_share"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 3)
        out["lds_cyc_per_kib_per_cu"] = round(m["SQ_LDS_IDX_ACTIVE"] / KIB, 2)
        out["valu_per_kib"] = round(m["SQ_INSTS_VALU"] / KIB, 1)
        out["lds_instr_per_kib"] = round(m["SQ_INSTS_LDS"] / KIB, 2)
    if "SQ_INSTS_SALU" in m:
        out["salu_per_kib"] = round(m["SQ_INSTS_SALU"] / KIB, 1)
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES"):
        if k in m:
            out[k] = "%.4g" % m[k]
    if "GRBM_GUI_ACTIVE" in m and durs:
        out["eff_clock_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / d, 3)
    print(out)
