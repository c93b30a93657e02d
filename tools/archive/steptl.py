"""Per-step GPU timeline from a rocprofv3 kernel + memory-copy trace
(tools/exp_steptl.sh): for each scan kernel, the gaps and durations of the
operations that follow it until the next scan kernel starts.
  python tools/steptl.py gpurun_out/steptl"""
import csv
import glob
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/steptl"
ops = []
for f in glob.glob(os.path.join(base, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]))
for f in glob.glob(os.path.join(base, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    "copy " + r.get("Direction", r.get("Operation", ""))))
ops.sort()
scans = [i for i, o in enumerate(ops) if "lit_scan" in o[2]]
rows = []
for a, b in zip(scans, scans[1:]):
    seq = ops[a:b + 1]
    t0 = seq[0][0]
    desc = []
    for s, e, name in seq:
        desc.append("%s @%.1f +%.1f" % (name.split("(")[0], (s - t0) / 1e3, (e - s) / 1e3))
    rows.append(((ops[b][0] - ops[a][1]) / 1e3, (ops[a][1] - ops[a][0]) / 1e3, desc))
for gap, kern, desc in rows[-6:]:
    print("scan %.1f us, scan end -> next scan start %.1f us" % (kern, gap))
    print("   " + " | ".join(desc))
gaps = [g for g, _, _ in rows[len(rows) // 2:]]
if gaps:
    print("median scan end -> next scan start: %.1f us over %d steps" %
          (sorted(gaps)[len(gaps) // 2], len(gaps)))
