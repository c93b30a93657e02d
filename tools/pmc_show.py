"""Print per-launch averages of the counters collected by tools/pmc_fdr.sh
(full-size scan launches only)."""
import csv
import glob
import os
import sys

out = sys.argv[1]
vals = {}
for f in glob.glob(os.path.join(out, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "vsa_lit_scan" not in r["Kernel_Name"]:
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if dur < 200_000:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print("%-24s %16.4g  (n=%d)" % (k, sum(v) / len(v), len(v)))
t = glob.glob(os.path.join(out, "t", "run_kernel_stats.csv"))
if t:
    for r in csv.DictReader(open(t[0])):
        print("%-60s calls %s avg %.1f us" % (r["Name"][:60], r["Calls"],
                                               float(r["AverageNs"]) / 1e3))
