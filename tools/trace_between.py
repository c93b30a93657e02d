"""What the device does between consecutive scans: reads a rocprofv3
kernel trace and (optionally) its memory-copy trace (-f csv) and, for the
last N literal scans, prints per gap the kernels and copies that start in
it, with offsets from the scan's end (us).  Medians over the gaps at the
end.  python tools/trace_between.py <kernel_trace.csv> [<memory_copy_trace.csv>] [N]"""
import csv
import json
import statistics
import sys

kpath = sys.argv[1]
mpath = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2].endswith(".csv") else None
n = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 20
ev = []
with open(kpath) as f:
    for r in csv.DictReader(f):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r.get("Kernel_Name", "").split("(")[0][:40]))
if mpath:
    with open(mpath) as f:
        for r in csv.DictReader(f):
            kind = r.get("Direction", r.get("Operation", "copy"))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + str(kind)))
ev.sort()
scans = [i for i, e in enumerate(ev) if e[2].startswith("void vsa_lit_scan") or
         e[2].startswith("vsa_lit_scan")]
tail = scans[-n - 1:]
gaps, steps, scan_us = [], [], []
for a, b in zip(tail, tail[1:]):
    s0, e0, _ = ev[a]
    s1 = ev[b][0]
    scan_us.append((e0 - s0) / 1e3)
    steps.append((s1 - s0) / 1e3)
    gaps.append((s1 - e0) / 1e3)
    mid = [e for e in ev[a + 1:] if e[0] < s1]
    print(json.dumps({"scan_us": round((e0 - s0) / 1e3, 1), "gap_us": round((s1 - e0) / 1e3, 1),
                      "between": [(m[2], round((m[0] - e0) / 1e3, 1), round((m[1] - m[0]) / 1e3, 1))
                                  for m in mid]}))
print(json.dumps({"scans": len(tail) - 1, "scan_us_median": round(statistics.median(scan_us), 1),
                  "gap_us_median": round(statistics.median(gaps), 1),
                  "step_us_median": round(statistics.median(steps), 1)}))
