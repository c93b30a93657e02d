"""Per-step device timeline of a scan loop from a rocprofv3 kernel trace
(--kernel-trace -f csv): the literal-scan kernels and what runs between two
of them on the device -- the binned sort's launch (vsa_bin_finish) and the
gaps (kernel boundaries).  Takes the trace's last N scans (the timed tail
of a tools/exp_stripes.py run of one size and mode).
  python tools/trace_gaps.py <kernel_trace.csv> [steps]
One JSON line: medians over the steps (us) of the scan, the sort launch,
scan end -> sort start, sort end -> next scan start (or scan end -> next
scan start when no sort launch is between), and scan start -> next scan
start (the device step)."""
import csv
import json
import statistics
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        name = r.get("Kernel_Name", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
scans = [i for i, r in enumerate(rows) if "vsa_lit_scan" in r[2]]
tail = scans[-steps - 1:]
out = {"scan_us": [], "sort_us": [], "scan_to_sort_us": [], "sort_to_scan_us": [],
       "scan_to_scan_us": [], "step_us": [], "between": {}}
for a, b in zip(tail, tail[1:]):
    s0, e0, _ = rows[a]
    s1 = rows[b][0]
    out["scan_us"].append((e0 - s0) / 1e3)
    out["step_us"].append((s1 - s0) / 1e3)
    mid = rows[a + 1:b]
    for m in mid:
        key = m[2].split("(")[0]
        out["between"][key] = out["between"].get(key, 0) + 1
    fin = [m for m in mid if "vsa_bin_finish" in m[2]]
    if fin:
        fs, fe, _ = fin[0]
        out["sort_us"].append((fe - fs) / 1e3)
        out["scan_to_sort_us"].append((fs - e0) / 1e3)
        out["sort_to_scan_us"].append((s1 - fe) / 1e3)
    else:
        out["scan_to_scan_us"].append((s1 - e0) / 1e3)  # scan end -> next scan
res = {"trace": path, "steps": len(tail) - 1}
for k, v in out.items():
    if k == "between":
        res[k] = v
    elif v:
        res[k] = round(statistics.median(v), 2)
print(json.dumps(res))
