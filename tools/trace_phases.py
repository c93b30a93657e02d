"""Split the traced bench's vsa_lit_scan launches into the bench's phases.

    python tools/trace_phases.py TAG  ->  profiles/TAG_prof/lit_scan_phases.json

Reads gpurun_out/prof_TAG/trace/*kernel_trace.csv (tools/profile.sh: the
default `python3 bench.py` under rocprofv3 --kernel-trace) and the bench line
in bench_trace.log for the settle / warmup / steps counts.  Launches in
dispatch order: settle (clock ramp), warmup, the timed steps, then the
parity / end-to-end / other launches."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
f = glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "vsa_lit_scan" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
bench = None
for line in open(os.path.join(src, "bench_trace.log")):
    if line.startswith("{") and '"metric"' in line:
        bench = json.loads(line)
assert bench is not None, "no bench line in bench_trace.log"
ns, nw, nt = bench["settle"]["launches"], bench["warmup"], bench["steps"]
cuts = [("settle (clock ramp)", 0, ns), ("warmup", ns, ns + nw),
        ("timed steps", ns + nw, ns + nw + nt), ("parity / end-to-end / other", ns + nw + nt, len(dur))]
out = {"source": "rocprofv3 --kernel-trace --stats -- python3 bench.py (tools/profile.sh %s); "
                 "launches in dispatch order" % tag,
       "bench_kernel_ms_hip_events": bench["roofline"]["kernel_ms"], "phases": {}}
for name, a, b in cuts:
    d = dur[a:b]
    if d:
        out["phases"][name] = {"launches": len(d), "mean_us": round(statistics.mean(d), 1),
                               "median_us": round(statistics.median(d), 1)}
dst = os.path.join(ROOT, "profiles", tag + "_prof")
os.makedirs(dst, exist_ok=True)
json.dump(out, open(os.path.join(dst, "lit_scan_phases.json"), "w"), indent=1)
print(json.dumps(out))
