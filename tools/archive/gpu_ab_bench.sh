#!/bin/bash
# Interleaved A/B of library variants on the default bench line (no CPU leg,
# no parity, no end-to-end): REPS rounds over default + the named variants
# (vectorscan_amd/libvsa_<name>.so); the value (pipelined step) and the
# kernel time of each run, then the medians.
OUT=gpurun_out/${AB_OUT:-ab_bench}
mkdir -p $OUT
REPS=${REPS:-3}
for r in $(seq $REPS); do
  for v in default "$@"; do
    lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
    VSA_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --no-cpu --no-parity --no-e2e ${BENCH_ARGS} 2>>$OUT/err.log | tail -1 | sed "s/^/$v /" >> $OUT/bench.txt || exit 1
  done
done
python3 - $OUT/bench.txt <<'P'
import json, statistics, sys
rows = {}
for l in open(sys.argv[1]):
    v, js = l.split(" ", 1)
    d = json.loads(js)
    rows.setdefault(v, []).append((d["ms_per_step"], d["roofline"]["kernel_ms"], d["value"]))
for v, rs in rows.items():
    print("%-10s step %.4f kernel %.4f value %.1f   runs %s" % (v, statistics.median(r[0] for r in rs),
          statistics.median(r[1] for r in rs), statistics.median(r[2] for r in rs), rs))
P
