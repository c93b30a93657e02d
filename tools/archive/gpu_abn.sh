#!/bin/bash
# Interleaved A/B of experiment variants (VSA_LIB_VARIANT, tools/build_variant.sh):
# REPS rounds over default + the named variants, kernel ms of each run, then
# the median per variant.   tools/gpu_abn.sh variant...
mkdir -p gpurun_out/abn
REPS=${REPS:-3}
for r in $(seq $REPS); do
  for v in default "$@"; do
    lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
    VSA_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --no-cpu --no-parity --warmup 10 --steps 20 ${BENCH_ARGS} 2>gpurun_out/abn/$v.err | tail -1 > gpurun_out/abn/${v}_$r.json || exit 1
  done
done
python3 - "$@" <<'P'
import json, statistics, sys
for v in ["default"] + sys.argv[1:]:
    ks, ms = [], []
    r = 1
    while True:
        try:
            d = json.load(open("gpurun_out/abn/%s_%d.json" % (v, r)))
        except (OSError, ValueError):
            break
        ks.append(d["roofline"]["kernel_ms"]); ms.append(d["ms_per_step"]); r += 1
    print("%-10s kernel median %.4f  runs %s  step median %.4f" % (v, statistics.median(ks), ks, statistics.median(ms)))
P
