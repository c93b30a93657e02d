#!/bin/bash
# same-box A/B: previous build (libvsa_base.so) vs current, cfg1
set -e
OUT=gpurun_out/ab4
mkdir -p $OUT
for rep in 1 2; do
for v in libvsa_base.so libvectorscan_amd.so; do
  echo "== $v rep $rep" >> $OUT/ab.txt
  VSA_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_configs.py --only 1 --steps 10 --warmup 2 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:32], d['kernel_ms'], d['value'], d['parity'])" >> $OUT/ab.txt
done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "noodle or nood" > $OUT/tests.log 2>&1
