#!/bin/bash
# same-box A/B: default vs class-scan depth-8 variant (cfg1/2 lines)
set -e
OUT=gpurun_out/ab3
mkdir -p $OUT
for rep in 1 2; do
for v in libvectorscan_amd.so libvsa_cls8.so; do
  echo "== $v rep $rep" >> $OUT/ab.txt
  VSA_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_configs.py --only 1,2 --steps 10 --warmup 2 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:32], d['kernel_ms'], d['value'], d['parity'])" >> $OUT/ab.txt
done
done
