#!/bin/bash
# A/B: default vs no-setprio build on cfg1/3 and the headline; stream probe; full bench with CPU baseline
set -e
OUT=gpurun_out/ab2
mkdir -p $OUT
timeout -k 10 120 ./tools/probe_stream > $OUT/probe.txt 2>&1
for v in libvectorscan_amd.so libvsa_noprio.so; do
  echo "== $v" >> $OUT/ab.txt
  VSA_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 5 --warmup 1 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:28], d['kernel_ms'], d['value'])" >> $OUT/ab.txt
  VSA_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr', d['roofline']['kernel_ms'])" >> $OUT/ab.txt
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $OUT/bench_full.log 2>&1
