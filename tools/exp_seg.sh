#!/bin/bash
# segment size sweep for the literal scan (prologue cost vs balance)
set -e
OUT=gpurun_out/seg
mkdir -p $OUT
for kib in 64 128 256 512; do
  echo "== seg max $kib KiB" >> $OUT/seg.txt
  VSA_SEG_MAX_KIB=$kib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr', d['roofline']['kernel_ms'], d['parity'])" >> $OUT/seg.txt
  VSA_SEG_MAX_KIB=$kib timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 5 --warmup 1 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:28], d['kernel_ms'], d['parity'])" >> $OUT/seg.txt
done
