#!/bin/bash
# dynamic (per-region tickets) vs static segment assignment
set -e
OUT=gpurun_out/static
mkdir -p $OUT
for st in 0 1; do
  if [ $st = 1 ]; then export VSA_STATIC_SEGS=1; fi
  echo "== static=$st" >> $OUT/ab.txt
  timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 5 --warmup 1 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:28], d['kernel_ms'], d['value'], d['parity'])" >> $OUT/ab.txt
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr', d['roofline']['kernel_ms'], d['parity'])" >> $OUT/ab.txt
  VSA_DEBUG_FLAGS=2 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr filter-only', d['roofline']['kernel_ms'])" >> $OUT/ab.txt
done
