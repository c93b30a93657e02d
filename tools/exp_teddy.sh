#!/bin/bash
# Teddy / Fat Teddy breakdown: full, filter only (2), expansion without
# confirm (16), first-stage candidate count (32)
set -e
OUT=gpurun_out/teddy
mkdir -p $OUT
for f in 0 2 16 32; do
  VSA_DEBUG_FLAGS=$f timeout -k 10 200 python tools/bench_configs.py --only 3 --steps 5 --warmup 1 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('flags $f', d['workload'][:28], d['kernel_ms'], d['value'], d['confirm_candidates'], d['parity'])"
done > $OUT/teddy.txt 2>&1
