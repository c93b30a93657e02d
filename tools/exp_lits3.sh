#!/bin/bash
set -e
OUT=gpurun_out/lits3
mkdir -p $OUT
for n in 5000 10000 20000; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --lits $n 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lits $n', d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'], d['confirm_candidates'], d['matches'])" >> $OUT/lits.txt
done
