#!/bin/bash
# literal-count sweep of the FDR path (4 GiB): time, confirm candidates, confirm-wave phases
set -e
OUT=gpurun_out/lits
mkdir -p $OUT
for n in 1000 5000 10000 20000 50000; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --lits $n 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lits $n', d['config']['workload'][-12:], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'], d['confirm_candidates'], d['matches'])" >> $OUT/lits.txt
done
