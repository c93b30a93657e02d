#!/bin/bash
# literal-count sweep: LDS d14 (default) vs global-memory d16 first stage
set -e
OUT=gpurun_out/lits2
mkdir -p $OUT
for n in 5000 10000 20000 50000; do
  for dom in def 16; do
    if [ $dom = def ]; then unset VSA_FDR_DOMAIN; else export VSA_FDR_DOMAIN=$dom; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --lits $n 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lits $n dom $dom', d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'], d['confirm_candidates'], d['matches'])" >> $OUT/lits.txt
  done
done
