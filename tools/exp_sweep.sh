#!/bin/bash
set -e
OUT=gpurun_out/sweep
mkdir -p $OUT
run() { echo "== $*" >> $OUT/s.txt; env "$@" timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 2 2>/dev/null | grep '^{' | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['value'], d['parity'], d['confirm_candidates'])" >> $OUT/s.txt; }
run X=0
run VSA_FDR_DOMAIN=13
run VSA_FDR_DOMAIN=12
run VSA_SEG_KB=32
run VSA_SEG_KB=128
run VSA_SEG_KB=256
run VSA_REGIONS=1
run X=0
