#!/bin/bash
# Teddy (cfg 3) kernel time under debug flags
set -e
for f in 0 2 32; do
  echo "flags $f"
  VSA_DEBUG_FLAGS=$f timeout -k 10 200 python tools/bench_configs.py --only 3 --steps 5 --warmup 1 2>&1 | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'], d['kernel_ms'], d['matches'])"
done
