#!/bin/bash
# literal-scan segment scheduling experiments (env knobs in runtime.hip)
set -e
for cfg in "" "VSA_REGIONS=1" "VSA_REGIONS=4" "VSA_STATIC_SEGS=1"; do
  echo "== $cfg"
  env $cfg VSA_DEBUG_FLAGS=0 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr', d['roofline']['kernel_ms'])"
  env $cfg VSA_DEBUG_FLAGS=2 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr-filter', d['roofline']['kernel_ms'])"
  env $cfg timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 5 --warmup 1 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:22], d['kernel_ms'])"
done
