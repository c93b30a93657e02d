#!/bin/bash
# summarize gpurun_out/quick (exp_quick.sh results)
D=${1:-gpurun_out/quick}
tail -1 $D/gpu_tests.log
for f in bench bench_d13 bench_f2; do
  [ -f $D/$f.log ] && tail -1 $D/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['roofline']['kernel_ms'], 'ms', d['roofline']['achieved'], 'GB/s frac', d['roofline']['frac'], 'parity', d['parity'], 'cand', d['confirm_candidates'])" 2>/dev/null || echo "$f: no json"
done
grep '^{' $D/configs.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:40], d['kernel_ms'], d['value'], d['parity'])"
