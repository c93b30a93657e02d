#!/bin/bash
# kernel time + confirm-wave counters vs literal-set size (4 GiB, FDR)
timeout -k 10 120 python3 bench.py --steps 20 --warmup 20 --no-cpu --no-parity | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1
for n in 1000 5000 10000 20000 50000; do
  LITS=$n VSA_DEBUG_FLAGS=64 timeout -k 10 200 python3 tools/exp_counters.py || exit 1
done
