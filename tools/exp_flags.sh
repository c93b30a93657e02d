#!/bin/bash
# kernel time of the cfg-4 bench: product vs debug variants
mkdir -p gpurun_out
for v in "" "VSA_DEBUG_FLAGS=1024" "" "VSA_DEBUG_FLAGS=1024"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 bench.py --steps 20 --warmup 20 --no-cpu --no-parity | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['matches'], d['confirm_candidates'])" || exit 1
done
