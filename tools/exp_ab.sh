#!/bin/bash
# A/B the default library against a variant build (VSA_LIB_VARIANT)
set -e
for v in libvectorscan_amd.so $VARIANTS; do
  echo "== $v"
  for f in 0 2; do
    VSA_LIB_VARIANT=$v VSA_DEBUG_FLAGS=$f timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fdr flags $f', d['roofline']['kernel_ms'], d['parity'])"
  done
  VSA_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 5 --warmup 1 2>/dev/null | grep '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['workload'][:22], d['kernel_ms'], d['parity'])"
done
