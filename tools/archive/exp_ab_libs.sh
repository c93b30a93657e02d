#!/bin/bash
# kernel times of configs 3 / 4s under library variants (VSA_LIB_VARIANT)
for v in "$@"; do
  echo "== $v"
  VSA_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_configs.py --only 3,4s --steps 20 --warmup 20 2>/dev/null | python -c '
import json,sys
for l in sys.stdin:
    if l.startswith("{"):
        d=json.loads(l); print("%-50s %.4f" % (d["workload"][:50], d["kernel_ms"]))' || exit 1
done
