#!/bin/bash
# segment scheduling variants on configs 1 / 3 and the bench kernel
for v in "X=1" "VSA_STATIC_SEGS=1" "VSA_REGIONS=4" "VSA_SEG_MAX_KIB=512" "VSA_SEG_MAX_KIB=32"; do
  echo "== $v"
  env $v timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 20 --warmup 20 2>/dev/null | python -c '
import json,sys
for l in sys.stdin:
    if l.startswith("{"):
        d=json.loads(l); print("%-50s %.4f" % (d["workload"][:50], d["kernel_ms"]))' || exit 1
  env $v timeout -k 10 200 python bench.py --no-cpu --no-parity --steps 10 --warmup 10 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("bench kernel", d["roofline"]["kernel_ms"], d["ms_per_step"])' || exit 1
done
