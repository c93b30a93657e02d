#!/bin/bash
# kernel time of the bench workload under debug flags (see kernels.h dbg)
set -e
for f in ${FLAGS:-0 2 8 16}; do
  echo "flags $f"
  VSA_DEBUG_FLAGS=$f timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > /tmp/exp_$f.log 2>&1
  python3 - /tmp/exp_$f.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["roofline"]["kernel_ms"], d["confirm_candidates"], d["matches"])
PY
done
