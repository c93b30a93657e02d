#!/bin/bash
# Sweep ring depth (chunks in flight per scanning wave): cfg-4 bench line and
# configs 1 / 3 kernel times per library variant
#   tools/build_variant.sh d6 -DLIT_DEPTH=6; tools/exp_depth.sh libvsa_d6.so ...
mkdir -p gpurun_out
for v in libvectorscan_amd.so "$@"; do
  VSA_LIB_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu > gpurun_out/dep_$v.json 2>/dev/null || exit 1
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], "cfg4", d["ms_per_step"], d["roofline"]["kernel_ms"], d["parity"])' gpurun_out/dep_$v.json $v || exit 1
  VSA_LIB_VARIANT=$v timeout -k 10 200 python tools/bench_configs.py --only 1,3 --steps 20 --warmup 20 2>/dev/null | python -c '
import json,sys
for l in sys.stdin:
    if l.startswith("{"):
        d=json.loads(l); print("   %-50s %.4f %s" % (d["workload"][:50], d["kernel_ms"], d.get("parity")))' || exit 1
done
