#!/bin/bash
# Round 6: the rank step with device kernel arguments, sampled timing (every
# 4th launch, as bench.py) and the fused finish off / on, interleaved
mkdir -p gpurun_out
export HIP_FORCE_DEV_KERNARG=1
for i in 1 2 3; do
  for f in 0 1; do
    VSA_FUSED_FINISH=$f EXP_TIMING=4 EXP_RANKS=8,4,2 EXP_MODES=pack1 timeout -k 10 200 python tools/exp_stripes.py 300 30 | sed "s/^{/{\"fused\": $f, /" >> gpurun_out/fk_ab.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/fk_ab.jsonl'):
    r = json.loads(l)
    d[(r['ranks'], r['fused'])].append((r['step_ms'], r['kernel_ms']))
for k in sorted(d):
    print(k, d[k])
PY
