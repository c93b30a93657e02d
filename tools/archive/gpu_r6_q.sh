#!/bin/bash
# Round 6: fused finish, publish from the look-back's totals (no counter
# reads, no feedback copy): its tests, the suite, then the rank step A/B
# (device kernel arguments, every 4th launch timed), fused off / on
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fused or binned_sort or plan_pack or feedback or timing or crowd" > gpurun_out/fusedtest.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -3 gpurun_out/fusedtest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
export HIP_FORCE_DEV_KERNARG=1
for i in 1 2 3; do
  for f in 0 1; do
    VSA_FUSED_FINISH=$f EXP_TIMING=4 EXP_RANKS=8,4,1 EXP_MODES=pack1 timeout -k 10 200 python tools/exp_stripes.py 300 30 | sed "s/^{/{\"fused\": $f, /" >> gpurun_out/fq_ab.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/fq_ab.jsonl'):
    r = json.loads(l)
    d[(r['ranks'], r['fused'])].append((r['step_ms'], r['kernel_ms']))
for k in sorted(d):
    print(k, d[k])
PY
