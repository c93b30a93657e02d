#!/bin/bash
# Round 6: fused finish A/B (VSA_FUSED_FINISH 0 / 1 interleaved, 3 rounds):
# the per-rank step packed for the collective at N = 8 / 4 / 1, then the
# bench line twice each
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fused or binned_sort or plan_pack" > gpurun_out/fusedtest.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -2 gpurun_out/fusedtest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for f in 0 1; do
    VSA_FUSED_FINISH=$f EXP_RANKS=8,4,1 EXP_MODES=pack1 timeout -k 10 200 python tools/exp_stripes.py 200 30 | sed "s/^{/{\"fused\": $f, /" >> gpurun_out/fused3_ab.jsonl 2>>gpurun_out/fused3_ab.err || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/fused3_ab.jsonl'):
    r = json.loads(l)
    d[(r['ranks'], r['fused'])].append((r['step_ms'], r['kernel_ms']))
for k in sorted(d):
    print(k, d[k])
PY
for i in 1 2; do
  for f in 0 1; do
    VSA_FUSED_FINISH=$f timeout -k 10 400 python bench.py --no-cpu --no-cfg5 --no-e2e 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print($f, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])" || exit 1
  done
done
