#!/bin/bash
# vsa_bin_finish with its publish in a workgroup of its own: parity, then A/B
mkdir -p gpurun_out
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "binned or plan_pack or feedback or fdr_5k or crowd or fused or sampled" > gpurun_out/pub_tests.txt 2>&1 || { tail -30 gpurun_out/pub_tests.txt; exit 1; }
tail -1 gpurun_out/pub_tests.txt
for i in 1 2; do
  for w in 0 1; do
    VSA_BF_PUB_WG=$w EXP_TIMING=4 EXP_MODES=pipe,pack1 EXP_RANKS=8,1 timeout -k 10 300 python tools/exp_stripes.py 200 30 | sed "s/^{/{\"pub_wg\": $w, /" >> gpurun_out/pub_ab.jsonl || exit 1
    VSA_BF_PUB_WG=$w timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 100 --warmup 32 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'pub_wg':$w,'bench':d['value'],'ms':d['ms_per_step'],'kms':d['roofline']['kernel_ms']}))" >> gpurun_out/pub_ab.jsonl || exit 1
  done
done
cut -c1-200 gpurun_out/pub_ab.jsonl
