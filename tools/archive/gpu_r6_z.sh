#!/bin/bash
# dynamic shares: parity tests, then bench A/B (VSA_DYN_SHARES 0 / 1, interleaved)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "dyn_shares or schedule_feedback or fdr_5k or fused_finish" > gpurun_out/dyn_tests.txt 2>&1 || { tail -40 gpurun_out/dyn_tests.txt; exit 1; }
tail -3 gpurun_out/dyn_tests.txt
for i in 1 2 3; do
  for d in 0 1; do
    VSA_DYN_SHARES=$d timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 64 --warmup 32 > gpurun_out/abd_$d.json 2>gpurun_out/abd.err || { tail -5 gpurun_out/abd.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abd_$d.json').read().strip().splitlines()[-1]); print(json.dumps({'dyn':$d,'value':d['value'],'ms':d['ms_per_step'],'kGBs':d['roofline']['achieved']}))" | tee -a gpurun_out/ab_dyn.jsonl
  done
done
