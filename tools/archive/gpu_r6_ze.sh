#!/bin/bash
# dynamic shares (FDR, >= 2 GiB): parity tests, then bench A/B interleaved, then cfg1/3 sanity
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "dyn_shares or schedule_feedback or fdr_5k or fused_finish or plan_pack or binned" > gpurun_out/dyn_tests2.txt 2>&1 || { tail -40 gpurun_out/dyn_tests2.txt; exit 1; }
tail -3 gpurun_out/dyn_tests2.txt
for i in 1 2 3; do
  for d in 0 1; do
    VSA_DYN_SHARES=$d timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 100 --warmup 32 > gpurun_out/abe_$d.json 2>gpurun_out/abe.err || { tail -5 gpurun_out/abe.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abe_$d.json').read().strip().splitlines()[-1]); print(json.dumps({'dyn':$d,'value':d['value'],'ms':d['ms_per_step'],'kGBs':d['roofline']['achieved']}))" | tee -a gpurun_out/ab_dyn2.jsonl
  done
done
