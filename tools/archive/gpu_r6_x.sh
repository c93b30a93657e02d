#!/bin/bash
# schedule feedback gain rule A/B: VSA_FB_GAIN_US=-1 (2 % rule) vs default
mkdir -p gpurun_out
VSA_XCD_FEEDBACK=1 HIP_FORCE_DEV_KERNARG=1 VSA_LIB_VARIANT=libvsa_diag.so timeout -k 10 300 python tools/exp_wg_spread.py > gpurun_out/wg_spread_gain.jsonl 2>gpurun_out/wg_spread.err || { tail -5 gpurun_out/wg_spread.err; exit 1; }
cat gpurun_out/wg_spread_gain.jsonl
for i in 1 2 3; do
  for g in -1 4; do
    VSA_FB_GAIN_US=$g timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 64 --warmup 32 > gpurun_out/ab_$g.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$g.json').read().strip().splitlines()[-1]); print(json.dumps({'gain':$g,'value':d['value'],'ms':d['ms_per_step'],'kms':d['roofline']['achieved']}))" | tee -a gpurun_out/ab_gain.jsonl
  done
done
