#!/bin/bash
# dynamic shares with the segment windows preloaded: parity, bench A/B, synchronous 4 GiB A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "dyn_shares or schedule_feedback or fdr_5k" > gpurun_out/dyn_tests3.txt 2>&1 || { tail -40 gpurun_out/dyn_tests3.txt; exit 1; }
tail -2 gpurun_out/dyn_tests3.txt
for i in 1 2 3; do
  for d in 0 1; do
    VSA_DYN_SHARES=$d timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 100 --warmup 32 > gpurun_out/abf_$d.json 2>gpurun_out/abf.err || { tail -5 gpurun_out/abf.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abf_$d.json').read().strip().splitlines()[-1]); print(json.dumps({'dyn':$d,'value':d['value'],'ms':d['ms_per_step'],'kGBs':d['roofline']['achieved']}))" | tee -a gpurun_out/ab_dyn3.jsonl
  done
done
for d in 1 0; do
  VSA_DYN_SHARES=$d HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python tools/exp_fb_trace.py 150 > gpurun_out/sync_dyn$d.json 2>/dev/null || exit 1
  python -c "import json,statistics as s; k=json.load(open('gpurun_out/sync_dyn$d.json'))['kernel_us']; print('sync dyn $d median', s.median(k[-100:]))" | tee -a gpurun_out/ab_dyn3.jsonl
done
