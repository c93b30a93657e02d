#!/bin/bash
# dynamic shares on the other configs (cfg1 noodle, cfg3 Teddy, 1 GiB): A/B interleaved
mkdir -p gpurun_out
for i in 1 2; do
  for d in 0 1; do
    VSA_DYN_SHARES=$d timeout -k 10 400 python tools/bench_configs.py --only 1,3 --steps 30 > gpurun_out/cfg_dyn$d.$i.jsonl 2>gpurun_out/cfg_dyn.err || { tail -5 gpurun_out/cfg_dyn.err; exit 1; }
    python -c "
import json
for l in open('gpurun_out/cfg_dyn$d.$i.jsonl'):
    d=json.loads(l); print(json.dumps({'dyn':$d,'w':d.get('workload',d.get('config',{}).get('workload')),'v':d.get('value'),'wall':d.get('wall_ms_per_call',d.get('ms_per_call'))}))" | tee -a gpurun_out/cfg_dyn_ab.jsonl
  done
done
