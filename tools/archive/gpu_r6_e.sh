#!/bin/bash
# Round 6: per-rank steps with a one-workgroup stand-in collective, with and
# without 2 reserved CUs, then the profile recipe (tools/profile.sh r06)
mkdir -p gpurun_out
for r in 0 2; do
  EXP_RESERVE=$r timeout -k 10 300 python tools/exp_stripes.py 50 20 > gpurun_out/stripes_tiny_res$r.jsonl 2>gpurun_out/stripes_tiny_res$r.err || exit 1
  echo "== reserve $r"; grep '"side"\|"pack1"' gpurun_out/stripes_tiny_res$r.jsonl
done
bash tools/profile.sh r06 && echo profile-ok
