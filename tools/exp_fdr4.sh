#!/bin/bash
# FDR4 (4-field first stage, default) vs the 8-field pair table (VSA_FDR8=1):
# interleaved bench runs, REPS rounds -> gpurun_out/r03/fdr4_ab.jsonl
O=gpurun_out/r03
mkdir -p $O
: > $O/fdr4_ab.jsonl
for r in $(seq ${REPS:-3}); do
  for v in fdr4 fdr8; do
    e=""; [ $v = fdr8 ] && e="VSA_FDR8=1"
    env $e timeout -k 10 300 python bench.py --no-cpu --no-e2e 2>$O/fdr4.err | tail -1 > $O/fdr4.json || exit 1
    python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({"table": sys.argv[2], "round": int(sys.argv[3]), "step_ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"], "value": d["value"], "candidates": d["confirm_candidates"], "parity": d["parity"]}))' $O/fdr4.json $v $r >> $O/fdr4_ab.jsonl || exit 1
  done
done
cat $O/fdr4_ab.jsonl
