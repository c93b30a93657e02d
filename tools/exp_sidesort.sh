#!/bin/bash
# Side-stream sort A/B (VSA_SIDE_SORT=0 / default): bench step vs kernel,
# pipelined (shared-stream contexts) and one step at a time, REPS rounds
# interleaved.  Output: gpurun_out/r03/sidesort.jsonl
O=gpurun_out/r03
mkdir -p $O
: > $O/sidesort.jsonl
for r in $(seq ${REPS:-2}); do
  for v in 0 1; do
    for m in pipe nopipe; do
      a=""; [ $m = nopipe ] && a="--no-pipeline"
      VSA_SIDE_SORT=$v timeout -k 10 300 python bench.py --no-cpu $a 2>$O/ss.err | tail -1 > $O/ss.json || exit 1
      python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({"side_sort": int(sys.argv[2]), "mode": sys.argv[3], "step_ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"], "overhead_us": round((d["ms_per_step"]-d["roofline"]["kernel_ms"])*1e3,1), "value": d["value"], "parity": d["parity"]}))' $O/ss.json $v $m >> $O/sidesort.jsonl || exit 1
    done
  done
done
cat $O/sidesort.jsonl
