#!/bin/bash
# cfg-5 pass split (one at a time vs pipelined, per replay thread count),
# then the bench A/B with the shared-stream second context and the stripe table.
mkdir -p gpurun_out/r03c
VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 > gpurun_out/r03c/cfg5.jsonl 2> gpurun_out/r03c/cfg5.err || { tail -5 gpurun_out/r03c/cfg5.err; exit 1; }
cat gpurun_out/r03c/cfg5.jsonl
timeout -k 10 300 python bench.py --no-cpu 2>gpurun_out/r03c/b1.err | tail -1 > gpurun_out/r03c/bench_pipe.json || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-pipeline 2>gpurun_out/r03c/b2.err | tail -1 > gpurun_out/r03c/bench_nopipe.json || exit 1
timeout -k 10 300 python bench.py --no-cpu --warmup 5 2>gpurun_out/r03c/b3.err | tail -1 > gpurun_out/r03c/bench_w5.json || exit 1
for f in bench_pipe bench_nopipe bench_w5; do python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"], d.get("settle",{}).get("launches"))' gpurun_out/r03c/$f.json $f || exit 1; done
timeout -k 10 300 python tools/exp_stripes.py 50 20 > gpurun_out/r03c/stripes.jsonl 2>gpurun_out/r03c/stripes.err || exit 1
cat gpurun_out/r03c/stripes.jsonl
