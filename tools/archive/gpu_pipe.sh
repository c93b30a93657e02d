#!/bin/bash
# Pipelined vs one-at-a-time bench steps, the per-rank stripe table (sync and
# pipelined) and the N = 2 rehearsal (2 ranks on one GPU over gloo).
mkdir -p gpurun_out/pipe
timeout -k 10 300 python bench.py --no-cpu 2>gpurun_out/pipe/b1.err | tail -1 > gpurun_out/pipe/bench_pipe.json || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-pipeline 2>gpurun_out/pipe/b2.err | tail -1 > gpurun_out/pipe/bench_nopipe.json || exit 1
timeout -k 10 300 python bench.py --no-cpu --warmup 5 2>gpurun_out/pipe/b3.err | tail -1 > gpurun_out/pipe/bench_w5.json || exit 1
for f in bench_pipe bench_nopipe bench_w5; do python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"], d.get("settle",{}).get("launches"))' gpurun_out/pipe/$f.json $f || exit 1; done
timeout -k 10 300 python tools/exp_stripes.py 50 20 > gpurun_out/pipe/stripes.jsonl 2>gpurun_out/pipe/stripes.err || exit 1
cat gpurun_out/pipe/stripes.jsonl
VSA_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu > gpurun_out/pipe/n2.out 2> gpurun_out/pipe/n2.err || { tail -20 gpurun_out/pipe/n2.err; exit 1; }
tail -1 gpurun_out/pipe/n2.out
