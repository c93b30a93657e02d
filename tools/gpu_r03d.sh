#!/bin/bash
# runs (back-to-back blocks as one range): parity first, then the block-size
# table with and without runs, the cfg-5 pass split, bench A/B, stripes.
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hsbench.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03d/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_blocks.py > gpurun_out/r03d/blocks_runs.txt 2>&1 || exit 1
VSA_NO_RUNS=1 timeout -k 10 300 python tools/exp_blocks.py > gpurun_out/r03d/blocks_noruns.txt 2>&1 || exit 1
cat gpurun_out/r03d/blocks_runs.txt gpurun_out/r03d/blocks_noruns.txt
VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 > gpurun_out/r03d/cfg5.jsonl 2> gpurun_out/r03d/cfg5.err || { tail -5 gpurun_out/r03d/cfg5.err; exit 1; }
cat gpurun_out/r03d/cfg5.jsonl
timeout -k 10 300 python bench.py --no-cpu 2>gpurun_out/r03d/b1.err | tail -1 > gpurun_out/r03d/bench_pipe.json || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-pipeline 2>gpurun_out/r03d/b2.err | tail -1 > gpurun_out/r03d/bench_nopipe.json || exit 1
for f in bench_pipe bench_nopipe; do python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"], d.get("settle",{}).get("launches"))' gpurun_out/r03d/$f.json $f || exit 1; done
timeout -k 10 300 python tools/exp_stripes.py 50 20 > gpurun_out/r03d/stripes.jsonl 2>gpurun_out/r03d/stripes.err || exit 1
cat gpurun_out/r03d/stripes.jsonl
