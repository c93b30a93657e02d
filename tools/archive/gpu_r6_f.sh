#!/bin/bash
# Round 6: suite, the default bench line (CPU baseline included), configs
# 1 and 3, the cfg-5 proxy's replay at 16 / 12 / 8 host threads
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py 2>gpurun_out/bench_full.err | tail -1 > gpurun_out/bench_full.json || exit 1
cat gpurun_out/bench_full.json
timeout -k 10 300 python tools/bench_configs.py --only 1,3 > gpurun_out/cfg13.jsonl 2>gpurun_out/cfg13.err || exit 1
cat gpurun_out/cfg13.jsonl
EXP_THREADS=16,12,8 timeout -k 10 300 python tools/exp_cfg5.py 20 > gpurun_out/cfg5_threads.jsonl 2>gpurun_out/cfg5_threads.err || exit 1
cat gpurun_out/cfg5_threads.jsonl
