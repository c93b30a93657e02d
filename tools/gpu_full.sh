#!/bin/bash
# whole GPU suite, then the default bench line
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
