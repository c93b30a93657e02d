#!/bin/bash
# Round-6 GPU check: suite, smoke, the default bench line (no CPU leg), the
# cfg-5 proxy's host-replay split (VSA_HOST_TIMING) and the per-rank stripe
# steps with the collective-buffer modes; logs under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --no-cpu ${BENCH_ARGS} 2>gpurun_out/bench.err | tail -1 > gpurun_out/bench.json || exit 1
cat gpurun_out/bench.json
VSA_HOST_TIMING=1 EXP_THREADS=16 timeout -k 10 300 python tools/exp_cfg5.py 10 > gpurun_out/cfg5.jsonl 2>gpurun_out/cfg5.err || exit 1
cat gpurun_out/cfg5.jsonl; grep -c . gpurun_out/cfg5.err; tail -4 gpurun_out/cfg5.err
timeout -k 10 300 python tools/exp_stripes.py 50 20 > gpurun_out/stripes.jsonl 2>gpurun_out/stripes.err || exit 1
cat gpurun_out/stripes.jsonl
