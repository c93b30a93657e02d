#!/bin/bash
# replay: cfg-5 tests (sequence digests), then the pass split on the hsbench
# cfg-5 corpus shape and on a dense one.
mkdir -p gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_hsbench.py tests/test_hs_lit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03e/test.log; [ $rc -eq 0 ] || exit $rc
VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 64 0 > gpurun_out/r03e/cfg5_h.jsonl 2> gpurun_out/r03e/cfg5_h.err || { tail -5 gpurun_out/r03e/cfg5_h.err; exit 1; }
VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 4 1 > gpurun_out/r03e/cfg5_d.jsonl 2> gpurun_out/r03e/cfg5_d.err || { tail -5 gpurun_out/r03e/cfg5_d.err; exit 1; }
cat gpurun_out/r03e/cfg5_h.jsonl gpurun_out/r03e/cfg5_d.jsonl
grep corpus_replay gpurun_out/r03e/cfg5_h.err | tail -4
grep corpus_replay gpurun_out/r03e/cfg5_d.err | tail -4
