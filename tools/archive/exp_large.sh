#!/bin/bash
# large-set parity, then kernel time vs literal-set size
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "large or cfg3" -x -q --timeout 300 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; echo par rc=$rc; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
for n in 5000 10000 20000 50000; do LITS=$n timeout -k 10 200 python3 tools/exp_counters.py | grep lits || exit 1; done
