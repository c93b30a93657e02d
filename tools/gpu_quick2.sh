#!/bin/bash
# quick GPU check: FDR/Teddy parity tests, then literal-set-size sweep
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_flood.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/exp_lits.sh
