#!/bin/bash
# GPU run of the pure-literal hs API tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hs_lit.py tests/test_hsbench.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/hs_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/hs_gpu.log
exit $rc
