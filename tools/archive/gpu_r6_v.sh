#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hsbench.py -m gpu -x -v --timeout 200 --timeout-method thread -k "few_large or ragged or cfg5" > gpurun_out/hsb.log 2>&1
rc=$?; tail -8 gpurun_out/hsb.log; exit $rc
