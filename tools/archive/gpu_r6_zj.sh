#!/bin/bash
# the GPU suite with the dynamic shares on for every FDR launch >= 256 MiB
mkdir -p gpurun_out
VSA_DYN_SHARES=1 VSA_DYN_MIN_MIB=256 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_dyn.log 2>&1
rc=$?; tail -4 gpurun_out/gputest_dyn.log; exit $rc
