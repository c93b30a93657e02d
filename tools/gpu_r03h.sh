#!/bin/bash
# rotated-lane spill: full GPU suite, interleaved A/B against the previous
# kernel (libvsa_prev.so), then the cfg-5 map A/B.
mkdir -p gpurun_out/r03h
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03h/gputest.log; [ $rc -eq 0 ] || exit $rc
REPS=3 bash tools/gpu_abn.sh prev || exit 1
bash tools/gpu_r03g.sh
