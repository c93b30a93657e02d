#!/bin/bash
# Round 6: device timeline of the N = 8 rank step (512 MiB, records packed
# for the collective) with and without the fused finish: rocprofv3 kernel
# trace of tools/exp_stripes.py, scan / sort / gaps per step
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
for f in 0 1; do
  VSA_FUSED_FINISH=$f EXP_RANKS=8 EXP_MODES=pack1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/tl/f$f -o run -- python3 tools/exp_stripes.py 100 20 > gpurun_out/tl/f$f.log 2>&1 || exit 1
done
for f in 0 1; do
  python3 tools/trace_gaps.py $(find gpurun_out/tl/f$f -name '*kernel_trace.csv' | head -1) 80
done
