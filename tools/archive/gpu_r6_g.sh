#!/bin/bash
# Round 6: vsa_bin_finish with two round trips (suite, then A/B of the
# per-rank step against the previous kernel build, libvsa_base.so), and the
# cfg-5 replay at 16 / 12 / 8 host threads after a warm call
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in libvsa_base.so libvectorscan_amd.so; do
    VSA_LIB_VARIANT=$v EXP_RANKS=8,1 EXP_MODES=pipe,pack1 timeout -k 10 200 python tools/exp_stripes.py 100 20 >> gpurun_out/fin_ab.jsonl 2>>gpurun_out/fin_ab.err || exit 1
  done
done
cat gpurun_out/fin_ab.jsonl
EXP_THREADS=16,12,8,16 timeout -k 10 300 python tools/exp_cfg5.py 20 > gpurun_out/cfg5_threads.jsonl 2>gpurun_out/cfg5_threads.err || exit 1
cat gpurun_out/cfg5_threads.jsonl
