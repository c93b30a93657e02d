#!/bin/bash
# Round 6: vsa_bin_finish's sorting networks on DPP / swizzle strides, in
# lockstep over passes (new test first, then the suite), then A/B against
# the previous kernel build (libvsa_base.so): the per-rank step (FDR 5k) and
# configs 1 / 3 (dense records: wall_ms_per_call includes the sort)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "binned_sort or crowded" > gpurun_out/sorttest.log 2>&1
rc=$?; echo "sort tests rc=$rc"; tail -3 gpurun_out/sorttest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in libvsa_base.so libvectorscan_amd.so; do
    VSA_LIB_VARIANT=$v EXP_RANKS=8,1 EXP_MODES=pack1 timeout -k 10 200 python tools/exp_stripes.py 100 20 >> gpurun_out/fin2_ab.jsonl 2>>gpurun_out/fin2_ab.err || exit 1
    echo "{\"lib\": \"$v\"}" >> gpurun_out/fin2_cfg.jsonl
    VSA_LIB_VARIANT=$v timeout -k 10 300 python tools/bench_configs.py --only 1,3 >> gpurun_out/fin2_cfg.jsonl 2>>gpurun_out/fin2_ab.err || exit 1
  done
done
cat gpurun_out/fin2_ab.jsonl
python3 -c "
import json
for l in open('gpurun_out/fin2_cfg.jsonl'):
    d=json.loads(l)
    print(d.get('lib') or (d['workload'], d['kernel_ms'], d['wall_ms_per_call']))
"
timeout -k 10 300 python tools/exp_dense.py 6000 > gpurun_out/dense.jsonl 2>gpurun_out/dense.err || exit 1
cat gpurun_out/dense.jsonl
