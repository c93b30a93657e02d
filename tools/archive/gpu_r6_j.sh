#!/bin/bash
# Round 6: the fused finish, second form (sort overlapped with the look-back, no ticket) -- its tests
# first, then the suite, then A/B against VSA_FUSED_FINISH=0 (the
# vsa_bin_finish launch): per-rank step at N = 8 / 1 and the bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fused or binned_sort or crowded or plan_pack or feedback" > gpurun_out/fusedtest.log 2>&1
rc=$?; echo "fused tests rc=$rc"; tail -15 gpurun_out/fusedtest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 0 1; do
    VSA_FUSED_FINISH=$f EXP_RANKS=8,1 EXP_MODES=pipe,pack1 timeout -k 10 200 python tools/exp_stripes.py 100 20 | sed "s/^{/{\"fused\": $f, /" >> gpurun_out/fused2_ab.jsonl 2>>gpurun_out/fused2_ab.err || exit 1
  done
done
cat gpurun_out/fused2_ab.jsonl
VSA_FUSED_FINISH=1 timeout -k 10 400 python bench.py --no-cpu --no-cfg5 2>gpurun_out/bench_f1.err | tail -1 > gpurun_out/bench_f1.json || exit 1
VSA_FUSED_FINISH=0 timeout -k 10 400 python bench.py --no-cpu --no-cfg5 2>gpurun_out/bench_f0.err | tail -1 > gpurun_out/bench_f0.json || exit 1
python3 -c "
import json
for f in ('gpurun_out/bench_f1.json','gpurun_out/bench_f0.json'):
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'], d.get('end_to_end',{}).get('ms_per_pass'))
"
