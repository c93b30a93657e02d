#!/bin/bash
# Round 6 closing measurements: the default bench line (CPU baseline,
# end_to_end, cfg-5 proxy), the rank step at N = 1 / 2 / 4 / 8 as bench.py
# runs it (device kernel arguments, every 4th launch timed), the 10k / 20k
# literal sets at 512 MiB / 1 GiB / 4 GiB
mkdir -p gpurun_out/final
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 500 python bench.py 2>gpurun_out/final/bench.err | tail -1 > gpurun_out/final/bench.json || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], d['end_to_end']['ms_per_pass'], d['end_to_end_cfg5proxy']['ms_per_gib'], d['parity'])"
EXP_TIMING=4 EXP_MODES=pipe,pack1 timeout -k 10 300 python tools/exp_stripes.py 200 30 > gpurun_out/final/stripes.jsonl 2>gpurun_out/final/stripes.err || exit 1
cat gpurun_out/final/stripes.jsonl | cut -c1-200
for L in 10000 20000; do
  LITS=$L timeout -k 10 300 python tools/exp_sizes.py >> gpurun_out/final/large_sets.jsonl 2>>gpurun_out/final/large_sets.err || exit 1
done
cat gpurun_out/final/large_sets.jsonl
