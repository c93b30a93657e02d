#!/bin/bash
# Round 6: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) and
# sampled kernel timing in bench.py: bench lines with the setting 0 / 1
# interleaved, and the kernel time of the 512 MiB / 4 GiB scans under both
mkdir -p gpurun_out
for i in 1 2; do
  for k in 0 1; do
    HIP_FORCE_DEV_KERNARG=$k timeout -k 10 400 python bench.py --no-cpu --no-cfg5 --no-e2e 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernarg', $k, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])" || exit 1
  done
done
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k EXP_RANKS=8,1 EXP_MODES=sync,pack1 timeout -k 10 200 python tools/exp_stripes.py 200 30 | sed "s/^{/{\"kernarg\": $k, /" >> gpurun_out/kernarg_ab.jsonl || exit 1
done
cat gpurun_out/kernarg_ab.jsonl
