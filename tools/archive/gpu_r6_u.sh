#!/bin/bash
# Round 6: where a launch's fixed costs go now (diagnostic build's wave log:
# start, wave tail, last confirm batch) at 512 MiB / 1 GiB / 4 GiB, with
# device kernel arguments (as bench.py) and without
mkdir -p gpurun_out
for k in 1 0; do
  HIP_FORCE_DEV_KERNARG=$k VSA_LIB_VARIANT=libvsa_diag.so WL=fdr5k timeout -k 10 300 python tools/exp_overhead.py 2>/dev/null | sed "s/^{/{\"kernarg\": $k, /" >> gpurun_out/overhead.jsonl || exit 1
done
cat gpurun_out/overhead.jsonl
