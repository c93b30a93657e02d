#!/bin/bash
# dynamic shares at 1 GiB: noodle / Teddy / FDR, trace on and off
mkdir -p gpurun_out
for k in nood teddy fdr; do
  for d in 1 0; do
    EXP_LITS=$k EXP_MIB=1024 VSA_DYN_SHARES=$d HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 timeout -k 10 300 python tools/exp_fb_trace.py 120 > gpurun_out/t1g_${k}_$d.json 2> gpurun_out/t1g_${k}_$d.txt || { tail -5 gpurun_out/t1g_${k}_$d.txt; exit 1; }
  done
done
