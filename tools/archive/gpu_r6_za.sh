#!/bin/bash
# dynamic shares trace: per-launch XCD deviations and device weights (4 GiB FDR 5k)
mkdir -p gpurun_out
HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 timeout -k 10 300 python tools/exp_fb_trace.py 150 > gpurun_out/dyn_trace.json 2> gpurun_out/dyn_trace.txt || { tail -5 gpurun_out/dyn_trace.txt; exit 1; }
HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 VSA_DYN_SHARES=0 timeout -k 10 300 python tools/exp_fb_trace.py 150 > gpurun_out/dyn_off_trace.json 2> gpurun_out/dyn_off_trace.txt || { tail -5 gpurun_out/dyn_off_trace.txt; exit 1; }
EXP_MIB=512 HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 timeout -k 10 300 python tools/exp_fb_trace.py 150 > gpurun_out/dyn_trace512.json 2> gpurun_out/dyn_trace512.txt || { tail -5 gpurun_out/dyn_trace512.txt; exit 1; }
EXP_MIB=512 HIP_FORCE_DEV_KERNARG=1 VSA_DYN_SHARES=0 timeout -k 10 300 python tools/exp_fb_trace.py 150 > gpurun_out/dyn_off_trace512.json 2> gpurun_out/dyn_off_trace512.txt || { tail -5 gpurun_out/dyn_off_trace512.txt; exit 1; }
