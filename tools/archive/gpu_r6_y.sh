#!/bin/bash
# schedule feedback trace: 4 GiB FDR 5k, 200 launches, both rules
mkdir -p gpurun_out
HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 timeout -k 10 300 python tools/exp_fb_trace.py 200 > gpurun_out/fbt_gain.json 2> gpurun_out/fbt_gain.txt || { tail -5 gpurun_out/fbt_gain.txt; exit 1; }
HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 VSA_FB_GAIN_US=-1 timeout -k 10 300 python tools/exp_fb_trace.py 200 > gpurun_out/fbt_2pc.json 2> gpurun_out/fbt_2pc.txt || { tail -5 gpurun_out/fbt_2pc.txt; exit 1; }
HIP_FORCE_DEV_KERNARG=1 VSA_FB_TRACE=1 VSA_XCD_FEEDBACK=0 timeout -k 10 300 python tools/exp_fb_trace.py 100 > gpurun_out/fbt_off.json 2> gpurun_out/fbt_off.txt || { tail -5 gpurun_out/fbt_off.txt; exit 1; }
