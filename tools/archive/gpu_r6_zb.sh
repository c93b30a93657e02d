#!/bin/bash
# the bench (pipelined) with the dynamic shares' per-launch trace, on and off
mkdir -p gpurun_out
VSA_FB_TRACE=1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 64 --warmup 32 > gpurun_out/bt_dyn.json 2> gpurun_out/bt_dyn.txt || { tail -5 gpurun_out/bt_dyn.txt; exit 1; }
VSA_FB_TRACE=1 VSA_DYN_SHARES=0 timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 64 --warmup 32 > gpurun_out/bt_off.json 2> gpurun_out/bt_off.txt || { tail -5 gpurun_out/bt_off.txt; exit 1; }
VSA_FB_TRACE=1 timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-cfg5 --no-ceiling --steps 64 --warmup 32 > gpurun_out/bt_dyn2.json 2> gpurun_out/bt_dyn2.txt || { tail -5 gpurun_out/bt_dyn2.txt; exit 1; }
tail -c 300 gpurun_out/bt_dyn.json gpurun_out/bt_off.json gpurun_out/bt_dyn2.json
