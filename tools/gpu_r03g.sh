#!/bin/bash
# cfg-5 replay A/B: parallel vs serial record map, alternating, 16 threads
mkdir -p gpurun_out/r03g
nproc > gpurun_out/r03g/nproc.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r03g/nproc.txt 2>/dev/null
for i in 1 2; do
  EXP_THREADS=16 timeout -k 10 300 python tools/exp_cfg5.py 20 64 0 > gpurun_out/r03g/par_$i.jsonl 2>/dev/null || exit 1
  VSA_MAP_SERIAL=1 EXP_THREADS=16 timeout -k 10 300 python tools/exp_cfg5.py 20 64 0 > gpurun_out/r03g/ser_$i.jsonl 2>/dev/null || exit 1
done
EXP_THREADS=16 timeout -k 10 300 python tools/exp_cfg5.py 20 4 1 > gpurun_out/r03g/par_d.jsonl 2>/dev/null || exit 1
VSA_MAP_SERIAL=1 EXP_THREADS=16 timeout -k 10 300 python tools/exp_cfg5.py 20 4 1 > gpurun_out/r03g/ser_d.jsonl 2>/dev/null || exit 1
cat gpurun_out/r03g/nproc.txt; for f in gpurun_out/r03g/*.jsonl; do echo "$f $(cat $f)"; done
