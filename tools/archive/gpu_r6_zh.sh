#!/bin/bash
# a second stream for the pipelined slot: does scan k+1 start in scan k's tail?
mkdir -p gpurun_out
export HIP_FORCE_DEV_KERNARG=1 EXP_TIMING=4 EXP_MODES=pipe,pack1 EXP_RANKS=8,4,1
for i in 1 2; do
  for s in 1 2; do
    EXP_STREAMS=$s timeout -k 10 300 python tools/exp_stripes.py 200 30 >> gpurun_out/streams_ab.jsonl 2>gpurun_out/streams.err || { tail -5 gpurun_out/streams.err; exit 1; }
  done
done
cut -c1-220 gpurun_out/streams_ab.jsonl
