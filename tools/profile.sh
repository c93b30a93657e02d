#!/bin/bash
# Profiling recipe for the bench workload (run on the GPU box from the repo
# root).  Kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in their own
# passes (TCC slots cannot hold both).  Outputs land in gpurun_out/prof_<tag>.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/bench_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/cfg -o run -- \
    python3 tools/bench_configs.py --steps 5 --warmup 1 > $OUT/configs_trace.log 2>&1
