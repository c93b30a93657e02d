#!/bin/bash
# Profiling recipe for the bench workload (run on the GPU box from the repo
# root).  Kernel trace + stats of the default bench command, then FETCH_SIZE,
# WRITE_SIZE and the SQ / LDS counters in their own passes (no counter pass
# shares a run with tracing), then the configs 1-3 lines with a kernel trace.
# Outputs land in gpurun_out/prof_<tag>.
set -e
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export HIP_FORCE_DEV_KERNARG=1  # as bench.py sets it for itself
B="python3 bench.py --steps 3 --warmup 2 --no-cpu --no-parity --no-e2e --no-cfg5 --no-ceiling"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python3 bench.py > $OUT/bench_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- $B > $OUT/bench_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- $B > $OUT/bench_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex vsa_lit_scan -f csv -d $OUT/sq -o run -- $B > $OUT/bench_sq.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/cfg -o run -- \
    python3 tools/bench_configs.py --steps 20 --warmup 20 > $OUT/configs_trace.log 2>&1
