#!/bin/bash
# What bounds the FDR filter: filter-only timing (flags 2) for the default
# build, with all lookups broadcast (no LDS bank conflicts, same VALU), and
# with 32 extra VALU ops per iteration (libvsa_x32.so).
set -e
OUT=gpurun_out/bound
mkdir -p $OUT
run() { timeout -k 10 200 env "$@" python bench.py --steps 5 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['roofline']['kernel_ms'])"; }
{
run VSA_DEBUG_FLAGS=2
run VSA_DEBUG_FLAGS=2 VSA_EXP_DMASK_ZERO=1
run VSA_DEBUG_FLAGS=2 VSA_LIB_VARIANT=libvsa_x32.so
run VSA_DEBUG_FLAGS=2 VSA_LIB_VARIANT=libvsa_x32.so VSA_EXP_DMASK_ZERO=1
run VSA_DEBUG_FLAGS=0
} > $OUT/bound.txt 2>&1
