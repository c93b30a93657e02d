#!/bin/bash
# SQ counters of the scan kernel under debug flags (filter only / no push / full)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_exp
mkdir -p $OUT
for f in 2 0; do
  VSA_DEBUG_FLAGS=$f timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex vsa_lit_scan -f csv -d $OUT/f$f -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu > $OUT/f$f.log 2>&1
done
