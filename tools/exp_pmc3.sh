#!/bin/bash
# SQ counters + timing of the FDR scan kernel under debug flags
# (2 = no buckets / filter only, 8 = candidates detected but not extracted, 0 = full)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_exp3
mkdir -p $OUT
for f in 0 2 8; do
  VSA_DEBUG_FLAGS=$f timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_f$f.log 2>&1
  VSA_DEBUG_FLAGS=$f timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex vsa_lit_scan -f csv -d $OUT/f$f -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu > $OUT/f$f.log 2>&1
done
