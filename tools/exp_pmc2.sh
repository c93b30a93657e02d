#!/bin/bash
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_exp2
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for f in 2 0; do
  VSA_DEBUG_FLAGS=$f timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex vsa_lit_scan -f csv -d $OUT/f$f -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu > $OUT/f$f.log 2>&1
done
