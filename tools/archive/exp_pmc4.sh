#!/bin/bash
# SQ/LDS counters of the FDR scan (full run) + configs timing
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc4
mkdir -p $OUT
timeout -k 10 300 python tools/bench_configs.py --steps 5 --warmup 1 > $OUT/configs.log 2>&1
for f in 0 2; do
  VSA_DEBUG_FLAGS=$f timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex vsa_lit_scan -f csv -d $OUT/f$f -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu > $OUT/f$f.log 2>&1
done
