#!/bin/bash
# SQ / LDS counters of the cfg-4 FDR scan kernel (one pass per counter set,
# kernel trace and counters in separate runs).  Usage: tools/pmc_fdr.sh TAG
# [extra env assignments are inherited].  Output: gpurun_out/pmc_<TAG>/
set -e
TAG=${1:-cur}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 2 --no-cpu --no-parity"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex vsa_lit_scan -f csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex vsa_lit_scan -f csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/t -o run -- $B > $OUT/t.log 2>&1
python3 tools/pmc_show.py $OUT
