#!/bin/bash
# SQ / LDS counters of the cfg-4 scan kernel for the in-tree library and
# each experiment variant (VSA_LIB_VARIANT), two passes each:
#   tools/exp_pmc_ab.sh variant...   -> gpurun_out/pmcab/<variant>_p{1,2}/
export TMPDIR=/tmp
OUT=gpurun_out/pmcab
mkdir -p $OUT
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for v in default "$@"; do
  lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
  i=1
  for P in "$P1" "$P2"; do
    VSA_LIB_VARIANT=$lib timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex vsa_lit_scan -f csv -d $OUT/${v}_p$i -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu --no-parity > $OUT/${v}_p$i.log 2>&1 || { echo "pmc $v pass $i failed"; tail -5 $OUT/${v}_p$i.log; exit 1; }
    i=$((i+1))
  done
  echo "pmc $v ok"
done
