#!/bin/bash
# 20k-literal regime: expansion ILP (EXP_U variants) and more confirm waves
# on a domain-13 table (frees 64 KiB of LDS); 5k as the regression check
run() { echo "== $*"; env "$@" timeout -k 10 200 python3 tools/exp_counters.py | head -1 || exit 1; }
for n in 20000 5000; do
  run LITS=$n X=0
  run LITS=$n VSA_LIB_VARIANT=libvsa_exp2.so
  run LITS=$n VSA_LIB_VARIANT=libvsa_exp4.so
  run LITS=$n VSA_FDR_DOMAIN=13 VSA_NCONF=1
  run LITS=$n VSA_FDR_DOMAIN=13 VSA_NCONF=2
  run LITS=$n VSA_FDR_DOMAIN=13 VSA_NCONF=4
  run LITS=$n VSA_FDR_DOMAIN=13 VSA_NCONF=4 VSA_LIB_VARIANT=libvsa_exp4.so
done
