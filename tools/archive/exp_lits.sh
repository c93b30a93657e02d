#!/bin/bash
# kernel time vs literal-set size (4 GiB, FDR, adaptive confirm waves), then
# the confirm-wave phase counters (VSA_DEBUG_FLAGS=64 fixes the confirm-wave
# count, so set VSA_NCONF for those runs)
for n in 1000 5000 10000 20000 50000; do
  LITS=$n timeout -k 10 200 python3 tools/exp_counters.py | grep lits || exit 1
done
for n in 5000 20000; do
  nc=1; [ $n -gt 10000 ] && nc=2
  LITS=$n VSA_NCONF=$nc VSA_DEBUG_FLAGS=64 timeout -k 10 200 python3 tools/exp_counters.py || exit 1
done
