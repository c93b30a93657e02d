#!/bin/bash
# kernel time vs confirm waves per workgroup and literal-set size (4 GiB, FDR)
for n in 20000 5000 10000 50000; do
  for nc in 1 2 3; do
    echo "== lits $n nconf $nc"
    LITS=$n VSA_NCONF=$nc timeout -k 10 200 python3 tools/exp_counters.py 2>/dev/null | head -1 || exit 1
  done
done
