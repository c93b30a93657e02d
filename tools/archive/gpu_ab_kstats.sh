#!/bin/bash
# Interleaved A/B of library variants by rocprofv3 kernel statistics: REPS
# rounds over default + the named variants (vectorscan_amd/libvsa_<name>.so),
# each a kernel-trace run of the bench line (BENCH_ARGS added); prints every
# run's average duration of the kernels whose names match KRE.
OUT=gpurun_out/${AB_OUT:-ab_kstats}
mkdir -p $OUT
export TMPDIR=/tmp
REPS=${REPS:-2}
KRE=${KRE:-vsa_}
for r in $(seq $REPS); do
  for v in default "$@"; do
    lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
    d=$OUT/${v}_$r
    VSA_LIB_VARIANT=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $d -o run -- \
        python3 bench.py --no-cpu --no-parity --no-e2e ${BENCH_ARGS} > $d.log 2>&1 || exit 1
    f=$(find $d -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" "$KRE" >> $OUT/summary.txt <<'P'
import csv, re, sys
for row in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], row["Name"]):
        print("%-8s %-40s calls %5s avg %9.1f ns" % (sys.argv[2], row["Name"][:40], row["Calls"], float(row["AverageNs"])))
P
    tail -1 $d.log | cut -c1-160 >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
