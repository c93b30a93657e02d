#!/bin/bash
# Interleaved A/B of library variants on many-block scans (tools/exp_blocks.py,
# 1 GiB cut into CHUNKS KiB blocks; NO_RUNS=1 for the per-block path).
OUT=gpurun_out/${AB_OUT:-ab_blocks}
mkdir -p $OUT
for r in $(seq ${REPS:-2}); do
  for v in default "$@"; do
    lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
    echo "== $v" >> $OUT/blocks.txt
    env ${NO_RUNS:+VSA_NO_RUNS=1} VSA_LIB_VARIANT=$lib timeout -k 10 200 python tools/exp_blocks.py 1024 ${CHUNKS:-2 16 64} >> $OUT/blocks.txt 2>>$OUT/err.log || exit 1
  done
done
cat $OUT/blocks.txt
