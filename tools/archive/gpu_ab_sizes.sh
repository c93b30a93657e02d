#!/bin/bash
# Interleaved A/B of library variants on the cfg-4 scan at 512 MiB / 1 GiB /
# 4 GiB (tools/exp_sizes.py): REPS rounds over default + the named variants
# (vectorscan_amd/libvsa_<name>.so, tools/build_variant.sh).
OUT=gpurun_out/${AB_OUT:-ab_sizes}
mkdir -p $OUT
REPS=${REPS:-3}
for r in $(seq $REPS); do
  for v in default "$@"; do
    lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
    VSA_LIB_VARIANT=$lib timeout -k 10 120 python tools/exp_sizes.py 2>>$OUT/err.log >> $OUT/sizes.jsonl || exit 1
  done
done
python3 - $OUT/sizes.jsonl <<'P'
import json, statistics, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for v in dict.fromkeys(r["variant"] for r in rows):
    rs = [r for r in rows if r["variant"] == v]
    print("%-24s " % v + "  ".join("%s %.1f %s" % (k, statistics.median(r[k] for r in rs),
          [r[k] for r in rs]) for k in ("us_512", "us_1024", "us_4096")))
P
