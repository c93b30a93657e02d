#!/bin/bash
# Launch breakdown (tools/exp_launch.py) under scheduling variants, to split
# a segment start's cost: default dynamic tickets, static assignment, fixed
# segment sizes, one ticket region.  One process per variant (the plan reads
# the variables when it is built).  Output: gpurun_out/<tag>/sweep.jsonl
TAG=${1:-r04b}
SIZES=${SIZES:-32,512,4096}
mkdir -p gpurun_out/$TAG
OUT=gpurun_out/$TAG/sweep.jsonl
: > $OUT
VARIANTS=${VARIANTS:-"default VSA_SCHED_OLD=1 VSA_STATIC_SEGS=1 VSA_SEG_KB=16 VSA_SEG_KB=32 VSA_SEG_KB=64 VSA_SEG_KB=256 VSA_REGIONS=1"}
for v in $VARIANTS; do
    [ "$v" = default ] && v=""
    v=${v//,/ }
    echo "variant: ${v:-default}" >&2
    env $v timeout -k 10 200 python -u tools/exp_launch.py --sizes $SIZES --extra "" --launches 5 \
        | sed "s/^{/{\"variant\": \"${v:-default}\", /" >> $OUT || exit 1
done
