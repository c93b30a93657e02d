#!/bin/bash
# Step timeline (kernel + memory-copy trace, no counters) of the per-rank
# stripe steps (tools/exp_stripes.py), then the stripe table itself untraced.
export TMPDIR=/tmp
OUT=gpurun_out/steptl
mkdir -p $OUT
timeout -k 10 300 python tools/exp_stripes.py 50 20 > $OUT/stripes.jsonl 2> $OUT/stripes.err || exit 1
cat $OUT/stripes.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/trace -o run -- python3 tools/exp_stripes.py 10 5 > $OUT/trace.log 2>&1 || exit 1
python3 tools/steptl.py $OUT
