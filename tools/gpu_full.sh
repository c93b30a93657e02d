#!/bin/bash
# Whole GPU suite, then the default bench line; with "ab", also the bench
# under VSA_SYNC_BLOCK / VSA_LIB_SORT (blocking wait / library sort A/B).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/gputest.log
[ $rc -eq 0 ] || exit $rc
V="DEFAULT"
[ "$1" = "ab" ] && V="DEFAULT VSA_SYNC_BLOCK VSA_LIB_SORT"
for v in $V; do
  env $v=1 timeout -k 10 300 python bench.py --no-cpu 2>/dev/null | tail -1 > gpurun_out/bench_$v.json || exit 1
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"])' gpurun_out/bench_$v.json $v || exit 1
done
