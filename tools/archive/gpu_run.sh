#!/bin/bash
# One GPU check: the GPU suite and the default bench line (no CPU leg);
# logs under gpurun_out/$1 (default: run).  Stops at the first failure.
OUT=gpurun_out/${1:-run}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} 2>$OUT/bench.err | tail -1 > $OUT/bench.json || exit 1
cat $OUT/bench.json
