#!/bin/bash
# GPU suite (optional), then the default bench line for the in-tree library
# and each experiment variant named on the command line (VSA_LIB_VARIANT,
# built by tools/build_variant.sh), on the same box.
#   tools/gpu_ab.sh [--tests] variant...
mkdir -p gpurun_out
if [ "$1" = "--tests" ]; then
  shift
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
fi
for v in default "$@" default; do
  lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
  VSA_LIB_VARIANT=$lib timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} 2>gpurun_out/bench_$v.err | tail -1 > gpurun_out/bench_$v.json || exit 1
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"], d["confirm_candidates"])' gpurun_out/bench_$v.json $v || exit 1
done
