#!/bin/bash
# Parity tests + headline bench + cfg1-3 lines (one GPU call).
set -e
OUT=gpurun_out/quick
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/bench.log 2>&1
timeout -k 10 300 python tools/bench_configs.py --steps 5 --warmup 1 > $OUT/configs.log 2>&1
VSA_FDR_DOMAIN=13 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_d13.log 2>&1
VSA_DEBUG_FLAGS=2 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_f2.log 2>&1
timeout -k 10 300 python tools/exp_confirm.py > $OUT/confirm.txt 2>&1
