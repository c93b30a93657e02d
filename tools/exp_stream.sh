#!/bin/bash
set -e
OUT=gpurun_out/stream
mkdir -p $OUT
timeout -k 10 300 python tools/bench_configs.py --only 4s --steps 3 --warmup 1 > $OUT/stream.log 2>&1
