#!/bin/bash
# Round 6: device timeline of bench.py's end_to_end passes (kernel and
# memory-copy trace): what runs between two corpus scans
mkdir -p gpurun_out/e2etl
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d gpurun_out/e2etl -o run -- python3 bench.py --no-cpu --no-cfg5 --steps 5 --warmup 5 > gpurun_out/e2etl/bench.log 2>&1 || exit 1
ls gpurun_out/e2etl/*/ 2>/dev/null | head; find gpurun_out/e2etl -name '*.csv' | head
