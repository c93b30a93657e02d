#!/bin/bash
# quick GPU check: FDR-relevant parity tests, then bench timing + counters
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 bench.py --steps 20 --warmup 20 --no-cpu > gpurun_out/quick_bench.json || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/quick_bench.json')); print('step', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'GB/s', d['value'], 'parity', d['parity'], 'cand', d['confirm_candidates'])"
VSA_DEBUG_FLAGS=64 timeout -k 10 120 python3 tools/exp_counters.py
