set -e
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "split or large" -x -v --timeout 300 --timeout-method thread > $O/split_tests.log 2>&1
timeout -k 10 600 python -u tools/exp_split.py 20000 30000 50000 > $O/split.jsonl 2> $O/split.err
timeout -k 10 300 python -u tools/bench_configs.py --only 4 > $O/cfg4.jsonl 2>&1
