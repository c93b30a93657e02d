set -e
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "split or large or expansion" -x -v --timeout 300 --timeout-method thread > $O/xp_tests.log 2>&1
timeout -k 10 600 python -u tools/exp_xp_cost.py 20000 50000 > $O/xp_cost.jsonl 2> $O/xp_cost.err
