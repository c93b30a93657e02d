set -e
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "class or shufti or truffle or verm" -x -q --timeout 300 --timeout-method thread > $O/class_tests.log 2>&1
tail -1 $O/class_tests.log
timeout -k 10 300 python -u tools/bench_configs.py --only 2 > $O/cfg2.jsonl 2>&1
VSA_XCD_FEEDBACK=0 timeout -k 10 300 python -u tools/bench_configs.py --only 2 > $O/cfg2_nofb.jsonl 2>&1
timeout -k 10 300 python -u tools/bench_configs.py --only 2 > $O/cfg2_b.jsonl 2>&1
