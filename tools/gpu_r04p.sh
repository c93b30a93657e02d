set -e
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -k "class or shufti or truffle or feedback" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/bench_configs.py --only 2 > $O/cfg2.jsonl 2>&1
VSA_XCD_FEEDBACK=0 timeout -k 10 300 python -u tools/bench_configs.py --only 2 > $O/cfg2_nofb.jsonl 2>&1
bash tools/gpu_round4.sh r04p configs bench
VSA_XCD_FEEDBACK=0 timeout -k 10 400 python -u bench.py --no-cpu --no-e2e > $O/bench_nofb.json 2> $O/bench_nofb.err
