set -e
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -k "feedback or plan or stripe or hsbench" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu --no-e2e > $O/bench_fb_$r.json 2> $O/bench_fb_$r.err
  VSA_XCD_FEEDBACK=0 timeout -k 10 400 python -u bench.py --no-cpu --no-e2e > $O/bench_nofb_$r.json 2> $O/bench_nofb_$r.err
done
timeout -k 10 300 python -u tools/bench_configs.py --only 3 > $O/cfg3.jsonl 2>&1
VSA_NCONF=2 timeout -k 10 300 python -u tools/bench_configs.py --only 3 > $O/cfg3_nc2.jsonl 2>&1
VSA_XP=1 timeout -k 10 300 python -u tools/bench_configs.py --only 3 > $O/cfg3_xp.jsonl 2>&1
