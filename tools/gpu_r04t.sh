set -e
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -k "feedback or plan or stripe or hsbench or large" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in default VSA_XCD_FEEDBACK=0; do
    e=""; [ $v != default ] && e=$v
    env $e timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --no-parity > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
bash tools/gpu_round4.sh r04t stripes
