set -e
O=gpurun_out/r04r
mkdir -p $O
for r in 1 2; do
  for v in default VSA_XCD_FEEDBACK=0 VSA_FB_DEV=0 VSA_FB_REFRESH=0 VSA_FB_PERIOD=8; do
    e=""; [ $v != default ] && e=$v
    env $e timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --no-parity > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
