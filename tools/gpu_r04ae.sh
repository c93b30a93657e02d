set -e
# cfg4s (a 1 GiB stream of 16 KiB / 1 MiB writes): scheduling knobs
O=gpurun_out/r04ae; mkdir -p $O
for e in "X=0" "VSA_NO_RUNS=1" "VSA_WG_K=1" "VSA_WG_MAX_KIB=1024" "VSA_WG_MAX_KIB=1024 VSA_WG_K=1" "VSA_STEAL=0" "X=0"; do
  echo "# $e" >> $O/knobs.jsonl
  env $e timeout -k 10 200 python -u tools/bench_configs.py --only 4s >> $O/knobs.jsonl 2>> $O/knobs.err
done
cat $O/knobs.jsonl
