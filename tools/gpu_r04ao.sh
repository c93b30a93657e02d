set -e
# stealing knobs at 512 MiB (the N = 8 stripe) and 4 GiB, clock settled, x2
O=gpurun_out/r04ao; mkdir -p $O
for r in 1 2; do
  for e in "VSA_STEAL=4" "VSA_STEAL=2" "VSA_STEAL=8" "VSA_STEAL=1" "VSA_STEAL_W=0"; do
    for m in 512 4096; do
      env SETTLE=300 $e timeout -k 10 120 python -u tools/exp_seg_small.py $m >> $O/steal.txt 2>> $O/steal.err
    done
  done
done
cat $O/steal.txt
