# the ~1.4-rounds segment rule against the old balanced rule at stripe sizes
set -e
O=gpurun_out/seg; mkdir -p $O
for mib in 256 384 512 768 1024; do
  VSA_SEG_ROUNDS_OLD=1 timeout -k 10 120 python tools/exp_seg_small.py $mib | sed 's/^/old /' >> $O/rule.txt 2>&1
  timeout -k 10 120 python tools/exp_seg_small.py $mib | sed 's/^/new /' >> $O/rule.txt 2>&1
done
