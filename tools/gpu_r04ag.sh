set -e
# VSA_WG_K 2 against 1 on small launches of small blocks (32 / 128 MiB), x2
O=gpurun_out/r04ag; mkdir -p $O
for r in 1 2; do
  for K in 2 1; do
    for T in 32 128; do
      echo "# K=$K total $T MiB round $r" >> $O/wgk_small.txt
      VSA_WG_K=$K timeout -k 10 200 python -u tools/exp_blocks.py $T 2 16 64 >> $O/wgk_small.txt 2>> $O/wgk_small.err
    done
  done
done
cat $O/wgk_small.txt
