set -e
# VSA_WG_K (per-workgroup list sizing: groups of small blocks up to
# r / (K x waves)) 2 (default) against 1, interleaved x2: blocks of 2 KiB ..
# 256 MiB, the cfg4s streams, the default bench kernel
O=gpurun_out/r04af; mkdir -p $O
for r in 1 2; do
  for K in 2 1; do
    echo "# K=$K round $r" >> $O/wgk.txt
    VSA_WG_K=$K timeout -k 10 300 python -u tools/exp_blocks.py >> $O/wgk.txt 2>> $O/wgk.err
    VSA_WG_K=$K timeout -k 10 200 python -u tools/bench_configs.py --only 4s >> $O/wgk.txt 2>> $O/wgk.err
    VSA_WG_K=$K timeout -k 10 300 python -u bench.py --no-cpu --no-e2e >> $O/wgk.txt 2>> $O/wgk.err
  done
done
cat $O/wgk.txt
