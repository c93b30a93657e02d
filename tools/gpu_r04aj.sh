set -e
# runs stolen like block parts: GPU layout / run / stream parity, then A/B
# against the build without it (libvsa_nors.so, -DVSA_NO_RUN_STEAL), x2
O=gpurun_out/r04aj; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "layout or run or stream or split or batch or block or hsbench" > $O/gputest_runsteal.log 2>&1 || { tail -30 $O/gputest_runsteal.log; exit 1; }
tail -1 $O/gputest_runsteal.log
for r in 1 2; do
  for lib in libvsa_nors.so libvectorscan_amd.so; do
    echo "# $lib round $r" >> $O/runsteal.txt
    VSA_LIB_VARIANT=$lib timeout -k 10 200 python -u tools/exp_blocks.py 1024 1 2 16 64 >> $O/runsteal.txt 2>> $O/runsteal.err
    VSA_LIB_VARIANT=$lib timeout -k 10 200 python -u tools/exp_blocks.py 128 2 16 >> $O/runsteal.txt 2>> $O/runsteal.err
    VSA_LIB_VARIANT=$lib timeout -k 10 200 python -u tools/bench_configs.py --only 4s >> $O/runsteal.txt 2>> $O/runsteal.err
  done
done
cat $O/runsteal.txt
