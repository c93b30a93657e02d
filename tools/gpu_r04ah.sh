set -e
# groups that can be runs cut at VSA_RUN_MAX blocks: GPU layout / run / stream
# parity, then A/B against the previous runtime (libvsa_prevrt.so) on 1-4 KiB
# blocks, x2
O=gpurun_out/r04ah; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "layout or run or stream or split or batch or block" > $O/gputest_runs.log 2>&1 || { tail -30 $O/gputest_runs.log; exit 1; }
tail -1 $O/gputest_runs.log
for r in 1 2; do
  for lib in libvsa_prevrt.so libvectorscan_amd.so; do
    echo "# $lib round $r" >> $O/runcap.txt
    VSA_LIB_VARIANT=$lib timeout -k 10 200 python -u tools/exp_blocks.py 1024 1 2 4 >> $O/runcap.txt 2>> $O/runcap.err
    VSA_LIB_VARIANT=$lib timeout -k 10 200 python -u tools/exp_blocks.py 128 1 >> $O/runcap.txt 2>> $O/runcap.err
  done
done
cat $O/runcap.txt
