set -e
# parity of the expansion tests on the new build, then an A/B: batched scanner
# expansion with 64-bit bit extraction (new, the default library) against the
# previous extraction (libvsa_prev.so), interleaved x3
O=gpurun_out/r04ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "scanner_expansion or split_passes or large_literal" > $O/gputest_xp.log 2>&1 || { tail -30 $O/gputest_xp.log; exit 1; }
tail -1 $O/gputest_xp.log
for r in 1 2 3; do
  for lib in libvsa_prev.so libvectorscan_amd.so; do
    XP_COST_QUICK=1 VSA_LIB_VARIANT=$lib timeout -k 10 240 python -u tools/exp_xp_cost.py 20000 50000 5000 >> $O/xp_ab.jsonl 2>> $O/xp_ab.err
  done
done
cat $O/xp_ab.jsonl
