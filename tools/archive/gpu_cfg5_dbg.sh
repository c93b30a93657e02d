mkdir -p gpurun_out
for mode in plain torchwork; do
  echo "== new replay $mode"; VSA_HOST_TIMING=1 timeout -k 10 200 python tools/exp_cfg5_bench.py $mode 2> gpurun_out/c5_new_$mode.err || exit 1
  grep corpus_replay gpurun_out/c5_new_$mode.err | tail -2
  echo "== unit replay $mode"; VSA_REPLAY_UNITS=1 VSA_HOST_TIMING=1 timeout -k 10 200 python tools/exp_cfg5_bench.py $mode 2> gpurun_out/c5_old_$mode.err || exit 1
  grep corpus_replay gpurun_out/c5_old_$mode.err | tail -2
done
