#!/bin/bash
# Round-4 measurement set (each step under its own time limit, chained; the
# script stops at the first failing step):
#   suite    the GPU test suite
#   bench    the default bench.py line
#   sortab   bench.py with the staged sort (one vsa_bin_finish launch) and the
#            round-3 chain (VSA_OLD_SORT=1), interleaved x REPS
#   sweep    launch breakdown under scheduling variants (tools/exp_launch_sweep.sh)
#   launch   launch breakdown of the default build (tools/exp_launch.py)
#   dropin   small drop-in calls from POSIX threads: GPU / batcher / CPU
#   stripes  per-rank step at N = 1/2/4/8 stripe sizes (tools/exp_stripes.py)
#   configs  tools/bench_configs.py (cfg 1-3, 4s)
#   tools/gpu_round4.sh TAG step...
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for step in "$@"; do
  case $step in
    suite) timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }; tail -1 $O/gputest.log ;;
    bench) timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }; cat $O/bench.json ;;
    sortab)
      for r in $(seq ${REPS:-2}); do
        for v in new old; do
          e=""; [ $v = old ] && e="VSA_OLD_SORT=1"
          env $e timeout -k 10 300 python -u bench.py --no-cpu --no-e2e > $O/sortab_$v.$r.json 2> $O/sortab_$v.$r.err || { tail $O/sortab_$v.$r.err; exit 1; }
          python3 -c "import json,sys;d=json.load(open('$O/sortab_$v.$r.json'));print('$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])"
        done
      done ;;
    sweep) SIZES=${SIZES:-32,512,4096} bash tools/exp_launch_sweep.sh $TAG 2> $O/sweep.err || { tail $O/sweep.err; exit 1; } ;;
    launch) timeout -k 10 400 python -u tools/exp_launch.py > $O/launch.jsonl 2> $O/launch.err || { tail $O/launch.err; exit 1; } ;;
    dropin) timeout -k 10 300 ./tools/dropin_threads ${DROPIN_SECS:-0.3} 32 > $O/dropin_threads.jsonl 2> $O/dropin.err || { tail $O/dropin.err; exit 1; } ;;
    stripes) timeout -k 10 300 python tools/exp_stripes.py 50 20 > $O/stripes.jsonl 2> $O/stripes.err || { tail $O/stripes.err; exit 1; }; cat $O/stripes.jsonl ;;
    configs) timeout -k 10 500 python tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail $O/configs.err; exit 1; }; cat $O/configs.jsonl ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
