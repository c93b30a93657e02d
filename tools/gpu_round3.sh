#!/bin/bash
# Round-3 measurement set (each step under its own time limit, chained):
#   suite    the GPU test suite
#   blocks   block-size table with and without runs (tools/exp_blocks.py)
#   cfg5     hs corpus replay, one pass at a time vs pipelined (tools/exp_cfg5.py)
#   stripes  per-rank step at N = 1/2/4/8 stripe sizes (tools/exp_stripes.py)
#   dropin   drop-in per-call latency vs one CPU thread (tools/exp_dropin.py)
#   batcher  concurrent calls, plain vs batched (tools/exp_batcher.py)
#   noodle   cfg 1 at 4 GiB (tools/bench_configs.py --cfg1-gib 4)
#   ab       interleaved A/B of variant libraries (tools/gpu_abn.sh VARIANTS)
#   sortab   bench with the split / fused (VSA_SORT_FUSED) sort, pipelined or not
#   profile  rocprofv3 trace + PMC passes (tools/profile.sh r03)
#   tools/gpu_round3.sh suite blocks cfg5 ...
O=gpurun_out/r03
mkdir -p $O
for step in "$@"; do
  case $step in
    suite) timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }; tail -1 $O/gputest.log ;;
    blocks) timeout -k 10 300 python tools/exp_blocks.py > $O/blocks_runs.txt 2>&1 && VSA_NO_RUNS=1 timeout -k 10 300 python tools/exp_blocks.py > $O/blocks_noruns.txt 2>&1 || exit 1; cat $O/blocks_runs.txt $O/blocks_noruns.txt ;;
    cfg5) VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 64 0 > $O/cfg5.jsonl 2> $O/cfg5.err || exit 1; cat $O/cfg5.jsonl ;;
    stripes) timeout -k 10 300 python tools/exp_stripes.py 50 20 > $O/stripes.jsonl 2> $O/stripes.err || exit 1; cat $O/stripes.jsonl ;;
    dropin) timeout -k 10 600 python tools/exp_dropin.py > $O/dropin.jsonl 2> $O/dropin.err || exit 1; cat $O/dropin.jsonl ;;
    batcher) timeout -k 10 400 python tools/exp_batcher.py 200 > $O/batcher.jsonl 2> $O/batcher.err || exit 1; cat $O/batcher.jsonl ;;
    noodle) timeout -k 10 300 python tools/bench_configs.py --only 1 --cfg1-gib 4 --steps 20 --warmup 40 > $O/noodle.jsonl 2>&1 || exit 1; grep workload $O/noodle.jsonl ;;
    ab) REPS=${REPS:-3} bash tools/gpu_abn.sh $VARIANTS || exit 1 ;;
    sortab)
      for v in fused split; do
        e=""; [ $v = fused ] && e="VSA_SORT_FUSED=1"
        for m in pipe nopipe; do
          a=""; [ $m = nopipe ] && a="--no-pipeline"
          env $e timeout -k 10 300 python bench.py --no-cpu $a 2>$O/b.err | tail -1 > $O/sort_${v}_${m}.json || exit 1
          python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], "step", d["ms_per_step"], "kernel", d["roofline"]["kernel_ms"], "overhead_us", round((d["ms_per_step"]-d["roofline"]["kernel_ms"])*1e3,1), "parity", d["parity"])' $O/sort_${v}_${m}.json "$v $m" || exit 1
        done
      done ;;
    profile) bash tools/profile.sh r03 || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
