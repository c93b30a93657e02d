#!/bin/bash
# Round 6: the bench with the host-replay split of its cfg-5 proxy
# (VSA_HOST_TIMING), then the cfg-2 class-scan A/B against the round-4 build
# (tools/ab_build_r04.sh), interleaved three times on this box.
mkdir -p gpurun_out
VSA_HOST_TIMING=1 timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err || exit 1
tail -1 gpurun_out/bench_t.json
grep -c "corpus_scan_repeats" gpurun_out/bench_t.err; grep "corpus_scan_repeats\|corpus_replay_blocks" gpurun_out/bench_t.err | tail -6
: > gpurun_out/class_ab.jsonl
for i in 1 2 3; do
  timeout -k 10 150 python tools/exp_class_ab.py ab/r04 r04 >> gpurun_out/class_ab.jsonl 2>>gpurun_out/class_ab.err || exit 1
  timeout -k 10 150 python tools/exp_class_ab.py . r06 >> gpurun_out/class_ab.jsonl 2>>gpurun_out/class_ab.err || exit 1
done
cat gpurun_out/class_ab.jsonl
