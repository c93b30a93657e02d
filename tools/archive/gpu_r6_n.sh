#!/bin/bash
# Round 6: what sits between two scans (the kernel boundary, 7-9 us before
# a 512 MiB scan): the per-rank step at N = 8 (pack1) with the timing events
# on every dispatch / none, and with the runtime's kernarg and signal knobs
mkdir -p gpurun_out
run() { env "$@" EXP_RANKS=8 EXP_MODES=pack1,pipe timeout -k 10 200 python tools/exp_stripes.py 300 30 | sed "s/^{/{\"env\": \"$*\", /" >> gpurun_out/gap_ab.jsonl 2>>gpurun_out/gap_ab.err; }
for i in 1 2; do
  run VSA_KTIME_EVERY=1 || exit 1
  run VSA_KTIME_EVERY=100000 || exit 1
  run HIP_FORCE_DEV_KERNARG=1 || exit 1
  run HIP_FORCE_DEV_KERNARG=0 || exit 1
  run ROC_SYSTEM_SCOPE_SIGNAL=0 || exit 1
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/gap_ab.jsonl'):
    r = json.loads(l)
    d[(r['env'], r['mode'])].append(r['step_ms'])
for k in sorted(d):
    print(k, d[k])
PY
