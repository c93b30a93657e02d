#!/bin/bash
# Round 6: suite + smoke, bench, stripes with and without 2 reserved CUs
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --no-cpu 2>gpurun_out/bench.err | tail -1 > gpurun_out/bench.json || exit 1
cat gpurun_out/bench.json
for r in 0 2; do
  EXP_RESERVE=$r timeout -k 10 300 python tools/exp_stripes.py 50 20 > gpurun_out/stripes_res$r.jsonl 2>gpurun_out/stripes_res$r.err || exit 1
  echo "== reserve $r"; cat gpurun_out/stripes_res$r.jsonl
done
