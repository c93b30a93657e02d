#!/bin/bash
# GPU suite, then the pipelined bench A/B + stripes + N=2 rehearsal
# (tools/gpu_pipe.sh), then the drop-in per-call costs.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pipe.sh || exit 1
timeout -k 10 600 python tools/exp_dropin.py > gpurun_out/dropin.jsonl 2> gpurun_out/dropin.err || { tail -5 gpurun_out/dropin.err; exit 1; }
cat gpurun_out/dropin.jsonl
bash tools/gpu_hsbench.sh cfg5 || exit 1
