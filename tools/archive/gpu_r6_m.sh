#!/bin/bash
# Round 6: GPU suite with the fused finish as a per-context option (default
# off; its tests switch it on), then smoke
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
