timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; echo suite rc=$?; tail -3 gpurun_out/gputest.log
for n in 5000 10000 20000; do LITS=$n VSA_DEBUG_FLAGS=64 timeout -k 10 200 python3 tools/exp_counters.py || exit 1; done
