timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; echo suite rc=$rc; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_bins.json 2>/dev/null && tail -1 gpurun_out/bench_bins.json | cut -c1-400
VSA_LIB_SORT=1 timeout -k 10 300 python bench.py --no-cpu 2>/dev/null | tail -1 | cut -c1-400
