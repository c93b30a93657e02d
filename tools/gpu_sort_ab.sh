# GPU suite, then the bench under the default path and two A/B switches
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; echo suite rc=$rc; tail -3 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
for v in DEFAULT VSA_SYNC_BLOCK VSA_LIB_SORT DEFAULT; do
  env $v=1 timeout -k 10 300 python bench.py --no-cpu 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"])' || exit 1
done
