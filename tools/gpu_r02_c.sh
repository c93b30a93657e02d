# round-2 GPU check: new flood tests first, then the whole GPU suite
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flood.py tests/test_gpu_replay.py tests/test_gpu_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_flood.log 2>&1
rc=$?; echo "flood rc=$rc"; tail -25 gpurun_out/r02_flood.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_gputest3.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/r02_gputest3.log
exit $rc
