timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_flood.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; echo par rc=$rc; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
bash tools/exp_nconf.sh
