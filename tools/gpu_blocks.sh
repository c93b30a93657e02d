timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_configs.py tests/test_hsbench.py tests/test_hs_lit.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; echo par rc=$rc; tail -5 gpurun_out/par.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_blocks.py && bash tools/gpu_hsbench.sh
