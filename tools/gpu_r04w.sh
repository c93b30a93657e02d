O=gpurun_out/r04w
mkdir -p $O
VSA_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "split_passes" -x -v --timeout 200 --timeout-method thread > $O/split_test.log 2>&1
echo rc=$?
