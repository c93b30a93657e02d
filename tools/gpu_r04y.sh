O=gpurun_out/r04y
mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "feedback_512mib or split_passes" -x -v --timeout 300 --timeout-method thread > $O/repro.log 2>&1
echo rc=$?
