O=gpurun_out/r04ac
mkdir -p $O
VSA_PRINT_LAUNCH=1 AMD_LOG_LEVEL=2 AMD_SERIALIZE_KERNEL=3 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -l --timeout 300 --timeout-method thread > $O/gputest_serial.log 2>&1
echo rc=$?
tail -3 $O/gputest_serial.log
