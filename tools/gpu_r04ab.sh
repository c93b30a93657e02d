O=gpurun_out/r04ab
mkdir -p $O
AMD_LOG_LEVEL=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest_serial.log 2>&1
echo rc=$?
tail -3 $O/gputest_serial.log
grep -n "vsa:\|assert\|AssertionError" $O/gputest_serial.log | head
