mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_gputest2.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r02_gputest2.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench1.json 2> gpurun_out/r02_bench1.err
echo "bench rc=$?"
cat gpurun_out/r02_bench1.json; tail -5 gpurun_out/r02_bench1.err
