cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/sortprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/sortprof.log 2>&1
rc=$?; echo rc=$rc; find $GRAFT_REPO_ROOT/gpurun_out/sortprof -name '*kernel_stats.csv' | head -1 | xargs cut -d, -f1-5 | cut -c1-160
