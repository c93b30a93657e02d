set -e
# the GPU suite with its files in reverse order (a different allocation
# layout for every test: reads past a buffer would show as faults)
O=gpurun_out/r04aq; mkdir -p $O
F=$(ls tests/test_*.py | sort -r | tr '\n' ' ')
timeout -k 10 800 python -u -m pytest $F -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest_rev.log 2>&1 || { tail -40 $O/gputest_rev.log; exit 1; }
tail -1 $O/gputest_rev.log
