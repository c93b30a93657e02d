set -e
O=gpurun_out/r04av; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k hsbench > $O/gputest_hsb.log 2>&1 || { tail -30 $O/gputest_hsb.log; exit 1; }
tail -1 $O/gputest_hsb.log
