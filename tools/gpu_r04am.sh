set -e
# expansion threshold 4e-4: defaults at 10k / 15k / 20k / 5k, expansion tests
O=gpurun_out/r04am; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "scanner_expansion or large_literal or split_passes" > $O/gputest_xp.log 2>&1 || { tail -30 $O/gputest_xp.log; exit 1; }
tail -1 $O/gputest_xp.log
XP_COST_QUICK=1 timeout -k 10 300 python -u tools/exp_xp_cost.py 10000 15000 20000 5000 > $O/xp_thresh.jsonl 2> $O/xp_thresh.err
cat $O/xp_thresh.jsonl
