set -e
O=gpurun_out/r04j
mkdir -p $O
bash tools/gpu_round4.sh r04j suite
timeout -k 10 600 python -u tools/exp_xp_cost.py 20000 50000 > $O/xp_cost.jsonl 2> $O/xp_cost.err
