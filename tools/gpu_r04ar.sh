set -e
# 30k / 40k literals (split passes): default against 1 / 2 / 3 confirm waves
O=gpurun_out/r04ar; mkdir -p $O
timeout -k 10 500 python -u tools/exp_xp_cost.py 30000 40000 > $O/xp_30k.jsonl 2> $O/xp_30k.err
cat $O/xp_30k.jsonl
