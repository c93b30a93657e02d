set -e
# 10k / 15k literals: the default (expansion off below 1e-3 candidates per
# byte) against expansion forced on with 1 / 2 / 3 confirm waves
O=gpurun_out/r04al; mkdir -p $O
timeout -k 10 400 python -u tools/exp_xp_cost.py 10000 15000 > $O/xp_10k.jsonl 2> $O/xp_10k.err
cat $O/xp_10k.jsonl
