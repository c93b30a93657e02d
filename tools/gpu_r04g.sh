set -e
O=gpurun_out/r04g
mkdir -p $O
GIB=4 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_4g_pool.txt 2>&1
VSA_POOL_PM=0 GIB=4 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_4g_nopool.txt 2>&1
GIB=0.03125 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_32m_pool.txt 2>&1
VSA_POOL_PM=0 timeout -k 10 200 python -u tools/bench_configs.py --only 3 > $O/cfg3_nopool.jsonl 2>&1
VSA_POOL_PM=0 VSA_STEAL=0 timeout -k 10 200 python -u tools/bench_configs.py --only 3 > $O/cfg3_nopool_nosteal.jsonl 2>&1
