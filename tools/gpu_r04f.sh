set -e
O=gpurun_out/r04f
mkdir -p $O
bash tools/gpu_round4.sh r04f suite
GIB=4 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_4g.txt 2>&1
SIZES=32,128,512,1024,4096 VARIANTS="default VSA_POOL_PM=0 VSA_POOL_PM=60 VSA_POOL_PM=250" bash tools/exp_launch_sweep.sh r04f 2> $O/sweep.err
timeout -k 10 200 python -u tools/bench_configs.py --only 3 > $O/cfg3_default.jsonl 2>&1
VSA_OLD_SORT=1 timeout -k 10 200 python -u tools/bench_configs.py --only 3 > $O/cfg3_oldsort.jsonl 2>&1
VSA_SCHED_OLD=1 timeout -k 10 200 python -u tools/bench_configs.py --only 3 > $O/cfg3_oldsched.jsonl 2>&1
bash tools/gpu_round4.sh r04f bench
