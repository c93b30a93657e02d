set -e
O=gpurun_out/r04i
mkdir -p $O
GIB=4 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_4g_fb.txt 2>&1
VSA_XCD_FEEDBACK=0 GIB=4 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_4g_nofb.txt 2>&1
SIZES=128,512,1024,4096 VARIANTS="default VSA_XCD_FEEDBACK=0 default VSA_XCD_FEEDBACK=0" bash tools/exp_launch_sweep.sh r04i 2> $O/sweep.err
timeout -k 10 200 python -u tools/bench_configs.py --only 3 > $O/cfg3.jsonl 2>&1
bash tools/gpu_round4.sh r04i bench
