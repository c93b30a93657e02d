set -e
O=gpurun_out/r04m
mkdir -p $O
WORKLOAD=noodle GIB=1 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_noodle_1g.txt 2>&1
SIZES=128,512,1024,4096 VARIANTS="default VSA_STEAL_W=1 VSA_STEAL=2 VSA_STEAL=2,VSA_STEAL_W=1 default VSA_STEAL_W=1" bash tools/exp_launch_sweep.sh r04m 2> $O/sweep.err
bash tools/gpu_round4.sh r04m stripes
