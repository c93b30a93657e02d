set -e
O=gpurun_out/r04x
mkdir -p $O
bash tools/gpu_round4.sh r04x suite
WORKLOAD=teddy GIB=1 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_teddy_1g.txt 2>&1
bash tools/gpu_round4.sh r04x configs
