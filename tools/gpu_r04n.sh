set -e
O=gpurun_out/r04n
mkdir -p $O
bash tools/gpu_round4.sh r04n suite
WORKLOAD=noodle GIB=1 timeout -k 10 200 python -u tools/exp_waves.py > $O/waves_noodle_1g.txt 2>&1
bash tools/gpu_round4.sh r04n configs bench
