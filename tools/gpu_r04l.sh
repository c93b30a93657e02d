set -e
O=gpurun_out/r04l
mkdir -p $O
bash tools/profile.sh r04l
bash tools/gpu_round4.sh r04l configs
timeout -k 10 500 python -u tools/exp_launch.py --sizes 128,512,1024,4096 --extra noodle,teddy > $O/launch.jsonl 2> $O/launch.err
