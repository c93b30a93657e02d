bash tools/profile.sh r02b && echo profile-ok && timeout -k 10 300 python tools/exp_blocks.py > gpurun_out/blocks.txt 2>&1 && echo blocks-ok
