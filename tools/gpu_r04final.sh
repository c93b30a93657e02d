set -e
# final measurement set of round 4: GPU suite, default bench, rocprof trace +
# PMC passes of the bench, configs (each step under its own time limit)
timeout -k 10 120 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 tools/hip_lasterror_probe.cpp -o gpurun_out/probe && timeout -k 10 60 ./gpurun_out/probe > gpurun_out/probe.txt 2>&1
bash tools/gpu_round4.sh r04z suite bench
bash tools/profile.sh r04z
bash tools/gpu_round4.sh r04z configs
