#!/bin/bash
# The bench's N > 1 path (striping, packed all-gather, rank-0 merge and
# full-corpus parity) rehearsed on a one-GPU box: 2 ranks share cuda:0 over
# gloo.  The driver's multi-GPU runs use RCCL, one GPU per rank.
VSA_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu
