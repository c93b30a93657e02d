#!/bin/bash
mkdir -p gpurun_out
HIP_FORCE_DEV_KERNARG=1 VSA_LIB_VARIANT=libvsa_diag.so timeout -k 10 300 python tools/exp_wg_spread.py > gpurun_out/wg_spread.jsonl 2>gpurun_out/wg_spread.err || { tail -5 gpurun_out/wg_spread.err; exit 1; }
VSA_XCD_FEEDBACK=1 HIP_FORCE_DEV_KERNARG=1 VSA_LIB_VARIANT=libvsa_diag.so timeout -k 10 300 python tools/exp_wg_spread.py >> gpurun_out/wg_spread.jsonl 2>>gpurun_out/wg_spread.err || exit 1
cat gpurun_out/wg_spread.jsonl
