#!/bin/bash
# FDR cfg-4 kernel time with parts of the candidate path switched off
# (VSA_DEBUG_FLAGS, kernels.hip): 8 = no ring push (filter only), 128 =
# confirm wave drops gathered entries, 256 = 32-byte ring entries (wrong
# confirm keys), 16 = no confirm-queue push after the slot bitmap
mkdir -p gpurun_out
for f in 0 8 128 256 384 16; do
  if [ $f = 0 ]; then
    timeout -k 10 300 python bench.py --no-cpu > gpurun_out/cp_$f.json 2>/dev/null || exit 1
  else
    VSA_DEBUG_FLAGS=$f timeout -k 10 300 python bench.py --no-cpu --no-parity > gpurun_out/cp_$f.json 2>/dev/null || exit 1
  fi
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print("dbg", sys.argv[2], d["ms_per_step"], d["roofline"]["kernel_ms"], d["parity"])' gpurun_out/cp_$f.json $f || exit 1
done
