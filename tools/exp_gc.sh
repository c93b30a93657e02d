#!/bin/bash
# VSA_CONF_KERNEL=1 (16 scanning waves, candidate slabs, vsa_lit_confirm
# behind the scan) vs the default (15 scanners + a confirm wave): the FDR
# parity tests under it, then interleaved bench runs.
O=gpurun_out/r03
mkdir -p $O
VSA_CONF_KERNEL=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gc_tests.log 2>&1 || { tail -30 $O/gc_tests.log; exit 1; }
tail -1 $O/gc_tests.log
: > $O/gc_ab.jsonl
for r in 1 2 3; do
  for v in 0 1; do
    VSA_CONF_KERNEL=$v timeout -k 10 300 python bench.py --no-cpu --no-e2e 2>$O/gc.err | tail -1 > $O/gc.json || exit 1
    python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({"conf_kernel": int(sys.argv[2]), "round": int(sys.argv[3]), "step_ms": d["ms_per_step"], "kernel_ms": d["roofline"]["kernel_ms"], "value": d["value"], "parity": d["parity"]}))' $O/gc.json $v $r >> $O/gc_ab.jsonl || exit 1
  done
done
cat $O/gc_ab.jsonl
