#!/bin/bash
# parallel map: cfg-5 tests, cfg-5 pass split; then noodle at 4 GiB with
# scheduling variants (the skeleton's cost split, verdict r02 item 9).
mkdir -p gpurun_out/r03f
timeout -k 10 600 python -u -m pytest tests/test_hsbench.py tests/test_hs_lit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f/test.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03f/test.log; [ $rc -eq 0 ] || exit $rc
VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 64 0 > gpurun_out/r03f/cfg5_h.jsonl 2> gpurun_out/r03f/cfg5_h.err || { tail -5 gpurun_out/r03f/cfg5_h.err; exit 1; }
VSA_HOST_TIMING=1 timeout -k 10 400 python tools/exp_cfg5.py 10 4 1 > gpurun_out/r03f/cfg5_d.jsonl 2> gpurun_out/r03f/cfg5_d.err || { tail -5 gpurun_out/r03f/cfg5_d.err; exit 1; }
cat gpurun_out/r03f/cfg5_h.jsonl gpurun_out/r03f/cfg5_d.jsonl
grep corpus_replay gpurun_out/r03f/cfg5_h.err | tail -3
for v in default SEG_KB=256 SEG_KB=512 SEG_KB=64 STATIC_SEGS=1 REGIONS=16 REGIONS=32; do
  if [ $v = default ]; then e=""; else e="VSA_$v"; fi
  env $e timeout -k 10 300 python tools/bench_configs.py --only 1 --cfg1-gib 4 --steps 20 --warmup 40 > gpurun_out/r03f/nood_$v.jsonl 2>&1 || { tail -5 gpurun_out/r03f/nood_$v.jsonl; exit 1; }
  echo "$v $(head -1 gpurun_out/r03f/nood_$v.jsonl)"
done
