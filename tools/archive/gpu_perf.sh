#!/bin/bash
# GPU suite, then the bench line, the configs 1-3 lines and the block-size
# table (kernel / wall) -- the numbers DESIGN.md section 5 quotes
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; echo suite rc=$rc; tail -2 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu 2>/dev/null | tail -1 > gpurun_out/bench.json || exit 1
python -c 'import json; d=json.load(open("gpurun_out/bench.json")); print("bench", d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["parity"])' || exit 1
timeout -k 10 300 python tools/bench_configs.py --steps 20 --warmup 20 > gpurun_out/configs.jsonl 2>&1 || exit 1
python - <<'P' || exit 1
import json
for l in open("gpurun_out/configs.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["workload"][:60], d.get("kernel_ms"), d.get("value"))
P
timeout -k 10 300 python tools/exp_blocks.py || exit 1
