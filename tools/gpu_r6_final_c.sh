#!/bin/bash
# Round 6 closing measurements on the final code: the default bench line,
# its kernel trace + stats, FETCH / WRITE PMC passes, the rank step table
set -e
mkdir -p gpurun_out/final_c
O=gpurun_out/final_c
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
timeout -k 10 500 python bench.py 2>$O/bench.err | tail -1 > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], d['end_to_end']['ms_per_pass'], d['end_to_end_cfg5proxy']['ms_per_gib'], d['parity'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 bench.py --no-cpu --no-e2e --no-cfg5 > $O/bench_trace.log 2>&1
tail -1 $O/bench_trace.log | cut -c1-200
B="python3 bench.py --steps 3 --warmup 2 --no-cpu --no-parity --no-e2e --no-cfg5 --no-ceiling"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $B > $O/bench_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- $B > $O/bench_write.log 2>&1
EXP_TIMING=4 EXP_MODES=pipe,pack1 timeout -k 10 300 python tools/exp_stripes.py 200 30 > $O/stripes.jsonl 2>$O/stripes.err
cut -c1-200 $O/stripes.jsonl
