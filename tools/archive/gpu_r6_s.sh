#!/bin/bash
# Round 6: where the end-to-end pass goes now (copies on a copy stream):
# the library's per-pass host timing (VSA_HOST_TIMING) of bench.py's
# end_to_end field
mkdir -p gpurun_out
VSA_HOST_TIMING=1 timeout -k 10 500 python bench.py --no-cpu --no-cfg5 > gpurun_out/e2e_timing.json 2> gpurun_out/e2e_timing.err || exit 1
tail -1 gpurun_out/e2e_timing.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['kernel_ms'], 'e2e', d['end_to_end']['ms_per_pass'])"
grep "corpus_scan_repeats" gpurun_out/e2e_timing.err | tail -12
grep "corpus_replay" gpurun_out/e2e_timing.err | tail -4
