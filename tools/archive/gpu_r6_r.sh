#!/bin/bash
# Round 6: pipelined corpus repeats with the record copies on a copy stream
# (beside the next scan): the hs / hsbench tests, then the bench line's
# end_to_end and cfg-5 proxy fields, twice
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "hs or corpus or bench or repeat" > gpurun_out/hstest.log 2>&1
rc=$?; echo "hs tests rc=$rc"; tail -3 gpurun_out/hstest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 500 python bench.py --no-cpu 2>/dev/null | tail -1 > gpurun_out/bench_e2e_$i.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_e2e_$i.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], 'e2e', d['end_to_end']['value'], d['end_to_end']['ms_per_pass'], d['end_to_end']['parity'], 'cfg5', d['end_to_end_cfg5proxy']['ms_per_gib'], d['end_to_end_cfg5proxy']['parity'])"
done
