#!/bin/bash
# push vs confirm cost split: 16 = the confirm wave expands and prefilters
# but confirms nothing; 64 = confirm-wave phase counters (cycles)
for v in "VSA_DEBUG_FLAGS=16" "VSA_DEBUG_FLAGS=64"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, '.')
import numpy as np, torch, bench, vectorscan_amd as vsa
ctx = vsa.Context(0); lits = bench.make_literals(5000, seed=12); blob = vsa.hwlm_build(lits)
db = vsa.Database(ctx, blob); n = 4 << 30; bl = n // 4
data = bench.make_corpus_device(torch, 0, n, n, lits, 5, 64 << 10, torch.device('cuda', 0))
torch.cuda.synchronize()
ks = []
for i in range(30):
    ctx.scan_blocks(db, data.data_ptr(), [0, bl, 2*bl, 3*bl], [bl]*4); ks.append(ctx.kernel_ms())
print('kernel ms %.4f' % np.mean(ks[10:]), 'cand', ctx.candidates(), 'counters', ctx.debug_counters())
" || exit 1
done
