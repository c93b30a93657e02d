"""bench.py's end_to_end line alone (hsbench block mode over the cfg-4
corpus: 4 x 1 GiB hs_scan blocks, every match delivered through the report
program), for the host-side split with VSA_HOST_TIMING=1 (per pass: wait +
copy, replay) on stderr.  python tools/exp_e2e.py [passes]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
lits = bench.make_literals(5000, seed=12)
total, nblocks = 4 << 30, 4
data = bench.make_corpus_device(torch, 0, total, total, lits, 5, 64 << 10, dev)
torch.cuda.synchronize()
out = bench.end_to_end(lits, data.data_ptr(), total // nblocks, nblocks, total, 0, reps)
out.pop("_digests", None)
out.pop("_counts", None)
print(json.dumps(out), flush=True)
