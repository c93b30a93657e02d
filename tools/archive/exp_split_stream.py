"""Diagnostic: the stream part of tests/test_gpu_parity.py::test_gpu_split_passes
for one literal count, with the split passes on or off (VSA_SPLIT in the
environment), VSA_DEBUG=1 printing the failing HIP call.  The rng is
replayed exactly as the test draws it.  python tools/exp_split_stream.py N"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import oracle  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402
from test_gpu_parity import rand_lits, rand_data  # noqa: E402

nlits = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
rng = random.Random(5300 + nlits)
lits = rand_lits(rng, nlits, minlen=1 if nlits == 1 else 2, maxlen=8, msk_frac=0.3)
blob = vsa.hwlm_build(lits, engine_hint=0, allow_noodle=False)
sizes = [0, 1, 2, 7, 15, 16, 17, 100, 1023, 1024, 1025, 2047, 3000, 9000, 40000]
bufs = [rand_data(rng, rng.choice(sizes)) for _ in range(1200)]
starts = [rng.choice([0, 0, 0, 1, 5, 17]) if b else 0 for b in bufs]
alpha = b"abcdefghABCDEFGH" if nlits <= 30 else bytes(range(0x61, 0x7b))
rb = [bytearray(rand_data(rng, rng.choice([1024, 1500, 2048, 4096, 16384]), alpha))
      for _ in range(300)]
for k in range(len(rb) - 1):
    s = rng.choice(lits).s
    if len(s) > 1:
        cut = rng.randint(1, len(s) - 1)
        rb[k][len(rb[k]) - cut:] = s[:cut]
        rb[k + 1][:len(s) - cut] = s[cut:]
whole = b"".join(bytes(b) for b in rb)
cuts = [0]
while cuts[-1] < len(whole):
    cuts.append(min(len(whole), cuts[-1] + rng.choice([1, 7, 100, 1023, 1024, 5000, 40000])))
offs = np.array(cuts[:-1], np.uint64)
lens = np.diff(np.array(cuts, np.uint64))
hl = np.minimum(offs, 16).astype(np.uint64)
print("bytes", len(whole), "writes", len(offs), "split env", os.environ.get("VSA_SPLIT"), flush=True)
st, m = oracle.hwlm_exec(blob.ptr, whole, cap=1 << 22)
print("oracle matches", len(m), "status", st, flush=True)
ctx = vsa.Context(0)
host = np.frombuffer(whole, np.uint8)
d = ctx.malloc(len(host) + 64)
ctx.h2d(d, host)
db = vsa.Database(ctx, blob)
print("db split", db.split, flush=True)
k = ctx.scan_blocks_stream(db, d, offs, lens, hl)
got = ctx.results(k)
ends = (got["key"] >> np.uint64(24)).tolist()
print("records", k, "equal", list(zip(ends, got["id"].tolist())) == m, flush=True)
