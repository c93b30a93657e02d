"""Streaming-read ceiling (vsa_read_ceiling) at 64 MiB - 1 GiB: what a
scan of that size could reach on this box (launch and tail included)."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch, bench, vectorscan_amd as vsa
dev = torch.device("cuda", 0); ctx = vsa.Context(0)
lits = bench.make_literals(100, seed=1)
data = bench.make_corpus_device(torch, 0, 1 << 30, 1 << 30, lits, 5, 64 << 10, dev)
torch.cuda.synchronize()
for mib in (64, 128, 256, 512, 1024):
    best = ctx.read_ceiling(data.data_ptr(), mib << 20, 10)
    print(mib, "MiB ceiling %.1f GB/s %.1f us" % (best[0], best[1] * 1000))
