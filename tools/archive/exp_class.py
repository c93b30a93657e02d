"""Class scan (cfg 2's kernel, vsa_class_scan_lut) against the streaming-read
ceiling at several sizes, with and without the bitmap output: separates the
per-launch fixed cost from the per-byte rate.  One JSON line per size.
Usage: python tools/exp_class.py [out.jsonl]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

ctx = vsa.Context(0)
out = open(sys.argv[1], "a") if len(sys.argv) > 1 else None
N = 1 << 30
g = torch.Generator(device="cuda")
g.manual_seed(2)
data = torch.randint(0, 256, (N,), dtype=torch.uint8, device="cuda", generator=g)
bitmap = torch.zeros(N // 64, dtype=torch.int64, device="cuda")
a, b = vsa.shufti_build_masks(b"\x01\x7f\x80\xfe<>\"'")
torch.cuda.synchronize()


def kms(n, bm, reps=30):
    for _ in range(60):
        ctx.class_scan_masks("shufti", a, b, data.data_ptr(), n, bm)
    ks = []
    for _ in range(reps):
        ctx.class_scan_masks("shufti", a, b, data.data_ptr(), n, bm)
        ks.append(ctx.kernel_ms())
    return float(np.median(ks)) * 1000.0, float(np.min(ks)) * 1000.0


for mib in [int(x) for x in os.environ.get("SIZES", "32,64,128,256,512,1024").split(",")]:
    n = mib << 20
    with_bm = kms(n, bitmap.data_ptr())
    no_bm = kms(n, None)
    _, ms, _ = ctx.read_ceiling(data.data_ptr(), n, 5)
    rec = {"mib": mib, "bitmap_us_p50": round(with_bm[0], 1), "bitmap_us_min": round(with_bm[1], 1),
           "nobitmap_us_p50": round(no_bm[0], 1), "read_ceiling_us": round(ms * 1000.0, 1),
           "frac_of_ceiling": round(ms * 1000.0 / with_bm[0], 3)}
    print(json.dumps(rec), flush=True)
    if out:
        out.write(json.dumps(rec) + "\n")

if os.environ.get("WPROBE"):
    # write-side references: hipMemset of the bitmap sizes, a device copy
    def ev_time(fn, reps=30):
        for _ in range(10):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(reps):
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0)
        return round(float(np.median(ts)), 1)
    for mib in (32, 128):
        v = bitmap.view(torch.uint8)[:mib << 20]
        dst = torch.empty(mib << 20, dtype=torch.uint8, device="cuda")
        rec = {"write_mib": mib, "memset_us": ev_time(lambda: v.zero_()),
               "copy_us": ev_time(lambda: dst.copy_(data[:mib << 20]))}
        print(json.dumps(rec), flush=True)
