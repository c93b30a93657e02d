"""Class-scan (cfg 2) kernel time of one library build, for an interleaved
A/B against another build on the same box (verdict r05 item 5: round 4's
2ba43e1 against this tree).  Runs the package found under ROOT (argv[1]):
shufti class A (8 chars) and truffle class B (100 bytes) over 256 MiB and
1 GiB of uniform bytes 0x00-0xFF (seed 2, the cfg-2 corpus), bitmap
written, after a clock settle; one JSON line per (size, kind) with the
median / min kernel time of 50 launches and the count (both builds must
agree).  The r04 build is made by tools/ab_build_r04.sh into ab/r04/.
  python tools/exp_class_ab.py ROOT LABEL"""
import json
import random
import statistics
import sys
import time

root, label = sys.argv[1], sys.argv[2]
sys.path.insert(0, root)
import torch  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402

ctx = vsa.Context(0)
classA = b"\x01\x7f\x80\xfe<>\"'"
classB = bytes(random.Random(5).sample(range(256), 100))
for n in (256 << 20, 1 << 30):
    g = torch.Generator(device="cuda")
    g.manual_seed(2)
    data = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for kind, chars in (("shufti", classA), ("truffle", classB)):
        a, b = (vsa.shufti_build_masks(chars) if kind == "shufti" else
                vsa.truffle_build_masks(chars))
        hist, t0 = [], time.perf_counter()
        while len(hist) < 400 and time.perf_counter() - t0 < 3.0:  # clock settle
            res = ctx.class_scan_masks(kind, a, b, data.data_ptr(), n, bitmap.data_ptr())
            hist.append(ctx.kernel_ms())
            if len(hist) >= 40 and max(hist[-8:]) <= 1.02 * min(hist[-8:]):
                break
        ks = []
        for _ in range(50):
            res = ctx.class_scan_masks(kind, a, b, data.data_ptr(), n, bitmap.data_ptr())
            ks.append(ctx.kernel_ms())
        print(json.dumps({"build": label, "bytes": n, "kind": kind,
                          "kernel_ms_median": round(statistics.median(ks), 5),
                          "kernel_ms_min": round(min(ks), 5), "count": int(res[2]),
                          "frac": round(n * 1.125 / (statistics.median(ks) * 1e-3) / 8e12, 4)}),
              flush=True)
    del data, bitmap
    torch.cuda.empty_cache()
ctx.close()
