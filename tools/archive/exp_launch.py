"""Launch breakdown of vsa_lit_scan (verdict r03 item 1): where a launch's
fixed cost goes at a given size.  With VSA_DEBUG_FLAGS=4096|8192 every wave
logs its kernel entry (before the LDS table staging), its scan start and end
(100 MHz s_memrealtime) and its segment / KiB counts; confirm waves log entry
and end.  Per workload (median over the logged launches):

  kernel      hipEvent time of the launch (scan stream)
  body        last wave end - first wave entry (device-observed)
  launch      kernel - body: dispatch before the first wave and drain after
  dispatch    last wave entry - first wave entry (workgroup dispatch spread)
  staging     median (scan start - entry) of the scanning waves
  first/p50/last end   scanning-wave ends relative to the first entry
  tail        last end - mean end: what a perfectly balanced finish saves
  idle        mean over scanning waves of (last end - own end), in us
  conf        last confirm-wave end - last scanning-wave end

Usage: exp_launch.py [--sizes MiB,...] [--extra noodle,teddy] [--launches N]
One JSON line per workload; the plain (no debug flag) kernel time of the same
workload is measured first for comparison."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import vectorscan_amd as vsa  # noqa: E402


def settle(fn, ctx, n=40):
    for _ in range(n):
        fn()
    ks = []
    for _ in range(20):
        fn()
        ks.append(ctx.kernel_ms())
    return float(np.median(ks))


def breakdown(ctx, log, fn, launches):
    rows = []
    os.environ["VSA_DEBUG_FLAGS"] = str(4096 | 8192)
    try:
        for _ in range(launches):
            log.zero_()
            fn()
            k = ctx.kernel_ms()
            L = log.view(-1, 16, 8).cpu().numpy().astype(np.int64)
            wg_live = L[:, :, 0].any(axis=1)
            L = L[wg_live]
            # scanning waves: entry in lane 7 (dbg 8192), start lane 0, end lane 1,
            # segments lane 2, KiB lane 3; confirm waves: entry lane 0, end lane 1,
            # lane 2 == 1 and lane 3 == 0 (their wave field stays 0)
            scan = L[:, :, 7] != 0
            conf = (~scan) & (L[:, :, 0] != 0)
            ent = np.where(scan, L[:, :, 7], L[:, :, 0])
            e0 = ent[scan | conf].min()
            st = (L[:, :, 0][scan] - e0) / 100.0
            en = (L[:, :, 1][scan] - e0) / 100.0
            stage = ((L[:, :, 0] - L[:, :, 7])[scan]) / 100.0
            ce = (L[:, :, 1][conf] - e0) / 100.0 if conf.any() else np.array([0.0])
            entries = (ent[scan | conf] - e0) / 100.0
            last = max(en.max(), ce.max())
            segs = L[:, :, 2][scan]
            kib = L[:, :, 3][scan]
            rows.append(dict(
                kernel_us=k * 1e3, body_us=last, launch_us=k * 1e3 - last,
                dispatch_us=entries.max(), staging_us=float(np.median(stage)),
                start_p50_us=float(np.median(st)), first_end_us=en.min(),
                p50_end_us=float(np.median(en)), last_end_us=en.max(),
                tail_us=en.max() - en.mean(), idle_us=float(np.mean(en.max() - en)),
                conf_after_us=ce.max() - en.max(), workgroups=int(L.shape[0]),
                scan_waves=int(scan.sum()), segs_max=int(segs.max()),
                segs_mean=float(segs.mean()), kib_mean=float(kib.mean()),
                kib_rate_p50=float(np.median(kib / np.maximum(en - st, 1e-3)))))
    finally:
        del os.environ["VSA_DEBUG_FLAGS"]
    out = {}
    for key in rows[0]:
        out[key] = round(float(np.median([r[key] for r in rows])), 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8,32,128,512,1024,4096")
    ap.add_argument("--extra", default="noodle,teddy")
    ap.add_argument("--launches", type=int, default=7)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = vsa.Context(0)
    log = torch.zeros(1024 * 16 * 8, dtype=torch.int64, device=dev)
    vsa.lib.vsa_set_wave_log.argtypes = [ctypes.c_void_p]
    vsa.lib.vsa_set_wave_log(log.data_ptr())
    lits = bench.make_literals(5000, seed=12)
    work = []
    fdb = vsa.Database(ctx, vsa.hwlm_build(lits))
    for mib in [int(s) for s in args.sizes.split(",") if s]:
        work.append(("fdr5k", fdb, lits, mib))
    extra = set(args.extra.split(",")) if args.extra else set()
    if "noodle" in extra:
        nl = [vsa.HwlmLiteral(b"abcde", False, 0)]
        work.append(("noodle", vsa.Database(ctx, vsa.hwlm_build(nl)), nl, 1024))
    if "teddy" in extra:
        import tools.bench_configs as bc
        tl = bc.lits_printable(48, 55)
        work.append(("teddy48", vsa.Database(ctx, vsa.hwlm_build(tl, engine_hint=18)), tl, 1024))
    cur = None
    for name, db, wl, mib in work:
        total = mib << 20
        if cur is None or cur[0] != (id(wl), total):
            cur = None
            torch.cuda.empty_cache()
            data = bench.make_corpus_device(torch, 0, total, total, wl, 5, 64 << 10, dev)
            cur = ((id(wl), total), data)
        data = cur[1]
        bl = total // 4
        offs = [i * bl for i in range(4)]
        plan = ctx.plan(data.data_ptr(), offs, [bl] * 4)

        def fn():
            ctx.scan_plan(db, plan)

        plain = settle(fn, ctx)
        d = breakdown(ctx, log, fn, args.launches)
        d.update(workload=name, mib=mib, plain_kernel_us=round(plain * 1e3, 2),
                 plain_tbs=round(total / (plain * 1e-3) / 1e12, 3))
        print(json.dumps(d), flush=True)
        plan.close()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
