"""Debug helper: rerun one test_gpu_vs_oracle_random case and diff."""
import os, sys, random
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import vectorscan_amd as vsa, oracle
from test_cpu_oracle import rand_lits, rand_data
from test_gpu_parity import gpu_hwlm
seed, nlits, want_ln = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rng = random.Random(seed * 7919 + nlits)
lits = rand_lits(rng, nlits, msk_frac=0.15)
for l in lits:
    l.noruns = rng.random() < 0.3
    l.groups = rng.choice([1, 2, 3, vsa.HWLM_ALL_GROUPS])
blob = vsa.hwlm_build(lits)
print("engine", blob.engine_id)
for ln in (0, 1, 2, 7, 15, 16, 17, 31, 33, 64, 100, 1023, 1025, 4096, 70000):
    data = rand_data(rng, ln)
    if ln != want_ln:
        continue
    for start in sorted({0, 1, 3, min(17, ln), ln // 2}):
        if start >= max(ln, 1):
            continue
        for groups in (vsa.HWLM_ALL_GROUPS, 1):
            st_o, m_o = oracle.hwlm_exec(blob.ptr, data, start=start, groups=groups, cap=1 << 16)
            st_g, m_g = gpu_hwlm(blob, data, start=start, groups=groups)
            print("start", start, "groups", groups, "ok" if m_g == m_o else "BAD", len(m_g), len(m_o))
            if m_g != m_o:
                print(" gpu", m_g[:40])
                print(" orc", m_o[:40])
                print(" only gpu", sorted(set(m_g) - set(m_o))[:20], "only orc", sorted(set(m_o) - set(m_g))[:20])
            # raw device results
            ctx = vsa.Context(0)
            buf = ctx.malloc(max(len(data), 1) + 64)
            import numpy as np
            ctx.h2d(buf, np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8))
            db = vsa.Database(ctx, blob)
            n = ctx.scan_blocks(db, buf, [0], [len(data)], [start])
            r = ctx.results(n)
            print(" raw", [(int(k) >> 24, (int(k) >> 20) & 15, int(k) & 0xfffff, int(i)) for k, i in zip(r["key"], r["id"])][:60])
            db.close(); ctx.free(buf); ctx.close()
