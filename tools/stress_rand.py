"""Debug helper: repeat one random parity case to expose nondeterminism."""
import os, sys, random
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import vectorscan_amd as vsa, oracle
from test_cpu_oracle import rand_lits, rand_data
from test_gpu_parity import gpu_hwlm
seed, nlits, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rng = random.Random(seed * 7919 + nlits)
lits = rand_lits(rng, nlits, msk_frac=0.15)
for l in lits:
    l.noruns = rng.random() < 0.3
    l.groups = rng.choice([1, 2, 3, vsa.HWLM_ALL_GROUPS])
blob = vsa.hwlm_build(lits)
cases = []
for ln in (0, 1, 2, 7, 15, 16, 17, 31, 33, 64, 100, 1023, 1025, 4096, 70000):
    data = rand_data(rng, ln)
    for start in sorted({0, 1, 3, min(17, ln), ln // 2}):
        if start >= max(ln, 1):
            continue
        st_o, m_o = oracle.hwlm_exec(blob.ptr, data, start=start, cap=1 << 16)
        cases.append((ln, start, data, m_o))
bad = 0
for r in range(reps):
    for ln, start, data, m_o in cases:
        st_g, m_g = gpu_hwlm(blob, data, start=start)
        if m_g != m_o:
            bad += 1
            if bad <= 5:
                print("rep", r, "ln", ln, "start", start, "n", len(m_g), len(m_o))
                print(" only gpu", sorted(set(m_g) - set(m_o))[:10], "only orc", sorted(set(m_o) - set(m_g))[:10], flush=True)
print("cases", len(cases) * reps, "bad", bad)
