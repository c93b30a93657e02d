"""GPU: the batching service for concurrent drop-in calls
(vsa_batcher_hwlmExec, include/vectorscan_amd.h): every call's callback
sequence equals the oracle's hwlmExec of that buffer alone (hwlm.c:178),
whatever batch it was scanned in."""
import random
import threading

import pytest

import oracle
import vectorscan_amd as vsa
from test_cpu_oracle import rand_data, rand_lits

pytestmark = pytest.mark.gpu


def _calls(rng, n, blob_list):
    out = []
    for _ in range(n):
        blob = rng.choice(blob_list)
        data = rand_data(rng, rng.choice([0, 1, 15, 16, 17, 100, 1000, 4096, 20000, 70000]))
        start = rng.choice([0, 0, 0, 3, 17]) if data else 0
        out.append((blob, data, min(start, max(0, len(data) - 1)) if data else 0))
    return out


def test_gpu_batcher_concurrent_threads():
    rng = random.Random(31)
    blobs = [vsa.hwlm_build(rand_lits(rng, n, minlen=2, maxlen=8)) for n in (1, 5, 40, 300)]
    work = [_calls(random.Random(100 + t), 40, blobs) for t in range(8)]
    want = [[oracle.hwlm_exec(b.ptr, d, start=s, cap=1 << 16) for b, d, s in w] for w in work]
    b = vsa.Batcher(0, max_batch=64, window_us=200)
    got = [[None] * len(w) for w in work]
    errs = []

    def run(t):
        try:
            for i, (blob, d, s) in enumerate(work[t]):
                got[t][i] = b.hwlm_exec(blob, d, start=s)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs
    for t in range(8):
        for i in range(len(work[t])):
            assert got[t][i] == want[t][i], (t, i)
    launches, calls = b.stats()
    b.close()
    served = sum(1 for w in work for _, d, s in w if d and s < len(d))
    assert calls == served
    assert launches < calls  # calls of different threads shared launches


def test_gpu_batcher_terminate_and_groups():
    """the caller's callback return value: 0 terminates its own call only
    (HWLM_TERMINATED), a group mask becomes the live groups"""
    rng = random.Random(5)
    lits = rand_lits(rng, 40)
    for l in lits:
        l.groups = 1 << (l.id % 3)
    blob = vsa.hwlm_build(lits)
    data = rand_data(rng, 20000)
    b = vsa.Batcher(0, max_batch=8, window_us=0)
    try:
        for k in (1, 5):
            seq = []

            def cb(end, id_, seq=seq, k=k):
                seq.append((end, id_))
                return 0 if len(seq) >= k else vsa.HWLM_ALL_GROUPS

            rc = b.hwlm_exec(blob, data, cb=cb)
            st_o, m_o = oracle.hwlm_exec(blob.ptr, data, term_after=k, cap=1 << 16)
            assert (rc, seq) == (st_o, m_o)
        for ret in (1, 6):
            seq = []

            def cb2(end, id_, seq=seq, ret=ret):
                seq.append((end, id_))
                return ret

            rc = b.hwlm_exec(blob, data, cb=cb2)
            st_o, m_o = oracle.hwlm_exec(blob.ptr, data, cap=1 << 16, cb_ret=ret)
            assert (rc, seq) == (st_o, m_o)
    finally:
        b.close()
