"""Multi-rank striping of one block (vectorscan_amd/stripe.py), world size 2
over gloo on CPU.  Each rank's window is scanned by the test-only oracle in
place of the device (the device path is covered by test_gpu_parity); the
gathered union must equal the single-block scan."""
import os
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import vectorscan_amd as vsa
from vectorscan_amd import stripe as st
from test_cpu_oracle import rand_lits


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(seed, nlits, length):
    rng = random.Random(seed)
    lits = rand_lits(rng, nlits, minlen=1, maxlen=8, msk_frac=0.1)
    for l in lits:
        l.noruns = False  # NOREPEAT is sequential host state, replayed after the gather
    blob = vsa.hwlm_build(lits)
    r = np.random.default_rng(seed)
    data = bytes(r.choice(np.frombuffer(b"abcdefghABCD", np.uint8), length))
    return blob, data


def _worker(rank, world, port, seed, nlits, length, start, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob, data = _case(seed, nlits, length)
        plan = st.plan_block_stripes(len(data), start, world, min_stripe=64)
        s = plan[rank]
        win = data[s.wlo:s.wlo + s.wlen]
        _, m = oracle.hwlm_exec(blob.ptr, win, start=s.wstart, cap=1 << 20) if s.wlen else (0, [])
        ends = [e for e, _ in m]
        ids = [i for _, i in m]
        e, i = st.localize(s, ends, ids)
        ge, gi = st.gather_matches(dist, e, i)
        if rank == 0:
            q.put(list(zip(ge.tolist(), gi.tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("seed,nlits,length,start", [
    (1, 40, 5000, 0),      # Teddy
    (2, 300, 20000, 0),    # FDR
    (3, 300, 20000, 333),  # FDR, start inside rank 0's stripe
    (4, 5, 3000, 2900),    # start inside rank 1's stripe
    (5, 20, 40, 0),        # too short to split: rank 0 scans it whole
])
def test_striped_block_equals_single_scan(seed, nlits, length, start):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, nlits, length, start, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    blob, data = _case(seed, nlits, length)
    _, want = oracle.hwlm_exec(blob.ptr, data, start=start, cap=1 << 20)
    assert got == want
    assert len(want) > 0 or length < 64


def test_plan_covers_every_end_once():
    for length, start, world in [(10 ** 6, 0, 8), (10 ** 6, 12345, 8), (100, 0, 4),
                                 (1 << 20, (1 << 20) - 5, 2)]:
        plan = st.plan_block_stripes(length, start, world, min_stripe=64)
        owned = []
        for s in plan:
            assert s.wlo + s.wlen <= length
            if s.own_hi > s.own_lo:
                assert s.wlo <= max(0, s.own_lo - st.HALO) or s.wlo == 0
                assert s.wlo + s.wlen == s.own_hi
                owned.append((s.own_lo, s.own_hi))
        assert owned[0][0] == start
        assert owned[-1][1] == length
        for (a, b), (c, d) in zip(owned, owned[1:]):
            assert b == c


def _gather_worker(rank, world, port, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = [5, 0, 3][rank]
        keys = torch.arange(8, dtype=torch.int64) + 100 * rank
        ids = torch.arange(8, dtype=torch.int32) + 10 * rank
        got = st.gather_to_root(dist, keys, ids, n)
        if rank == 0:
            q.put((got[0].tolist(), got[1].tolist()))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_gather_to_root_world3():
    """bench.py's per-step gather (uneven counts, one empty rank)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    keys, ids = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert keys == [0, 1, 2, 3, 4, 200, 201, 202]
    assert ids == [0, 1, 2, 3, 4, 20, 21, 22]


# ------------------------------------------- whole-corpus striping (bench)

def _corpus_case(seed, total, block_len):
    rng = random.Random(seed)
    lits = rand_lits(rng, 300, minlen=1, maxlen=8, msk_frac=0.1)
    for l in lits:
        l.noruns = False
    blob = vsa.hwlm_build(lits)
    r = np.random.default_rng(seed)
    data = r.choice(np.frombuffer(b"abcdefghABCD", np.uint8), total)
    return blob, data


def _windows_matches(blob, data, wins):
    """oracle scan of each window as its own block from 0, ends >= rlo kept,
    as global (end, id) in window order"""
    out = []
    for w in wins:
        win = data[w.wlo:w.wlo + w.wlen]
        _, m = oracle.fdr_exec(vsa.engine_blob(blob), win, cap=1 << 20)
        out += [(e + w.wlo, i) for e, i in m if e >= w.rlo]
    return out


@pytest.mark.parametrize("total,block_len,world", [
    (50000, 20000, 2), (50000, 20000, 3), (65536, 65536, 8), (70001, 9999, 5)])
def test_corpus_stripes_union_equals_per_block_scan(total, block_len, world):
    """plan_corpus_stripes (bench.py's N-GPU split): the union over ranks of
    every window's reported ends equals the per-block single scans."""
    blob, data = _corpus_case(total + world, total, block_len)
    cuts, plan = st.plan_corpus_stripes(total, block_len, world, align=64)
    assert cuts[0] == 0 and cuts[-1] == total
    got = []
    for r in range(world):
        for w in plan[r]:
            assert cuts[r] <= w.wlo + w.rlo and w.wlo + w.wlen <= cuts[r + 1]
        got += _windows_matches(blob, data, plan[r])
    want = []
    for b in range(0, total, block_len):
        _, m = oracle.fdr_exec(vsa.engine_blob(blob), data[b:b + block_len], cap=1 << 20)
        want += [(e + b, i) for e, i in m]
    assert got == want and len(want) > 100


def _corpus_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob, data = _corpus_case(9, 40000, 15000)
        cuts, plan = st.plan_corpus_stripes(40000, 15000, world, align=64)
        m = _windows_matches(blob, data, plan[rank])
        ge, gi = st.gather_matches(dist, [e for e, _ in m], [i for _, i in m])
        if rank == 0:
            q.put(list(zip(ge.tolist(), gi.tolist())))
    finally:
        dist.destroy_process_group()


def test_corpus_stripes_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_corpus_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    blob, data = _corpus_case(9, 40000, 15000)
    want = []
    for b in range(0, 40000, 15000):
        _, m = oracle.fdr_exec(vsa.engine_blob(blob), data[b:b + 15000], cap=1 << 20)
        want += [(e + b, i) for e, i in m]
    assert got == want


def test_digest_matches_oracle_list():
    """oracle.digest_mt (bench.py's full-corpus check) == digest of the
    single-call oracle match list, for any thread count"""
    blob, data = _corpus_case(3, 300000, 300000)
    _, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 20)
    want = oracle.digest_of([e for e, _ in m], [i for _, i in m])
    for t in (1, 2, 7, 16):
        assert oracle.digest_mt(vsa.engine_blob(blob), data, t) == want


def test_records_mt_is_the_callback_sequence():
    """oracle.records_mt (bench.py's order-exact full-corpus check) == the
    single-call oracle's callback sequence element for element, for any
    thread count, and a small cap still reports the total"""
    blob, data = _corpus_case(3, 300000, 300000)
    _, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 20)
    assert len(m) > 100
    for t in (1, 2, 7, 16):
        e, i = oracle.records_mt(vsa.engine_blob(blob), data, t)
        assert list(zip(e.tolist(), i.tolist())) == m
    e, i = oracle.records_mt(vsa.engine_blob(blob), data, 3, cap=10)
    assert list(zip(e.tolist(), i.tolist())) == m


def test_hs_scan_records_equals_scan():
    """oracle.hs_lit.scan_records over records_mt's records == hs_lit.scan
    (bench.py's end-to-end check), for short-only and long-literal sets"""
    import bench
    from oracle import hs_lit as ohl
    data = bench.make_corpus(200000, bench.make_literals(50, seed=4), seed=6, plant_every=512)
    for maxlen in (8, 16):
        ex, fl, ids = bench.make_mixed_set(300, seed=5, maxlen=maxlen)
        # plant some of the set's own patterns
        d = data.copy()
        for k, p in enumerate(range(100, 190000, 997)):
            s = ex[k % len(ex)]
            d[p:p + len(s)] = np.frombuffer(s, np.uint8)
        odb = ohl.compile_lit_multi(ex, fl, ids)
        blob = vsa.hwlm_build([vsa.HwlmLiteral(t, nc, f, noruns=nr)
                               for t, nc, f, nr in odb.hwlm_literals()])
        want = ohl.scan(odb, blob.ptr, d)
        e, i = oracle.records_mt(vsa.engine_blob(blob), d, 5, nood=blob.is_noodle)
        got = ohl.scan_records(odb, d, zip(e.tolist(), i.tolist()))
        assert len(want) > 50 and got == want


def _packed_worker(rank, world, port, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pg = st.PackedGather(dist, world)
        out = []
        # step 1 fits the initial 1,024; step 2 passes it on rank 1 (grow +
        # repeat); step 3 has an empty rank
        for n in ([3, 7, 0][rank], [10, 1500, 4][rank], [0, 0, 9][rank]):
            keys = torch.arange(n, dtype=torch.int64) * 5 + (rank << 40)
            ids = torch.arange(n, dtype=torch.int32) + 1000 * rank

            counts = pg.gather(st.host_pack(keys, ids, n))
            if rank == 0:
                k, i = pg.merged(counts)
                out.append((counts, k.tolist(), i.tolist(), pg.cap))
            else:
                assert pg.merged(counts) is None
        # step 4: rank 2's first pack is not final (a scan that overflowed
        # its output): every rank sees the header bit, completes and packs again
        n = 5
        keys = torch.arange(n, dtype=torch.int64) * 5 + (rank << 40)
        ids = torch.arange(n, dtype=torch.int32) + 1000 * rank
        state = {"final": rank != 2, "packs": 0}
        base = st.host_pack(keys, ids, n)

        def pack(buf, cap):
            state["packs"] += 1
            base(buf, cap)
            if not state["final"]:
                buf[0] = n | st.NOT_READY

        counts = pg.gather(pack, complete=lambda: state.update(final=True))
        assert state["packs"] == 2, state
        if rank == 0:
            k, i = pg.merged(counts)
            out.append((counts, k.tolist(), i.tolist(), pg.cap))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def test_packed_gather_world3():
    """bench.py's per-step exchange (stripe.PackedGather): the headers
    all-gathered, the records gathered to rank 0 only, the buffers grown
    from the gathered headers when a rank passes them."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_packed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for counts, keys, ids, cap in out:
        want_k, want_i = [], []
        for r, n in enumerate(counts):
            want_k += [j * 5 + (r << 40) for j in range(n)]
            want_i += [j + 1000 * r for j in range(n)]
        assert keys == want_k and ids == want_i
    assert [o[0] for o in out] == [[3, 7, 0], [10, 1500, 4], [0, 0, 9], [5, 5, 5]]
    assert out[0][3] == 1024 and out[1][3] == 1875 and out[3][3] == 1875
