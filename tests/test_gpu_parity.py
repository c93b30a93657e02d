"""GPU parity tests: the HIP engine (through the C ABI) against the oracle
and the reference's known answers.  Integer/byte work: every comparison is
bit-exact (match lists compared in callback order)."""
import ctypes
import json
import os
import random

import numpy as np
import pytest

import oracle
import vectorscan_amd as vsa
from test_cpu_oracle import (FDR_HINTS, build_or_none, load, lits_of, rand_data,
                             rand_lits, _short_writings)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = vsa.Context(0)
    yield c
    c.close()


def gpu_hwlm(blob, data, start=0, groups=vsa.HWLM_ALL_GROUPS, term_after=-1, cb_ret=None):
    seq = []

    def cb(end, id_):
        seq.append((end, id_))
        if term_after >= 0 and len(seq) >= term_after:
            return 0
        return vsa.HWLM_ALL_GROUPS if cb_ret is None else cb_ret

    rc = vsa.hwlm_exec(blob, data, start=start, cb=cb, groups=groups)
    return rc, seq


# ------------------------------------------------------------- golden ---

def test_gpu_golden_noodle():
    for c in load("noodle.json"):
        blob = vsa.hwlm_build([vsa.HwlmLiteral(bytes.fromhex(c["lit"]), c["nocase"], 1000)])
        st, m = vsa.nood_exec(blob, bytes.fromhex(c["data"]))
        assert st == 0
        assert [e for e, _ in m] == c["expected"], c["src"]


@pytest.mark.parametrize("hint", FDR_HINTS)
def test_gpu_golden_fdr(hint):
    for c in load("fdr.json"):
        blob = build_or_none(lits_of(c), hint)
        if blob is None:
            continue
        data = bytes.fromhex(c["data"])
        if c["expected"] is None:
            seq = []

            def cb(end, id_):
                seq.append((end, id_))
                return 0
            rc = vsa.fdr_exec(blob, data, cb=cb)
            assert rc == vsa.HWLM_TERMINATED and len(seq) == c["expected_len"]
            continue
        st, m = vsa.fdr_exec(blob, data, start=c["start"])
        assert st == 0
        assert [list(x) for x in m] == c["expected"], (c["src"], hint)


def test_gpu_golden_accel():
    from test_cpu_oracle import accel_expected_oracle  # noqa: F401
    for c in load("accel.json"):
        data = bytes.fromhex(c["data"])
        k = c["kind"]
        if k in ("shufti", "rshufti"):
            lo, hi = vsa.shufti_build_masks(c["chars"])
            got = (vsa.rshufti_exec if k == "rshufti" else vsa.shufti_exec)(lo, hi, data)
        elif k in ("truffle", "rtruffle"):
            m1, m2 = vsa.truffle_build_masks(c["chars"])
            got = (vsa.rtruffle_exec if k == "rtruffle" else vsa.truffle_exec)(m1, m2, data)
        elif k == "verm":
            got = vsa.vermicelli_exec(c["c"], c["nocase"], data)
        elif k == "nverm":
            got = vsa.nvermicelli_exec(c["c"], c["nocase"], data)
        elif k == "rverm":
            got = vsa.rvermicelli_exec(c["c"], c["nocase"], data)
        elif k == "rnverm":
            got = vsa.rnvermicelli_exec(c["c"], c["nocase"], data)
        elif k == "dverm":
            got = vsa.vermicelli_double_exec(c["c1"], c["c2"], c["nocase"], data)
        elif k == "rdverm":
            got = vsa.rvermicelli_double_exec(c["c1"], c["c2"], c["nocase"], data)
        else:
            raise AssertionError(k)
        assert got == c["expected"], c["src"]


def test_gpu_short_writings_batched(ctx):
    """fdr.cpp:594-692: every buffer of a literal group is one block of a
    single device launch."""
    spec = load("fdr_shortwritings.json")[0]

    def run(blob, bufs):
        return batch_run(ctx, blob, bufs)

    for hint in (0, 11, 17, 3, 9):
        _short_writings(spec, hint, run)


# ---------------------------------------------------------- batch API ---

def batch_run(ctx, blob, bufs, starts=None, misalign=0):
    """Scan bufs as blocks of one launch; return per-block [(end, id)]."""
    offs, pos = [], misalign
    for b in bufs:
        offs.append(pos)
        pos += len(b) + 3  # gaps between blocks: bytes outside every block
    host = np.full(pos + 16, 0x61, np.uint8)
    for o, b in zip(offs, bufs):
        host[o:o + len(b)] = np.frombuffer(b, np.uint8)
    dbuf = ctx.malloc(len(host))
    try:
        ctx.h2d(dbuf, host)
        db = vsa.Database(ctx, blob)
        n = ctx.scan_blocks(db, dbuf, offs, [len(b) for b in bufs], starts)
        res = ctx.results(n)
        db.close()
    finally:
        ctx.free(dbuf)
    out = [[] for _ in bufs]
    ends = res["key"] >> np.uint64(24)
    bi = np.searchsorted(np.array(offs, np.uint64), ends, side="right") - 1
    for e, i, b in zip(ends.tolist(), res["id"].tolist(), bi.tolist()):
        out[b].append((e - offs[b], i))
    return out


def replay_set(blob, seq):
    return seq


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("nlits", [1, 5, 30, 60, 96, 300, 3000])
def test_gpu_vs_oracle_random(seed, nlits):
    rng = random.Random(seed * 7919 + nlits)
    lits = rand_lits(rng, nlits, msk_frac=0.15)
    for l in lits:
        l.noruns = rng.random() < 0.3
        l.groups = rng.choice([1, 2, 3, vsa.HWLM_ALL_GROUPS])
    blob = vsa.hwlm_build(lits)
    for ln in (0, 1, 2, 7, 15, 16, 17, 31, 33, 64, 100, 1023, 1025, 4096, 70000):
        data = rand_data(rng, ln)
        for start in sorted({0, 1, 3, min(17, ln), ln // 2}):
            if start >= max(ln, 1):
                continue
            for groups in (vsa.HWLM_ALL_GROUPS, 1):
                st_o, m_o = oracle.hwlm_exec(blob.ptr, data, start=start, groups=groups,
                                             cap=1 << 16)
                st_g, m_g = gpu_hwlm(blob, data, start=start, groups=groups)
                assert st_g == st_o
                assert m_g == m_o, (nlits, ln, start, groups)


@pytest.mark.parametrize("hint", FDR_HINTS)
def test_gpu_vs_oracle_engines(hint):
    rng = random.Random(100 + hint)
    for trial in range(4):
        lits = rand_lits(rng, rng.randint(1, 40), msk_frac=0.1)
        blob = build_or_none(lits, hint)
        if blob is None:
            continue
        for ln in (5, 16, 40, 300, 5000):
            data = rand_data(rng, ln)
            st_o, m_o = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 16)
            st_g, m_g = vsa.fdr_exec(blob, data)
            assert m_g == m_o, (hint, trial, ln)


def test_gpu_terminate_and_control():
    rng = random.Random(3)
    lits = rand_lits(rng, 40)
    blob = vsa.hwlm_build(lits)
    data = rand_data(rng, 20000)
    for k in (1, 2, 5, 50):
        st_o, m_o = oracle.hwlm_exec(blob.ptr, data, term_after=k, cap=1 << 16)
        st_g, m_g = gpu_hwlm(blob, data, term_after=k)
        assert (st_g, m_g) == (st_o, m_o)
    # the callback's return value becomes the live group mask
    # (confWithBit: li->groups & *control, fdr_confirm_runtime.h:91-96)
    for l in lits:
        l.groups = 1 << (l.id % 3)
        l.noruns = l.id % 2 == 0
    blob = vsa.hwlm_build(lits)
    for ret in (1, 2, 6):
        st_o, m_o = oracle.hwlm_exec(blob.ptr, data, cap=1 << 16, cb_ret=ret)
        st_g, m_g = gpu_hwlm(blob, data, cb_ret=ret)
        assert (st_g, m_g) == (st_o, m_o)
        assert len(m_o) > 1


def test_gpu_batch_blocks_misaligned(ctx):
    rng = random.Random(11)
    lits = rand_lits(rng, 500, minlen=3, maxlen=8)
    blob = vsa.hwlm_build(lits)
    bufs = [rand_data(rng, rng.choice([0, 1, 5, 17, 100, 1000, 5000, 70000])) for _ in range(40)]
    starts = [rng.randint(0, max(0, len(b) - 1)) if b else 0 for b in bufs]
    for mis in (0, 1, 7, 13):
        got = batch_run(ctx, blob, bufs, starts=starts, misalign=mis)
        for b, s, g in zip(bufs, starts, got):
            if s >= len(b):
                assert g == []
                continue
            st, m = oracle.fdr_exec(vsa.engine_blob(blob), b, start=s, cap=1 << 16)
            assert g == m


# --------------------------------------------------------- full sizes ---

def test_gpu_fdr_5k_64mib(ctx):
    """cfg-4 shape (5,000 printable literals, len 4-8, 2% nocase, planted
    occurrences) on a 64 MiB block: exact sequence vs the oracle."""
    import bench
    lits = bench.make_literals(5000, seed=12)
    blob = vsa.hwlm_build(lits)
    assert blob.engine_id == 0
    data = bench.make_corpus(64 << 20, lits, seed=5, plant_every=64 << 10)
    got = batch_run(ctx, blob, [data.tobytes()])[0]
    st, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 20)
    assert st == 0
    assert got == m
    assert len(m) >= (64 << 20) // (64 << 10)


@pytest.mark.parametrize("engine", ["fdr", "teddy", "noodle"])
def test_gpu_dyn_shares_ragged(ctx, engine):
    """Dynamic shares (kernels.hip dyn_bounds; on here from 256 MiB): ~400
    MiB of 40 ragged blocks (4-16 MiB plus odd bytes, gaps between them, some
    with a start) scanned 5 times through one prebuilt plan and 3 times per
    call.  Each FDR launch after the first cuts the workgroups' KiB ranges at
    the weights the previous launch's end times give, so every launch splits
    the bytes differently, at arbitrary KiB inside segments: each launch's
    records equal the oracle's, block by block, and every FDR launch used the
    dynamic shares.  Teddy and noodle launches of the same plan keep the
    static lists (and their owned bins)."""
    import bench
    ctx.dyn_shares(True, min_mib=256)
    rng = random.Random(77)
    if engine == "fdr":
        lits = bench.make_literals(5000, seed=12)
    elif engine == "teddy":
        lits = bench.make_literals(24, seed=13)
    else:
        lits = [vsa.HwlmLiteral(b"needle", False, 7)]
    blob = vsa.hwlm_build(lits)
    offs, lens, starts, pos = [], [], [], 3
    for i in range(40):
        ln = rng.randint(4 << 20, 16 << 20) + rng.randint(0, 1023)
        offs.append(pos)
        lens.append(ln)
        starts.append(rng.choice([0, 0, 0, 5, 1000]))
        pos += ln + rng.choice([0, 64, rng.randint(1, 5000)])
    host = bench.make_corpus(pos + 64, lits, seed=6, plant_every=64 << 10)
    want = [oracle.hwlm_exec(blob.ptr, host[o:o + ln], start=s, cap=1 << 20)[1]
            for o, ln, s in zip(offs, lens, starts)]
    d = ctx.malloc(len(host))
    db = vsa.Database(ctx, blob)
    plan = None
    try:
        ctx.h2d(d, host)
        plan = ctx.plan(d, offs, lens, starts)
        for k in range(8):
            m = (ctx.scan_plan(db, plan) if k < 5
                 else ctx.scan_blocks(db, d, offs, lens, starts))
            assert ctx.last_dyn() == (engine == "fdr"), k
            res = ctx.results(m)
            ends = res["key"] >> np.uint64(24)
            bi = np.searchsorted(np.array(offs, np.uint64), ends, side="right") - 1
            got = [[] for _ in offs]
            for e, i, b in zip(ends.tolist(), res["id"].tolist(), bi.tolist()):
                got[b].append((e - offs[b], i))
            for b in range(len(offs)):
                assert got[b] == want[b], (k, b)
    finally:
        ctx.dyn_shares(False)
        if plan is not None:
            plan.close()
        db.close()
        ctx.free(d)


@pytest.mark.parametrize("fused,dyn", [(False, False), (True, False), (False, True)])
def test_gpu_schedule_feedback_512mib(ctx, fused, dyn):
    """Schedule feedback (runtime.hip take_feedback / refresh_plan): 512 MiB
    in 4 blocks scanned 8 times through one prebuilt plan and 8 times per
    call (scan_blocks), so the XCD weights are learned and the plans rebuilt
    with weighted shares between launches: every launch's records equal the
    first one's, and that one's digest equals the oracle's.  With the fused
    finish too (its last workgroup publishes the feedback record), and with
    the dynamic shares instead of the host's feedback (each launch re-cuts
    the shares from the previous launch's end times)."""
    import bench
    ctx.fused_finish(fused)
    ctx.dyn_shares(dyn, min_mib=256)
    lits = bench.make_literals(5000, seed=12)
    blob = vsa.hwlm_build(lits)
    db = vsa.Database(ctx, blob)
    n = 512 << 20
    bl = n // 4
    offs = [i * bl for i in range(4)]
    host = bench.make_corpus(n, lits, seed=5, plant_every=64 << 10)
    d = ctx.malloc(n + 64)
    first = None
    plan = None
    fused_seen = []
    try:
        ctx.h2d(d, host)
        plan = ctx.plan(d, offs, [bl] * 4)
        for k in range(16):
            m = ctx.scan_plan(db, plan) if k < 8 else ctx.scan_blocks(db, d, offs, [bl] * 4)
            res = ctx.results(m)
            cur = (res["key"].copy(), res["id"].copy())
            if first is None:
                first = cur
                want = oracle.digest_mt(vsa.engine_blob(blob), host, 16)
                assert oracle.digest_of(res["key"] >> np.uint64(24), res["id"]) == want
            else:
                assert np.array_equal(cur[0], first[0]) and np.array_equal(cur[1], first[1]), k
            fused_seen.append(ctx.last_fused())
            assert ctx.last_dyn() == (dyn and not fused), k
            if k == 7 and not dyn:
                # the first complete feedback record always publishes weights
                # (feedback_update), so the prebuilt plan was rebuilt for them
                assert plan.rebuilds() >= 1
        assert any(fused_seen) == fused
    finally:
        ctx.fused_finish(False)
        ctx.dyn_shares(False)
        if plan is not None:
            plan.close()
        db.close()
        ctx.free(d)


@pytest.mark.parametrize("kind", ["shufti", "truffle"])
def test_gpu_class_scan_256mib(ctx, kind):
    """cfg-2: 256 MiB uniform bytes, class A, driven by the shufti / truffle
    masks (vsa_class_scan_masks: the class the bytecode accepts, derived as
    the drop-ins do): bitmap, count, first and last == the oracle's per-byte
    mask test over the whole buffer (orc_shufti_bitmap / orc_truffle_bitmap),
    and that equals numpy membership of the class's characters."""
    rng = np.random.default_rng(2)
    n = 256 << 20
    data = rng.integers(0, 256, n, dtype=np.uint8)
    chars = [0x01, 0x7F, 0x80, 0xFE, ord("<"), ord(">"), ord('"'), ord("'")]
    a, b = (vsa.shufti_build_masks(bytes(chars)) if kind == "shufti"
            else vsa.truffle_build_masks(bytes(chars)))
    dbuf = ctx.malloc(n)
    dbm = ctx.malloc(n // 8)
    try:
        ctx.h2d(dbuf, data)
        f, l, cnt = ctx.class_scan_masks(kind, a, b, dbuf, n, d_bitmap=dbm)
        bm = np.zeros(n // 64, np.uint64)
        ctx.d2h(bm, dbm)
    finally:
        ctx.free(dbuf)
        ctx.free(dbm)
    want, want_n = oracle.class_bitmap_of_masks(kind, a, b, data)
    assert np.array_equal(bm, want) and cnt == want_n
    member = np.isin(data, np.array(chars, np.uint8))
    assert np.array_equal(bm.view(np.uint8), np.packbits(member, bitorder="little"))
    idx = np.nonzero(member)[0]
    assert cnt == len(idx) and f == idx[0] and l == idx[-1] + 1


@pytest.mark.parametrize("n,nchars,seed", [((8 << 20) + 13, 5, 31), ((9 << 20) + 1023, 100, 32),
                                           ((16 << 20) + 1, 0, 33), ((12 << 20) + 4097, 256, 34)])
def test_gpu_class_scan_lut_ragged(ctx, n, nchars, seed):
    """The pair-LUT class kernel (buffers >= 8 MiB): ragged lengths (last
    wave span and last lane partial), empty and full classes, random
    classes; bitmap, first, last and count against numpy."""
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, n, dtype=np.uint8)
    chars = sorted(rng.choice(256, nchars, replace=False).tolist()) if nchars < 256 \
        else list(range(256))
    cls = vsa.class_bitmap(chars)
    nbm = ((n + 63) // 64) * 8
    dbuf = ctx.malloc(n + 64)
    dbm = ctx.malloc(nbm)
    try:
        ctx.h2d(dbuf, data)
        ctx.h2d(dbm, np.zeros(nbm, np.uint8))
        f, l, cnt = ctx.class_scan(cls, dbuf, n, d_bitmap=dbm)
        bm = np.zeros(nbm, np.uint8)
        ctx.d2h(bm, dbm)
    finally:
        ctx.free(dbuf)
        ctx.free(dbm)
    member = np.isin(data, np.array(chars, np.uint8))
    exp = np.packbits(member, bitorder="little")
    assert np.array_equal(bm[:len(exp)], exp)
    idx = np.nonzero(member)[0]
    assert cnt == len(idx)
    assert f == (idx[0] if len(idx) else n)
    assert l == (idx[-1] + 1 if len(idx) else 0)


@pytest.mark.parametrize("lit,nocase", [(b"abcde", False), (b"aBcDe", True), (b"q", False),
                                        (b"xy", True), (b"\x00\x00", False)])
def test_gpu_noodle_16mib_planted(ctx, lit, nocase):
    """Noodle over 16 MiB with planted occurrences (the key prefilter path
    and its full compare), exact sequence vs the oracle."""
    rng = np.random.default_rng(len(lit) * 7 + nocase)
    n = 16 << 20
    data = rng.integers(0x20, 0x7F, n, dtype=np.uint8)
    pos = rng.integers(0, n - 8, 3000)
    for p in pos.tolist():
        s = lit.swapcase() if nocase and p & 1 else lit
        data[p:p + len(s)] = np.frombuffer(s, np.uint8)
    blob = vsa.hwlm_build([vsa.HwlmLiteral(lit, nocase, 77)])
    assert blob.is_noodle
    got = batch_run(ctx, blob, [data.tobytes()])[0]
    st, m = oracle.nood_exec(vsa.engine_blob(blob), data, cap=1 << 22)
    assert st == 0
    assert got == m
    assert len(m) >= 1000


@pytest.mark.gpu
def test_gpu_dropin_reused_address():
    """A database freed and rebuilt at the same address (same size, other
    content) must not be served from the drop-in's cached device copy."""
    import ctypes
    lits_a = [vsa.HwlmLiteral(s, False, i) for i, s in enumerate(
        [b"abcdef", b"bcdefg", b"xyzw", b"hello", b"world"] * 20)]
    lits_b = [vsa.HwlmLiteral(l.s, False, l.id + 1000) for l in lits_a]
    a, b = vsa.hwlm_build(lits_a), vsa.hwlm_build(lits_b)
    assert a.size == b.size and a.tobytes() != b.tobytes()
    raw = ctypes.create_string_buffer(a.size + 64)
    base = (ctypes.addressof(raw) + 63) & ~63
    data = b"..abcdefg..hello world xyzw" * 50
    shared = vsa.Blob(base, a.size, owned=False)
    for blob in (a, b, a):
        ctypes.memmove(base, blob.ptr, blob.size)
        _, m_g = vsa.hwlm_exec(shared, data)
        _, m_o = oracle.hwlm_exec(blob.ptr, data, cap=1 << 16)
        assert m_g == m_o and m_g


@pytest.mark.parametrize("nlits,lo", [(300, 6), (200, 8), (1000, 4), (2000, 7)])
def test_gpu_fdr_long_literal_strides(nlits, lo):
    """Stride 2 / 4 FDR bytecode: the device first stage is rebuilt as a
    stride-1 table from the confirm records; matches must equal the
    oracle's (which follows the bytecode's own stride)."""
    rng = random.Random(nlits * 31 + lo)
    lits = rand_lits(rng, nlits, minlen=lo, maxlen=8, nocase_frac=0.1, msk_frac=0.1)
    blob = vsa.hwlm_build(lits)
    assert blob.engine_id == 0
    for ln in (5, 16, 17, 40, 300, 5000, 70000):
        data = rand_data(rng, ln, alphabet=b"abcdefghAB")
        for start in sorted({0, 1, 3, 9, ln // 2}):
            if start >= ln:
                continue
            st_o, m_o = oracle.hwlm_exec(blob.ptr, data, start=start, cap=1 << 18)
            st_g, m_g = gpu_hwlm(blob, data, start=start)
            assert m_g == m_o, (nlits, lo, ln, start)


@pytest.mark.parametrize("vsize", [16, 32, 64])
def test_gpu_golden_dshufti(vsize):
    """shuftiDoubleExec drop-in: the reference's known answers (shufti.cpp:
    482-890) and exact agreement with the oracle at several alignments."""
    from test_cpu_oracle import dshufti_expect_ok, dshufti_masks, placed
    vsa.set_accel_vector_size(vsize)
    try:
        spec = load("dshufti.json")
        for c in spec["exec"][::3]:
            m = dshufti_masks(c)
            full = bytes.fromhex(c["data"])
            for base_mis in (0, 3, 16, 47):
                keep, addr = placed(full, base_mis)
                p = addr + c["start"]
                n = c["end"] - c["start"]
                r = vsa.shufti_double_find(*m, p, n)
                want = oracle.shufti_double(*m, full[c["start"]:c["end"]], vector_size=vsize,
                                            mis=p % vsize)
                assert r == want, (c["src"], vsize, base_mis)
                assert dshufti_expect_ok(c, r, base_mis), (c["src"], vsize, base_mis)
    finally:
        vsa.set_accel_vector_size(64)


def test_gpu_dshufti_random():
    """Random byte pairs / one-byte literals: lane-end artifacts, short and
    long buffers, every alignment mod 64 — device == oracle."""
    from test_cpu_oracle import placed
    rng = random.Random(77)
    for trial in range(24):
        alpha = bytes(rng.sample(range(256), rng.randint(2, 12)))
        pairs = [(rng.choice(alpha), rng.choice(alpha)) for _ in range(rng.randint(0, 5))]
        one = bytes(rng.sample(alpha, rng.randint(0, 2)))
        m = vsa.shufti_build_double_masks(pairs, one)
        if m is None or (not pairs and not one):
            continue
        for vsize in (16, 32, 64):
            vsa.set_accel_vector_size(vsize)
            for n in (1, 7, 15, 16, 17, 31, 33, 63, 64, 65, 100, 200, 1000):
                data = bytes(rng.choice(alpha + b"..") for _ in range(n))
                mis = rng.randrange(64)
                keep, addr = placed(data, mis)
                r = vsa.shufti_double_find(*m, addr, n)
                want = oracle.shufti_double(*m, data, vector_size=vsize, mis=addr % vsize)
                assert r == want, (trial, vsize, n, mis)
    vsa.set_accel_vector_size(64)


@pytest.mark.parametrize("nlits", [1, 30, 500])
def test_gpu_many_small_blocks(ctx, nlits):
    """Thousands of small blocks in one launch (hsbench-style corpora): runs
    of blocks shorter than half a segment are packed whole into one segment
    (runtime.hip build_plan); every block still scans as its own hwlmExec
    call.  Same answers with packing disabled (VSA_NO_GROUPS)."""
    import os
    rng = random.Random(77 + nlits)
    lits = rand_lits(rng, nlits, minlen=1 if nlits == 1 else 2, maxlen=8)
    blob = vsa.hwlm_build(lits)
    sizes = [0, 1, 2, 7, 15, 16, 17, 100, 1023, 1024, 1025, 2047, 2048, 3000, 9000, 40000]
    bufs = [rand_data(rng, rng.choice(sizes)) for _ in range(3000)]
    starts = [rng.choice([0, 0, 0, 1, 5, 17]) if b else 0 for b in bufs]
    starts = [s if s < max(1, len(b)) else 0 for s, b in zip(starts, bufs)]
    want = []
    for b, s in zip(bufs, starts):
        if s >= len(b):
            want.append([])
            continue
        st, m = oracle.hwlm_exec(blob.ptr, b, start=s, cap=1 << 16)
        want.append(m)
    for mis in (0, 5):
        assert batch_run(ctx, blob, bufs, starts=starts, misalign=mis) == want
    os.environ["VSA_NO_GROUPS"] = "1"
    try:
        assert batch_run(ctx, blob, bufs, starts=starts) == want
    finally:
        del os.environ["VSA_NO_GROUPS"]


def test_gpu_plan_reuse(ctx):
    """vsa_plan_create / vsa_scan_plan: the tables built once give the same
    records as vsa_scan_blocks, scan after scan and for another database."""
    rng = random.Random(5)
    lits = rand_lits(rng, 200, minlen=2, maxlen=8)
    blob = vsa.hwlm_build(lits)
    blob2 = vsa.hwlm_build(rand_lits(rng, 20, minlen=2, maxlen=8))
    bufs = [rand_data(rng, rng.choice([1, 17, 1000, 3000, 20000])) for _ in range(500)]
    offs, pos = [], 3
    for b in bufs:
        offs.append(pos)
        pos += len(b) + 1
    host = np.zeros(pos + 16, np.uint8)
    for o, b in zip(offs, bufs):
        host[o:o + len(b)] = np.frombuffer(b, np.uint8)
    d = ctx.malloc(len(host))
    try:
        ctx.h2d(d, host)
        lens = [len(b) for b in bufs]
        for bl in (blob, blob2):
            db = vsa.Database(ctx, bl)
            n = ctx.scan_blocks(db, d, offs, lens)
            want = ctx.results(n)
            plan = ctx.plan(d, offs, lens)
            for _ in range(3):
                m = ctx.scan_plan(db, plan)
                got = ctx.results(m)
                assert m == n
                assert np.array_equal(got["key"], want["key"])
                assert np.array_equal(got["id"], want["id"])
            plan.close()
            db.close()
    finally:
        ctx.free(d)


def test_gpu_binned_sort(ctx):
    """The scan's records come back in key order whichever sort ran: the
    binned sort (sparse records), the library sort after a crowded bin (one
    end position matched by 80 literals), and the launches after it that
    skip the histogram.  Checked against the unsorted records sorted here."""
    rng = random.Random(11)
    sparse = vsa.hwlm_build(rand_lits(rng, 300, minlen=3, maxlen=8))
    crowd = vsa.hwlm_build([vsa.HwlmLiteral(b"ab", False, 10 + i) for i in range(80)] +
                           [vsa.HwlmLiteral(b"bab", False, 5)])
    host = np.frombuffer(rand_data(rng, 3 << 20), np.uint8).copy()
    host[1000:1400] = np.frombuffer(b"ab" * 200, np.uint8)
    d = ctx.malloc(len(host))
    try:
        ctx.h2d(d, host)
        offs, lens = [0, 1 << 20, 2 << 20], [1 << 20, 1 << 20, (1 << 20) - 7]
        dbs = [vsa.Database(ctx, sparse), vsa.Database(ctx, crowd)]
        for k in [0, 1] + [0] * 20:
            db = dbs[k]
            n = ctx.scan_blocks(db, d, offs, lens, sort=False)
            raw = ctx.results(n)
            order = np.argsort(raw["key"], kind="stable")
            m = ctx.scan_blocks(db, d, offs, lens)
            got = ctx.results(m)
            assert m == n and n > 0
            assert np.array_equal(got["key"], raw["key"][order])
            assert np.array_equal(got["id"], raw["id"][order])
        for db in dbs:
            db.close()
    finally:
        ctx.free(d)


def test_gpu_binned_sort_every_fill():
    """vsa_bin_finish at every bin fill 1..64 (every sorting network size,
    S = 2..64, and every mix of sizes among a wave's 4 bins): a block just
    under 2 MiB has 128-byte bins (bin_shift_for); 1,500 bins get f back-to-back "zq"
    (f random, ends inside the bin) over filler without 'z' / 'q', scanned
    with databases of one, two and three literals "zq" (1 / 2 / 3 records
    per occurrence, every bin <= 64 records: no crowd, one launch each).
    The binned result == the unsorted scan's records sorted here.  A fresh
    context: no bin_skip carried over from a crowded test."""
    ctx = vsa.Context(0)
    rng = random.Random(23)
    nprng = np.random.default_rng(23)
    # span < 2^21: end_bits 21, 128-byte bins (2^21 itself needs 22 bits)
    host = nprng.integers(ord("a"), ord("p") + 1, (2 << 20) - 64, dtype=np.uint8)
    d = ctx.malloc(len(host))
    try:
        for reps, fmax in ((1, 59), (2, 32), (3, 21)):
            buf = host.copy()
            for b in range(40, 40 + 1500):
                f = rng.randint(1, fmax)
                o = b * 128 + rng.randint(0, 128 - 2 * f - 1)
                buf[o:o + 2 * f] = np.frombuffer(b"zq" * f, np.uint8)
            ctx.h2d(d, buf)
            db = vsa.Database(ctx, vsa.hwlm_build(
                [vsa.HwlmLiteral(b"zq", False, 7 + i) for i in range(reps)]))
            n = ctx.scan_blocks(db, d, [0], [len(buf)], sort=False)
            raw = ctx.results(n)
            order = np.argsort(raw["key"], kind="stable")
            l0 = ctx.launches()
            m = ctx.scan_blocks(db, d, [0], [len(buf)])
            assert ctx.launches() == l0 + 1  # binned, not rerun
            got = ctx.results(m)
            assert m == n and n >= reps * 1500
            assert np.array_equal(got["key"], raw["key"][order])
            assert np.array_equal(got["id"], raw["id"][order])
            db.close()
    finally:
        ctx.free(d)
        ctx.close()


def test_gpu_crowded_bin_plans(ctx):
    """A binned scan's records live only in its sort bins, so a crowded bin
    (> VSA_SORT_BIN_MAX records) makes the scan run again without bins:
    through a plan (sync and asynchronous + wait) and through the packed
    collective buffer (header flagged not-ready until the host completes).
    Every result == the unsorted scan's records sorted here."""
    vsa_ctx = vsa.Context(0)  # a fresh context: no bin_skip carried over
    try:
        crowd = vsa.Database(vsa_ctx, vsa.hwlm_build(
            [vsa.HwlmLiteral(b"ab", False, 10 + i) for i in range(80)] +
            [vsa.HwlmLiteral(b"bab", False, 5)]))
        rng = random.Random(41)
        host = np.frombuffer(rand_data(rng, 2 << 20), np.uint8).copy()
        host[5000:5400] = np.frombuffer(b"ab" * 200, np.uint8)
        d = vsa_ctx.malloc(len(host))
        try:
            vsa_ctx.h2d(d, host)
            offs, lens = [0, 1 << 20], [1 << 20, (1 << 20) - 3]
            n0 = vsa_ctx.scan_blocks(crowd, d, offs, lens, sort=False)
            raw = vsa_ctx.results(n0)
            order = np.argsort(raw["key"], kind="stable")
            want_k, want_i = raw["key"][order], raw["id"][order]

            def check(n):
                got = vsa_ctx.results(n)
                assert n == n0
                assert np.array_equal(got["key"], want_k) and np.array_equal(got["id"], want_i)

            for mode in ("sync", "async", "pack", "plan_pack"):
                fresh = vsa.Context(0)
                try:
                    db = vsa.Database(fresh, vsa.hwlm_build(
                        [vsa.HwlmLiteral(b"ab", False, 10 + i) for i in range(80)] +
                        [vsa.HwlmLiteral(b"bab", False, 5)]))
                    plan = fresh.plan(d, offs, lens)
                    if mode == "sync":
                        n = fresh.scan_plan(db, plan)
                    elif mode == "plan_pack":
                        # the fused pack of a crowded launch: header flagged
                        # not ready; the host completes (rescan without
                        # bins) and repacks
                        cap = n0 + 16
                        buf = fresh.malloc(8 * (1 + cap + (cap + 1) // 2))
                        fresh.scan_plan_pack(db, plan, buf, cap)
                        n = fresh.scan_wait()
                        hdr = np.zeros(1, np.uint64)
                        fresh.d2h(hdr, buf)
                        assert int(hdr[0]) >> 62 & 1
                        fresh.scan_pack(buf, cap)
                        pk = np.zeros(1 + cap + (cap + 1) // 2, np.uint64)
                        fresh.d2h(pk, buf)
                        fresh.free(buf)
                        assert int(pk[0]) == n0
                        assert np.array_equal(pk[1:1 + n0], want_k)
                        assert np.array_equal(pk[1 + cap:].view(np.uint32)[:n0], want_i)
                    else:
                        fresh.scan_plan(db, plan, asynchronous=True)
                        if mode == "pack":
                            cap = n0 + 16
                            buf = fresh.malloc(8 * (1 + cap) + 4 * cap)
                            fresh.scan_pack(buf, cap)
                            hdr = np.zeros(1, np.uint64)
                            fresh.d2h(hdr, buf)
                            fresh.free(buf)
                            assert int(hdr[0]) >> 62 & 1  # not ready: the host completes
                        n = fresh.scan_wait()
                    got = fresh.results(n)
                    assert n == n0, mode
                    assert np.array_equal(got["key"], want_k), mode
                    assert np.array_equal(got["id"], want_i), mode
                    plan.close()
                    db.close()
                finally:
                    fresh.close()
            check(vsa_ctx.scan_blocks(crowd, d, offs, lens))
        finally:
            vsa_ctx.free(d)
            crowd.close()
    finally:
        vsa_ctx.close()


@pytest.mark.parametrize("fused", [False, True])
def test_gpu_plan_pack_fused(ctx, fused):
    """vsa_scan_plan_pack: the binned sort writes the records into the
    collective buffer itself (no vsa_pack launch).  Over ragged blocks with
    sparse records, pipelined over two contexts on one stream as bench.py
    does: header = the count, keys and ids == the scan's own sorted results,
    and a buffer too small keeps its first cap records with the full count
    in the header (the caller regrows and repacks).  With the binned sort
    launch and with the fused finish (the scan packs itself)."""
    rng = random.Random(17)
    ctx.fused_finish(fused)
    blob = vsa.hwlm_build(rand_lits(rng, 400, minlen=3, maxlen=8))
    host = np.frombuffer(rand_data(rng, 6 << 20), np.uint8).copy()
    c2 = vsa.Context(share_stream_with=ctx)
    d = ctx.malloc(len(host))
    try:
        ctx.h2d(d, host)
        offs, lens = [0, 3 << 20, (5 << 20) + 5], [(3 << 20) - 1, 2 << 20, 777000]
        assert c2.last_fused() is False
        fused_seen = []
        dbs = [vsa.Database(ctx, blob), vsa.Database(c2, blob)]
        plans = [ctx.plan(d, offs, lens), c2.plan(d, offs, lens)]
        want = None
        for k in range(6):
            c, db, pl = (ctx, c2)[k % 2], dbs[k % 2], plans[k % 2]
            n = c.scan_plan(db, pl)
            got = c.results(n)
            if want is None:
                want = got
            assert np.array_equal(got["key"], want["key"]) and n > 1000
            for cap in (n + 5, n // 3):
                buf = c.malloc(8 * (1 + cap + (cap + 1) // 2))
                c.scan_plan_pack(db, pl, buf, cap)
                assert c.scan_wait() == n
                pk = np.zeros(1 + cap + (cap + 1) // 2, np.uint64)
                c.d2h(pk, buf)
                c.free(buf)
                m = min(n, cap)
                assert int(pk[0]) == n, (k, cap)
                assert np.array_equal(pk[1:1 + m], want["key"][:m]), (k, cap)
                assert np.array_equal(pk[1 + cap:].view(np.uint32)[:m], want["id"][:m]), (k, cap)
                fused_seen.append(c.last_fused())
        # (the shared fixture context may still skip bins after an earlier
        # test's crowd: then some launches take the library sort)
        assert any(fused_seen) == fused
        for p_ in plans:
            p_.close()
        for db in dbs:
            db.close()
    finally:
        ctx.fused_finish(False)
        ctx.free(d)
        c2.close()


def test_gpu_fused_finish():
    """The fused finish (kernels.hip fused_finish, plan.hip plan_fused): a
    plan of >= 64 workgroups whose end ranges ascend is sorted by the scan
    kernel itself -- local bins counted in LDS, a look-back over the lower
    workgroups' totals, the last workgroup publishing -- with no
    vsa_bin_finish launch (vsa_ctx_set_fused_finish; off by default).  On a
    fresh context per case with it on: last_fused() is set
    and the records equal the unsorted scan's sorted here, for FDR over 4
    blocks, a stripe window with report_lo, 16 KiB back-to-back blocks
    (runs), noodle and Teddy databases, 30 launches in a row (one epoch
    each), a first launch that outgrows the output (rerun, fused again) and
    a crowded local bin (rerun without bins)."""
    rng = random.Random(31)
    host = np.frombuffer(rand_data(rng, 24 << 20), np.uint8).copy()
    host[(9 << 20) + 100:(9 << 20) + 700] = np.frombuffer(b"ab" * 300, np.uint8)
    dbs = {
        "fdr": vsa.hwlm_build(rand_lits(rng, 300, minlen=3, maxlen=8)),
        "noodle": vsa.hwlm_build([vsa.HwlmLiteral(b"q\x01", False, 3)]),
        "teddy": vsa.hwlm_build(rand_lits(rng, 20, minlen=3, maxlen=6)),
        "crowd": vsa.hwlm_build([vsa.HwlmLiteral(b"ab", False, 10 + i) for i in range(40)]),
    }
    q = 6 << 20
    layouts = {
        "blocks": ([0, q, 2 * q, 3 * q], [q, q, q, q - 5], None),
        "window": ([(8 << 20) - 7], [(12 << 20) + 7], [7]),
        "runs": ([i << 14 for i in range(1024)], [1 << 14] * 1024, None),
    }
    c0 = vsa.Context(0)
    d = c0.malloc(len(host))
    try:
        c0.h2d(d, host)
        for name, blob in dbs.items():
            for lname, (offs, lens, rlo) in layouts.items():
                c = vsa.Context(0)
                c.fused_finish(True)
                try:
                    db = vsa.Database(c, blob)
                    n0 = c.scan_blocks_ex(db, d, offs, lens, report_lo=rlo, sort=False)
                    raw = c.results(n0)
                    order = np.argsort(raw["key"], kind="stable")
                    for k in range(30 if (name, lname) == ("fdr", "blocks") else 3):
                        l0 = c.launches()
                        n = c.scan_blocks_ex(db, d, offs, lens, report_lo=rlo)
                        got = c.results(n)
                        assert n == n0, (name, lname, k)
                        assert np.array_equal(got["key"], raw["key"][order]), (name, lname, k)
                        assert np.array_equal(got["id"], raw["id"][order]), (name, lname, k)
                        if name == "crowd" and k == 0:
                            # crowded: rerun without bins, then bins skipped
                            assert c.launches() == l0 + 2 and not c.last_fused()
                        elif name != "crowd":
                            assert c.last_fused(), (name, lname, k)
                            assert c.launches() == l0 + 1 or (k == 0 and n > 65536)
                    db.close()
                finally:
                    c.close()
    finally:
        c0.free(d)
        c0.close()


def test_gpu_sampled_timing():
    """vsa_ctx_set_timing: every 3rd launch carries the kernel-timing events
    (kernel_ms > 0), the others report -1; 0 times none; results are the
    same whatever is timed, with the binned sort and the fused finish."""
    rng = random.Random(37)
    blob = vsa.hwlm_build(rand_lits(rng, 200, minlen=4, maxlen=8))
    host = np.frombuffer(rand_data(rng, 8 << 20), np.uint8).copy()
    c = vsa.Context(0)
    try:
        d = c.malloc(len(host))
        c.h2d(d, host)
        db = vsa.Database(c, blob)
        pl = c.plan(d, [0, 4 << 20], [4 << 20, 4 << 20])
        want = c.results(c.scan_plan(db, pl))
        assert c.kernel_ms() > 0
        for fused in (False, True):
            c.fused_finish(fused)
            c.timing(3)
            timed = []
            for _ in range(9):
                got = c.results(c.scan_plan(db, pl))
                assert np.array_equal(got["key"], want["key"])
                assert np.array_equal(got["id"], want["id"])
                timed.append(c.kernel_ms() > 0)
            assert sum(timed) == 3, timed
            c.timing(0)
            c.scan_plan(db, pl)
            assert c.kernel_ms() == -1.0
            c.timing(1)
            c.scan_plan(db, pl)
            assert c.kernel_ms() > 0
        pl.close()
        db.close()
        c.free(d)
    finally:
        c.close()


def test_gpu_reserved_cus_same_records():
    """vsa_ctx_set_reserved_cus (CUs left free beside the scan's persistent
    grid; measured, not used by bench.py): plans on a context with 1 or 7 CUs reserved --
    per-call and prebuilt, and a shared context inheriting the reserve --
    give the same sorted records as the full grid."""
    rng = random.Random(23)
    blob = vsa.hwlm_build(rand_lits(rng, 700, minlen=3, maxlen=8))
    host = np.frombuffer(rand_data(rng, 9 << 20), np.uint8).copy()
    full = vsa.Context(0)
    try:
        d = full.malloc(len(host))
        try:
            full.h2d(d, host)
            offs, lens = [0, 5 << 20, (7 << 20) + 3], [5 << 20, 2 << 20, (2 << 20) - 9]
            db = vsa.Database(full, blob)
            want = full.results(full.scan_blocks(db, d, offs, lens))
            assert len(want) > 1000
            for r in (1, 7):
                c = vsa.Context(0)
                c.reserve_cus(r)
                c2 = vsa.Context(share_stream_with=c)
                try:
                    cdb = vsa.Database(c, blob)
                    got = c.results(c.scan_blocks(cdb, d, offs, lens))
                    assert np.array_equal(got["key"], want["key"]), r
                    assert np.array_equal(got["id"], want["id"]), r
                    pl = c2.plan(d, offs, lens)
                    got2 = c2.results(c2.scan_plan(cdb, pl))
                    assert np.array_equal(got2["key"], want["key"]), r
                    pl.close()
                    cdb.close()
                finally:
                    c2.close()
                    c.close()
            db.close()
        finally:
            full.free(d)
    finally:
        full.close()


def test_gpu_crowded_bin_rerun_count():
    """a first dense scan on a fresh context outgrows the output
    (out_cap starts at 64 K records) AND crowds a sort bin.  It must rerun
    once, without bins (2 launches, not 3), and a persistently dense
    workload backs off: after a crowded binned launch 16 launches (its rerun
    included) skip the bins, after the next crowded one 64 (bin_backoff).  Every result equals
    the unsorted scan's records sorted here."""
    lits = [vsa.HwlmLiteral(b"ab", False, 10 + i) for i in range(80)] + \
           [vsa.HwlmLiteral(b"bab", False, 5)]
    rng = random.Random(43)
    host = np.frombuffer(rand_data(rng, 2 << 20), np.uint8).copy()
    host[9000:11000] = np.frombuffer(b"ab" * 1000, np.uint8)  # ~80 K records
    ref = vsa.Context(0)
    c = vsa.Context(0)
    try:
        rdb = vsa.Database(ref, vsa.hwlm_build(lits))
        db = vsa.Database(c, vsa.hwlm_build(lits))
        d = c.malloc(len(host))
        try:
            c.h2d(d, host)
            offs, lens = [0, 1 << 20], [1 << 20, (1 << 20) - 5]
            n0 = ref.scan_blocks(rdb, d, offs, lens, sort=False)
            assert n0 > 65536
            raw = ref.results(n0)
            order = np.argsort(raw["key"], kind="stable")
            want_k, want_i = raw["key"][order], raw["id"][order]
            plan = c.plan(d, offs, lens)
            launches = []
            for k in range(18):
                l0 = c.launches()
                n = c.scan_plan(db, plan)
                launches.append(c.launches() - l0)
                got = c.results(n)
                assert n == n0, k
                assert np.array_equal(got["key"], want_k), k
                assert np.array_equal(got["id"], want_i), k
            # scan 0: binned, crowded + output overflow -> one rerun without
            # bins (the first of the 16 launches that skip them); scans 1-15
            # skip them; scan 16 is binned again and crowds again -> one
            # rerun, and the next 64 launches skip (scan 17)
            assert launches == [2] + [1] * 15 + [2, 1], launches
            plan.close()
        finally:
            c.free(d)
            db.close()
            rdb.close()
    finally:
        c.close()
        ref.close()


def test_gpu_overlapping_blocks_dense(ctx):
    """Blocks that overlap each other (the runtime then owns no sort bin in
    any workgroup, plan_wg_bins) and blocks that do not (bins counted in LDS),
    with a match every few bytes: every block's records == the oracle's for
    that block, and the sorted output is in key order."""
    rng = random.Random(29)
    lits = rand_lits(rng, 200, minlen=3, maxlen=7)
    blob = vsa.hwlm_build(lits)
    host = np.frombuffer(b"abcdefghABCDEFGH", np.uint8)[
        np.random.default_rng(29).integers(0, 16, 3 << 20)]
    for p in range(0, len(host) - 16, 97):
        w = lits[rng.randrange(len(lits))].s
        host[p:p + len(w)] = np.frombuffer(w, np.uint8)
    d = ctx.malloc(len(host))
    try:
        ctx.h2d(d, host)
        db = vsa.Database(ctx, blob)
        for offs, lens in (([0, 1 << 20, (5 << 19) + 3], [2 << 20, 2 << 20, (1 << 19) - 9]),
                           ([0, (1 << 20) + 5, 2 << 20], [(1 << 20) + 5, (1 << 20) - 5, 1 << 20])):
            want = []
            for o, ln in zip(offs, lens):
                _, m = oracle.hwlm_exec(blob.ptr, host[o:o + ln].tobytes(), cap=1 << 21)
                want += [(o + e, i) for e, i in m]
            n = ctx.scan_blocks(db, d, offs, lens)
            got = ctx.results(n)
            assert n == len(want) and n > 20000
            assert np.all(np.diff(got["key"].astype(np.int64)) >= 0)
            ends = (got["key"] >> np.uint64(24)).tolist()
            assert sorted(zip(ends, got["id"].tolist())) == sorted(want)
        db.close()
    finally:
        ctx.free(d)


def test_gpu_plan_memo(ctx):
    """A repeated block list reuses the device tables of the previous call;
    any change (an offset, a length, a start, the buffer) rebuilds them."""
    rng = random.Random(23)
    db = vsa.Database(ctx, vsa.hwlm_build(rand_lits(rng, 150, minlen=2, maxlen=8)))
    host = np.frombuffer(rand_data(rng, 1 << 20), np.uint8).copy()
    d = ctx.malloc(len(host) + 64)
    try:
        ctx.h2d(d, host)
        offs = [0, 1000, 5000, 300000]
        lens = [900, 3000, 200000, 700000]

        def run(o, l, starts=None, ptr=d):
            n = ctx.scan_blocks(db, ptr, o, l, starts)
            return ctx.results(n)

        base = run(offs, lens)
        variants = [(offs, lens[:3] + [600000], None, d), (offs[:3] + [300016], lens, None, d),
                    (offs, lens, [0, 10, 0, 5], d), (offs, lens, None, d + 16)]
        for o, l, st, ptr in variants:
            plan = ctx.plan(ptr, o, l, st)  # tables built from scratch
            want = ctx.results(ctx.scan_plan(db, plan))
            plan.close()
            for _ in range(2):  # a rebuild, then the memoised tables
                got = run(o, l, st, ptr)
                assert np.array_equal(got["key"], want["key"])
                assert np.array_equal(got["id"], want["id"])
            back = run(offs, lens)
            assert np.array_equal(back["key"], base["key"])
            assert np.array_equal(back["id"], base["id"])
        db.close()
    finally:
        ctx.free(d)


def run_layout_scan(ctx, blob, bufs, misalign=0):
    """bufs laid back to back (no gaps: hsbench corpora), one launch;
    per-block [(end, id)]"""
    offs, pos = [], misalign
    for b in bufs:
        offs.append(pos)
        pos += len(b)
    host = np.zeros(pos + 16, np.uint8)
    for o, b in zip(offs, bufs):
        host[o:o + len(b)] = np.frombuffer(bytes(b), np.uint8)
    dbuf = ctx.malloc(len(host))
    try:
        ctx.h2d(dbuf, host)
        db = vsa.Database(ctx, blob)
        n = ctx.scan_blocks(db, dbuf, offs, [len(b) for b in bufs])
        res = ctx.results(n)
        db.close()
    finally:
        ctx.free(dbuf)
    out = [[] for _ in bufs]
    ends = res["key"] >> np.uint64(24)
    bi = np.searchsorted(np.array(offs, np.uint64), ends, side="right") - 1
    for e, i, b in zip(ends.tolist(), res["id"].tolist(), bi.tolist()):
        out[b].append((e - offs[b], i))
    return out


@pytest.mark.parametrize("nlits", [1, 5, 30, 300, 3000])
def test_gpu_back_to_back_runs(ctx, nlits):
    """Back-to-back block-mode blocks >= 1 KiB packed into one segment are
    scanned as one range (VSA_BLK_RUN, kernels.hip "runs"): every block's
    records equal the oracle's hwlmExec of that block alone -- with literals
    planted across every boundary (never reported), whole literals at block
    starts and ends (reported), masks reaching before the literal -- at the
    planner's segment size and at 128 KiB segments (runs of up to 128
    blocks), and equal the per-block path (VSA_NO_RUNS)."""
    import os
    rng = random.Random(900 + nlits)
    lo = 1 if nlits == 1 else (2 if nlits <= 30 else 4)
    lits = rand_lits(rng, nlits, minlen=max(lo, 2) if nlits > 1 else 3, maxlen=8,
                     msk_frac=0.15)
    blob = vsa.hwlm_build(lits)
    alpha = b"abcdefghABCDEFGH" if nlits <= 30 else bytes(range(0x61, 0x7b))
    sizes = [1024, 1025, 1500, 2047, 2048, 3000, 4096, 9000, 16384, 40000]
    bufs = [bytearray(rand_data(rng, rng.choice(sizes), alpha)) for _ in range(700)]
    for k in range(len(bufs) - 1):
        s = rng.choice(lits).s
        if len(s) > 1:  # across the boundary k | k + 1
            cut = rng.randint(1, len(s) - 1)
            bufs[k][len(bufs[k]) - cut:] = s[:cut]
            bufs[k + 1][:len(s) - cut] = s[cut:]
        if rng.random() < 0.3:  # whole literal ending the block / starting the next
            t = rng.choice(lits).s
            bufs[k][len(bufs[k]) - len(t):] = t
            u = rng.choice(lits).s
            bufs[k + 1][:len(u)] = u
    want = []
    for b in bufs:
        st, m = oracle.hwlm_exec(blob.ptr, bytes(b), cap=1 << 18)
        assert st == 0
        want.append(m)
    assert sum(map(len, want)) > 100
    for mis in (0, 3):
        assert run_layout_scan(ctx, blob, bufs, mis) == want, mis
    os.environ["VSA_SEG_KB"] = "128"
    try:
        assert run_layout_scan(ctx, blob, bufs, 5) == want
    finally:
        del os.environ["VSA_SEG_KB"]
    os.environ["VSA_NO_RUNS"] = "1"
    try:
        assert run_layout_scan(ctx, blob, bufs) == want
    finally:
        del os.environ["VSA_NO_RUNS"]


@pytest.mark.parametrize("nlits", [1, 30, 500, 3000])
def test_gpu_scanner_expansion(ctx, nlits, monkeypatch):
    """Scanner expansion (VSA_XP=1, kernels.hip xp_push: the scanning waves
    expand candidate bits, apply the slot-bitmap prefilter and push confirm
    entries; the runtime turns it on for large literal sets) forced on small
    sets: per-block records equal the oracle's hwlmExec of each block, for
    ragged blocks with starts and misalignment, back-to-back runs with
    literals across every boundary, and one or two confirm waves."""
    rng = random.Random(4200 + nlits)
    lits = rand_lits(rng, nlits, minlen=1 if nlits == 1 else 2, maxlen=8, msk_frac=0.15)
    blob = vsa.hwlm_build(lits)
    sizes = [0, 1, 2, 7, 15, 16, 17, 100, 1023, 1024, 1025, 2047, 3000, 9000, 40000]
    bufs = [rand_data(rng, rng.choice(sizes)) for _ in range(1500)]
    starts = [rng.choice([0, 0, 0, 1, 5, 17]) if b else 0 for b in bufs]
    starts = [s if s < max(1, len(b)) else 0 for s, b in zip(starts, bufs)]
    want = []
    for b, s in zip(bufs, starts):
        if s >= len(b):
            want.append([])
            continue
        st, m = oracle.hwlm_exec(blob.ptr, b, start=s, cap=1 << 16)
        want.append(m)
    monkeypatch.setenv("VSA_XP", "1")
    for nconf in ("1", "2"):
        monkeypatch.setenv("VSA_NCONF", nconf)
        for mis in (0, 5):
            assert batch_run(ctx, blob, bufs, starts=starts, misalign=mis) == want, (nconf, mis)
    # back-to-back runs with literals across the boundaries
    alpha = b"abcdefghABCDEFGH" if nlits <= 30 else bytes(range(0x61, 0x7b))
    rb = [bytearray(rand_data(rng, rng.choice([1024, 1500, 2048, 4096, 16384]), alpha))
          for _ in range(300)]
    for k in range(len(rb) - 1):
        s = rng.choice(lits).s
        if len(s) > 1:
            cut = rng.randint(1, len(s) - 1)
            rb[k][len(rb[k]) - cut:] = s[:cut]
            rb[k + 1][:len(s) - cut] = s[cut:]
    want = [oracle.hwlm_exec(blob.ptr, bytes(b), cap=1 << 18)[1] for b in rb]
    assert run_layout_scan(ctx, blob, rb, 3) == want


@pytest.mark.parametrize("nlits", [1, 30, 500, 3000])
def test_gpu_split_passes(ctx, nlits, monkeypatch):
    """Split passes (VSA_SPLIT=1; runtime.hip turns them on for large
    literal sets): one launch per bit 0 of the end byte, each with the
    first-stage table of the literals whose last byte has that bit (both
    for a last byte whose mask leaves bit 0 free), into one output.  Forced
    on small sets with masked literals: per-block records equal the
    oracle's hwlmExec of each block, for ragged blocks with starts and
    misalignment, with scanner expansion off and on, and back-to-back runs
    with literals across every boundary."""
    rng = random.Random(5300 + nlits)
    lits = rand_lits(rng, nlits, minlen=1 if nlits == 1 else 2, maxlen=8, msk_frac=0.3)
    blob = vsa.hwlm_build(lits, engine_hint=0, allow_noodle=False)
    if blob.engine_id != 0:
        pytest.skip("split passes are an FDR schedule (engine %d)" % blob.engine_id)
    sizes = [0, 1, 2, 7, 15, 16, 17, 100, 1023, 1024, 1025, 2047, 3000, 9000, 40000]
    bufs = [rand_data(rng, rng.choice(sizes)) for _ in range(1200)]
    starts = [rng.choice([0, 0, 0, 1, 5, 17]) if b else 0 for b in bufs]
    starts = [s if s < max(1, len(b)) else 0 for s, b in zip(starts, bufs)]
    want = []
    for b, s in zip(bufs, starts):
        if s >= len(b):
            want.append([])
            continue
        st, m = oracle.hwlm_exec(blob.ptr, b, start=s, cap=1 << 16)
        want.append(m)
    monkeypatch.setenv("VSA_SPLIT", "1")
    for xp in ("0", "1"):
        monkeypatch.setenv("VSA_XP", xp)
        for mis in (0, 5):
            assert batch_run(ctx, blob, bufs, starts=starts, misalign=mis) == want, (xp, mis)
    monkeypatch.delenv("VSA_XP")
    alpha = b"abcdefghABCDEFGH" if nlits <= 30 else bytes(range(0x61, 0x7b))
    rb = [bytearray(rand_data(rng, rng.choice([1024, 1500, 2048, 4096, 16384]), alpha))
          for _ in range(300)]
    for k in range(len(rb) - 1):
        s = rng.choice(lits).s
        if len(s) > 1:
            cut = rng.randint(1, len(s) - 1)
            rb[k][len(rb[k]) - cut:] = s[:cut]
            rb[k + 1][:len(s) - cut] = s[cut:]
    want = [oracle.hwlm_exec(blob.ptr, bytes(b), cap=1 << 18)[1] for b in rb]
    assert run_layout_scan(ctx, blob, rb, 3) == want
    # one stream cut into writes of ragged sizes, each with up to 16 history
    # bytes before it: the same records as the whole buffer in one block
    whole = b"".join(bytes(b) for b in rb)
    cuts = [0]
    while cuts[-1] < len(whole):
        cuts.append(min(len(whole), cuts[-1] + rng.choice([1, 7, 100, 1023, 1024, 5000, 40000])))
    offs = np.array(cuts[:-1], np.uint64)
    lens = np.diff(np.array(cuts, np.uint64))
    hl = np.minimum(offs, 16).astype(np.uint64)
    host = np.frombuffer(whole, np.uint8)
    st, m = oracle.hwlm_exec(blob.ptr, whole, cap=1 << 22)
    d = ctx.malloc(len(host) + 64)
    try:
        ctx.h2d(d, host)
        for split in ("0", "1"):
            monkeypatch.setenv("VSA_SPLIT", split)
            db = vsa.Database(ctx, blob)
            k = ctx.scan_blocks_stream(db, d, offs, lens, hl)
            got = ctx.results(k)
            db.close()
            ends = (got["key"] >> np.uint64(24)).tolist()
            assert list(zip(ends, got["id"].tolist())) == m, split
    finally:
        ctx.free(d)


def test_gpu_plan_free_after_async_overflow():
    """a plan freed while its asynchronous scan is still pending
    -- a scan that overflows the output (its rescan reads the plan's tables)
    -- is completed before the tables go (vsa_plan_free), and the scan's
    count still reads back right; a plan outliving its context frees only
    its own tables."""
    ctx = vsa.Context(0)
    lits = [vsa.HwlmLiteral(b"ab", False, 1), vsa.HwlmLiteral(b"bab", False, 2)]
    blob = vsa.hwlm_build(lits)
    n = 1 << 20
    host = np.frombuffer(b"ab" * (n // 2), np.uint8)
    want = n // 2 + (n // 2 - 1)  # every "ab", every "bab"
    d = ctx.malloc(n + 64)
    db = vsa.Database(ctx, blob)
    try:
        ctx.h2d(d, host)
        for _ in range(2):
            plan = ctx.plan(d, [0], [n])
            ctx.scan_plan(db, plan, asynchronous=True)  # > 65,536 records: overflows
            plan.close()                                  # completes the scan first
            assert ctx.scan_wait() == want
        plan = ctx.plan(d, [0], [n])
        assert ctx.scan_plan(db, plan) == want
        db.close()
        ctx.free(d)
        d = None
        ctx.close()      # the plan outlives its context
        plan.close()
    finally:
        if d is not None:
            ctx.free(d)
