"""GPU parity for streaming mode (fdrExecStreaming fdr.c:827,
noodExecStreaming noodle_engine.cpp:136, hwlmExecStreaming hwlm.c:207) and
for the HWLM header accel schemes (do_accel_block / do_accel_streaming,
hwlm.c:85-175): the HIP engine through the C ABI against the oracle, match
lists compared bit-exactly in callback order."""
import random

import numpy as np
import pytest

import oracle
import vectorscan_amd as vsa
from test_cpu_oracle import FDR_HINTS, build_or_none, load, rand_data, rand_lits, stream_lits

pytestmark = pytest.mark.gpu

FILLER = oracle.HIST_FILLER


@pytest.fixture(scope="module")
def ctx():
    c = vsa.Context(0)
    yield c
    c.close()


def recorder(term_after=-1, cb_ret=None):
    seq = []

    def cb(end, id_):
        seq.append((end, id_))
        if term_after >= 0 and len(seq) >= term_after:
            return vsa.HWLM_TERMINATE_MATCHING
        return vsa.HWLM_ALL_GROUPS if cb_ret is None else cb_ret

    return seq, cb


@pytest.mark.parametrize("hint", FDR_HINTS)
def test_gpu_golden_fdr_stream(hint):
    """fdr.cpp SmallStreaming / SmallStreaming2 / Stream1 / FDRTermS."""
    for c in load("fdr_stream.json"):
        lits = stream_lits(c)
        blob = build_or_none(lits, hint) if c["hinted"] else vsa.hwlm_build(lits)
        if blob is None or blob.is_noodle:
            continue
        seq, cb = recorder(c["term_after"])
        st = vsa.fdr_exec_stream(blob, bytes.fromhex(c["hist"]), bytes.fromhex(c["data"]),
                                 start=c["start"], cb=cb, filler=FILLER)
        assert st == c["status"], c["src"]
        if c["expected"] is not None:
            assert seq == [tuple(x) for x in c["expected"]], (c["src"], hint)
        if "expected_len" in c:
            assert len(seq) == c["expected_len"], c["src"]


def _stream_case(rng, blob, lits, nhist, ndata, start, groups=vsa.HWLM_ALL_GROUPS):
    hist = rand_data(rng, nhist)
    data = rand_data(rng, ndata)
    st_o, m_o = oracle.hwlm_exec_stream(blob.ptr, hist, data, start=start, groups=groups,
                                        cap=1 << 16)
    st_g, m_g = vsa.hwlm_exec_stream(blob, hist, data, start=start, groups=groups,
                                     filler=FILLER)
    return (st_o, m_o), (st_g, m_g)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("nlits", [1, 2, 7, 30, 96, 400, 3000])
def test_gpu_hwlm_stream_vs_oracle(seed, nlits):
    rng = random.Random(9001 + 31 * seed + nlits)
    lits = rand_lits(rng, nlits, msk_frac=0.15)
    for l in lits:
        l.groups = rng.choice([1, 2, 3, vsa.HWLM_ALL_GROUPS])
    blob = vsa.hwlm_build(lits)
    for nhist in (0, 1, 3, 7, 8, 15, 16, 17, 40, 300):
        for ndata in (1, 2, 9, 16, 17, 33, 257, 5000):
            for start in sorted({0, 1, ndata // 2}):
                if start >= ndata:
                    continue
                for groups in (vsa.HWLM_ALL_GROUPS, 1):
                    want, got = _stream_case(rng, blob, lits, nhist, ndata, start, groups)
                    assert got == want, (nlits, nhist, ndata, start, groups)


@pytest.mark.parametrize("hint", FDR_HINTS)
def test_gpu_fdr_stream_engines(hint):
    rng = random.Random(700 + hint)
    for trial in range(4):
        lits = rand_lits(rng, rng.randint(1, 40), msk_frac=0.1)
        blob = build_or_none(lits, hint)
        if blob is None:
            continue
        eng = vsa.engine_blob(blob)
        for nhist, ndata in ((1, 5), (5, 16), (16, 40), (7, 300), (64, 5000)):
            hist, data = rand_data(rng, nhist), rand_data(rng, ndata)
            for start in (0, 2):
                st_o, m_o = oracle.fdr_exec_stream(eng, hist, data, start=start, cap=1 << 16)
                st_g, m_g = vsa.fdr_exec_stream(blob, hist, data, start=start, filler=FILLER)
                assert (st_g, m_g) == (st_o, m_o), (hint, trial, nhist, ndata, start)


@pytest.mark.parametrize("nocase", [False, True])
def test_gpu_nood_stream(nocase):
    rng = random.Random(55 + nocase)
    for L in range(1, 9):
        lit = vsa.HwlmLiteral(rand_data(rng, L, b"abAB"), nocase, 77)
        blob = vsa.hwlm_build([lit])
        assert blob.is_noodle
        eng = vsa.engine_blob(blob)
        for nhist in (0, 1, 2, L - 1, L, 20):
            for ndata in (1, 2, L - 1, L, 3 * L, 200):
                if ndata < 1:
                    continue
                hist = rand_data(rng, nhist, b"abAB")
                data = rand_data(rng, ndata, b"abAB")
                want = oracle.nood_exec_stream(eng, hist, data, cap=1 << 12)
                got = vsa.nood_exec_stream(blob, hist, data, filler=FILLER)
                assert got == want, (L, nhist, ndata)


def test_gpu_stream_terminate():
    rng = random.Random(3)
    lits = rand_lits(rng, 20, alphabet=b"ab", maxlen=3)
    blob = vsa.hwlm_build(lits)
    hist, data = rand_data(rng, 30, b"ab"), rand_data(rng, 400, b"ab")
    for k in (1, 2, 5, 17):
        st_o, m_o = oracle.hwlm_exec_stream(blob.ptr, hist, data, term_after=k)
        seq, cb = recorder(k)
        st_g = vsa.hwlm_exec_stream(blob, hist, data, cb=cb, filler=FILLER)
        assert (st_g, seq) == (st_o, m_o), k


def test_gpu_stream_chunks_one_launch(ctx):
    """A stream cut into consecutive chunks and scanned as one launch of
    streaming blocks (history = everything before the chunk) reports each
    occurrence exactly once: the match set of one block over the whole
    stream."""
    rng = random.Random(12)
    for nlits in (1, 9, 60, 900):
        lits = rand_lits(rng, nlits, msk_frac=0.1)
        blob = vsa.hwlm_build(lits)
        total = 300000
        data = np.frombuffer(rand_data(rng, total), np.uint8)
        cuts = sorted(set([0, total] + [rng.randrange(1, total) for _ in range(40)] +
                          [5, 6, 7, 20, 21]))
        offs = cuts[:-1]
        lens = [b - a for a, b in zip(cuts, cuts[1:])]
        host = np.zeros(total + 64, np.uint8)
        host[32:32 + total] = data
        dbuf = ctx.malloc(len(host))
        try:
            ctx.h2d(dbuf, host)
            db = vsa.Database(ctx, blob)
            n = ctx.scan_blocks_stream(db, dbuf, [32 + o for o in offs], lens, hlens=offs)
            r = ctx.results(n)
            got = sorted(zip(((r["key"] >> np.uint64(24)) - np.uint64(32)).tolist(),
                             r["id"].tolist()))
            n1 = ctx.scan_blocks(db, dbuf, [32], [total])
            r1 = ctx.results(n1)
            want = sorted(zip(((r1["key"] >> np.uint64(24)) - np.uint64(32)).tolist(),
                              r1["id"].tolist()))
            db.close()
        finally:
            ctx.free(dbuf)
        assert got == want, nlits
        assert set(got) == oracle.brute_force(lits, data.tobytes()), nlits


# ---------------------------------------------------- HWLM header accel ---

def rand_accel(rng):
    kind = rng.choice(["verm", "verm_nocase", "dverm", "dverm_nocase", "shufti", "truffle"])
    off = rng.choice([0, 0, 1, 3, 7])
    chars = b"abcdefghABCDEFGH"
    if kind in ("shufti", "truffle"):
        cls = bytes(rng.sample(list(chars), rng.randint(1, 3)))
        m = (vsa.shufti_build_masks(cls) if kind == "shufti" else vsa.truffle_build_masks(cls))
        return vsa.accel_aux(kind, off, masks=m)
    return vsa.accel_aux(kind, off, rng.choice(chars), rng.choice(chars))


@pytest.mark.parametrize("seed", range(4))
def test_gpu_hwlm_accel_block_and_stream(seed):
    """Arbitrary accel schemes in the HWLM header: block and streaming
    start-skipping must agree with the oracle byte for byte (including
    schemes that skip real matches — the reference skips them too)."""
    rng = random.Random(321 + seed)
    for trial in range(6):
        lits = rand_lits(rng, rng.choice([2, 10, 50, 300]))
        blob = vsa.hwlm_build(lits)
        if blob.is_noodle:
            continue
        g1 = rng.choice([1, 2, 3])
        blob.set_accel(rand_accel(rng), rand_accel(rng), g1)
        for ndata in (10, 16, 17, 40, 300, 4000):
            data = rand_data(rng, ndata)
            for groups in (vsa.HWLM_ALL_GROUPS, g1):
                for start in (0, 3):
                    want = oracle.hwlm_exec(blob.ptr, data, start=start, groups=groups,
                                            cap=1 << 16)
                    got = vsa.hwlm_exec(blob, data, start=start, groups=groups)
                    assert got == want, (seed, trial, ndata, groups, start)
                    for nhist in (0, 5, 16, 40):
                        hist = rand_data(rng, nhist)
                        want = oracle.hwlm_exec_stream(blob.ptr, hist, data, start=start,
                                                       groups=groups, cap=1 << 16)
                        got = vsa.hwlm_exec_stream(blob, hist, data, start=start,
                                                   groups=groups, filler=FILLER)
                        assert got == want, (seed, trial, ndata, groups, start, nhist)
