"""BASELINE configs at parity-test scale through the HIP path (C ABI), bit
exact against the oracle:

* cfg 3 — Teddy / Fat Teddy on the 48-literal (seed 55) and 64-literal
  (seed 71) printable sets, >= 64 MiB printable corpus (seed 3) with a
  literal planted every 4 KiB, for the default engine choice (Fat Teddy 8 on
  an AVX2+ target, teddy_engine_description.cpp:111-115) and forced 8-bucket
  Teddy engines (the SSE build picks 18);
* cfg 4 striping — one corpus of several blocks cut into N rank stripes
  (bench.py's N-GPU split, stripe.plan_corpus_stripes), every stripe scanned
  through vsa_scan_blocks_ex on this one GPU: the union in rank order equals
  the per-block single scans (sequence, not just the set).
"""
import numpy as np
import pytest

import bench
import oracle
import vectorscan_amd as vsa
from vectorscan_amd import stripe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = vsa.Context(0)
    yield c
    c.close()


def cfg3_lits(n):
    """cfg 3 literal sets (tools/bench_configs.py lits_printable): length
    4-8, printable, seed 7 + n (48 -> 55, 64 -> 71)"""
    import random
    r = random.Random(7 + n)
    out = []
    for i in range(n):
        ln = r.randint(4, 8)
        out.append(vsa.HwlmLiteral(bytes(r.randint(0x20, 0x7E) for _ in range(ln)), False, i))
    return out


def scan_one(ctx, blob, data):
    """one device block scan of a host array; sorted (end, id) list"""
    n = len(data)
    d = ctx.malloc(n + 64)
    try:
        ctx.h2d(d, data)
        db = vsa.Database(ctx, blob)
        k = ctx.scan_blocks(db, d, [0], [n])
        res = ctx.results(k)
        db.close()
    finally:
        ctx.free(d)
    return list(zip((res["key"] >> np.uint64(24)).tolist(), res["id"].tolist()))


@pytest.mark.parametrize("nl,hint,engine", [
    (48, -1, 8),    # default choice: Fat Teddy, 4 masks
    (48, 18, 18),   # 8-bucket Teddy, 4 masks, packed (the SSE build's choice)
    (48, 17, 17),   # 8-bucket Teddy, 4 masks
    (48, 11, 11),   # 8-bucket Teddy, 1 mask (many more first-stage candidates)
    (64, -1, 8),    # default choice: Fat Teddy
    (64, 3, 3),     # Fat Teddy, 1 mask
])
def test_gpu_cfg3_teddy_64mib(ctx, nl, hint, engine):
    lits = cfg3_lits(nl)
    blob = vsa.hwlm_build(lits, engine_hint=hint)
    assert blob.engine_id == engine
    data = bench.make_corpus(64 << 20, lits, seed=3, plant_every=4096)
    got = scan_one(ctx, blob, data)
    st, want = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 22)
    assert st == 0
    assert got == want
    assert len(want) >= (64 << 20) // 4096


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gpu_corpus_stripes(ctx, world):
    """bench.py's split of one corpus (4 blocks) over `world` ranks, each
    rank's windows scanned as one launch on this GPU from a buffer holding
    only that rank's bytes: merged records == per-block oracle sequences."""
    lits = bench.make_literals(5000, seed=12)
    blob = vsa.hwlm_build(lits)
    total, bl = (48 << 20) + 4099, 12 << 20
    data = bench.make_corpus(total, lits, seed=5, plant_every=16 << 10)
    cuts, plan = stripe.plan_corpus_stripes(total, bl, world, align=1 << 12)
    db = vsa.Database(ctx, blob)
    got = []
    for r in range(world):
        wins = plan[r]
        g0 = min(w.wlo for w in wins) & ~255
        g1 = cuts[r + 1]
        d = ctx.malloc(g1 - g0 + 64)
        try:
            ctx.h2d(d, data[g0:g1])
            k = ctx.scan_blocks_ex(db, d, [w.wlo - g0 for w in wins], [w.wlen for w in wins],
                                   None, [w.rlo for w in wins])
            res = ctx.results(k)
        finally:
            ctx.free(d)
        got += list(zip(((res["key"] >> np.uint64(24)) + np.uint64(g0)).tolist(),
                        res["id"].tolist()))
    db.close()
    want = []
    for b in range(0, total, bl):
        _, m = oracle.fdr_exec(vsa.engine_blob(blob), data[b:b + bl], cap=1 << 20)
        want += [(e + b, i) for e, i in m]
    assert got == want
    assert len(want) >= total // (16 << 10)


def test_gpu_report_lo_keeps_start_state(ctx):
    """report_lo cuts reported ends without moving the FDR start state:
    a block scanned with report_lo = k reports exactly the block scan's ends
    >= k; scanned with start = k instead, short-literal buckets drop the
    literals that begin before k (fdr->start, fdr_compile.cpp:129-151)."""
    lits = [vsa.HwlmLiteral(s, False, i) for i, s in enumerate(
        [b"abcdefgh", b"cdefgh", b"efgh", b"gh", b"xyzw", b"zw"])]
    blob = vsa.hwlm_build(lits, engine_hint=0)
    data = np.frombuffer(b"..abcdefgh..xyzw.." * 4000, np.uint8)
    _, full = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 20)
    db = vsa.Database(ctx, blob)
    d = ctx.malloc(len(data) + 64)
    try:
        ctx.h2d(d, data)
        for k in (0, 1, 5, 9, 10, 11, 17, 1000, 40001):
            n = ctx.scan_blocks_ex(db, d, [0], [len(data)], None, [k])
            res = ctx.results(n)
            got = list(zip((res["key"] >> np.uint64(24)).tolist(), res["id"].tolist()))
            assert got == [(e, i) for e, i in full if e >= k], k
    finally:
        ctx.free(d)
        db.close()


@pytest.mark.parametrize("nlits", [20000, 50000])
def test_gpu_large_literal_sets(ctx, nlits, monkeypatch):
    """Large FDR sets, where the confirm stage is the bound: the first launch
    (>= 16 MiB) measures the confirm-candidate rate and the next ones run
    with the scanning waves expanding the candidates (scanner expansion,
    runtime.hip use_xp) and the confirm-wave count the rate asks for; one
    launch also forces a single confirm wave and one three (VSA_NCONF); the
    last two launches force expansion off and on (VSA_XP).  The
    database is loaded with the split passes at their default (on for 50k,
    runtime.hip split_passes) and forced off and on (VSA_SPLIT).  Every
    launch == the oracle."""
    lits = bench.make_literals(nlits, seed=12)
    blob = vsa.hwlm_build(lits)
    data = bench.make_corpus(24 << 20, lits, seed=5, plant_every=16 << 10)
    st, want = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 23)
    assert st == 0 and len(want) >= len(data) // (16 << 10)
    n = len(data)
    d = ctx.malloc(n + 64)
    try:
        ctx.h2d(d, data)
        for split in (None, "0", "1"):
            if split:
                monkeypatch.setenv("VSA_SPLIT", split)
            db = vsa.Database(ctx, blob)
            try:
                runs = (((None, None), (None, None), ("1", None), ("3", None), ("2", "0"),
                         ("2", "1")) if split is None else ((None, None), ("2", "1")))
                for nconf, xp in runs:
                    if nconf:
                        monkeypatch.setenv("VSA_NCONF", nconf)
                    if xp:
                        monkeypatch.setenv("VSA_XP", xp)
                    k = ctx.scan_blocks(db, d, [0], [n])
                    res = ctx.results(k)
                    got = list(zip((res["key"] >> np.uint64(24)).tolist(),
                                   res["id"].tolist()))
                    assert got == want, (split, nconf, xp)
            finally:
                monkeypatch.delenv("VSA_NCONF", raising=False)
                monkeypatch.delenv("VSA_XP", raising=False)
                db.close()
    finally:
        monkeypatch.delenv("VSA_SPLIT", raising=False)
        ctx.free(d)


def big_corpus(n, lits, seed, plant_every):
    """a printable corpus with `lits` planted every `plant_every` bytes,
    generated in 64 MiB pieces (uint8 draws: no 8-byte index array of the
    whole size) and planted as bench.plant_plan does"""
    r = np.random.default_rng(seed)
    data = np.empty(n, np.uint8)
    for o in range(0, n, 64 << 20):
        m = min(64 << 20, n - o)
        data[o:o + m] = r.integers(0x20, 0x7F, m, dtype=np.uint8)
    idx, val = bench.plant_plan(n, lits, seed, plant_every)
    data[idx] = val
    return data


def test_gpu_full_size_cfg1_cfg3(ctx):
    """cfg 1 and cfg 3 at their BASELINE size (1 GiB, the size the bench
    lines are quoted at), order-exact against the oracle's callback sequence
    (oracle.records_mt over 16 host stripes with a 7-byte halo): cfg 1 noodle
    'abcde' caseful and nocase on one corpus (planted every 4 KiB, seed 1),
    cfg 3 on the 48-literal set (default Fat Teddy engine 8 and the SSE
    build's 8-bucket engine 18) and the 64-literal set (engine 8), one corpus
    per set (planted every 4 KiB, seed 3)."""
    n = 1 << 30
    cases = [(1, [vsa.HwlmLiteral(b"abcde", False, 0)], [(-1, None)]),
             (1, [vsa.HwlmLiteral(b"abcde", True, 0)], [(-1, None)]),
             (3, cfg3_lits(48), [(-1, 8), (18, 18)]),
             (3, cfg3_lits(64), [(-1, 8)])]
    d = ctx.malloc(n + 64)
    try:
        cur = None
        for seed, lits, engines in cases:
            if cur != (seed, lits[0].s):
                cur = (seed, lits[0].s)
                host = big_corpus(n, lits, seed, 4096)
                ctx.h2d(d, host)
            for hint, engine in engines:
                blob = vsa.hwlm_build(lits, engine_hint=hint)
                if engine is not None:
                    assert blob.engine_id == engine
                db = vsa.Database(ctx, blob)
                try:
                    k = ctx.scan_blocks(db, d, [0], [n])
                    res = ctx.results(k)
                finally:
                    db.close()
                want_e, want_i = oracle.records_mt(vsa.engine_blob(blob), host, 16,
                                                   nood=blob.is_noodle)
                assert len(want_e) >= n // 4096, (seed, hint)
                assert k == len(want_e), (seed, hint, k, len(want_e))
                assert np.array_equal(res["key"] >> np.uint64(24), want_e), (seed, hint)
                assert np.array_equal(res["id"], want_i), (seed, hint)
    finally:
        ctx.free(d)
