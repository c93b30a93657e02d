"""Pure-literal database API: vsa_hs_compile_lit_multi /
vsa_hs_scan / vsa_hs_scan_vector / streams through the C ABI
(include/vectorscan_amd_hs.h, via vectorscan_amd.hs) against the oracle's
restatement of the reference's pure-literal runtime (oracle/hs_lit.py:
runtime.c:204-230 pureLiteralBlockExec, :802-831 pureLiteralStreamExec, on
the oracle.c HWLM scan) — exact callback sequences — and against the
engine-free brute force (match sets).  The grid of the reference's
unit/hyperscan/literals.cpp (modes x {0, SINGLEMATCH, SOM_LEFTMOST} x sizes
x length bounds x caseful / caseless / mixed, each literal scanned alone
must match) is restated at the end."""
import random

import numpy as np
import pytest

import oracle
from oracle import hs_lit as ohs
import vectorscan_amd as vsa
from vectorscan_amd import hs


def rand_patterns(rng, n, lo, hi, alphabet=b"abcd", flag_mix=(0,)):
    exprs, flags = [], []
    for _ in range(n):
        ln = rng.randint(lo, hi)
        exprs.append(bytes(rng.choice(alphabet) for _ in range(ln)))
        flags.append(rng.choice(flag_mix))
    return exprs, flags


def corpus(rng, n, exprs, alphabet=b"abcd", plants=20, runs=True):
    a = np.frombuffer(bytes(rng.choice(alphabet) for _ in range(n)), np.uint8).copy()
    for _ in range(plants):
        e = rng.choice(exprs)
        if len(e) < n:
            p = rng.randrange(0, n - len(e))
            a[p:p + len(e)] = np.frombuffer(e, np.uint8)
    if runs and n > 600:
        for _ in range(3):  # byte runs: the flood shortcut fires on them
            p = rng.randrange(0, n - 300)
            a[p:p + rng.randint(64, 300)] = rng.choice(alphabet)
    return a


def normalize(flags, ids):
    """SINGLEMATCH agrees per id (a compile error otherwise) and, where an id
    has several patterns, so does SOM_LEFTMOST: which of two same-offset
    reports of one id survives dedupe is the first delivered, and with mixed
    SOM the reference's separate SOM dedupe (DEDUPE_SOM) is not restated."""
    single, som = {}, {}
    out = []
    for i, f in enumerate(flags):
        s = single.setdefault(ids[i], bool(f & hs.FLAG_SINGLEMATCH))
        f = (f | hs.FLAG_SINGLEMATCH) if s else (f & ~hs.FLAG_SINGLEMATCH)
        if s:
            f &= ~hs.FLAG_SOM_LEFTMOST
        m = som.setdefault(ids[i], bool(f & hs.FLAG_SOM_LEFTMOST))
        f = (f | hs.FLAG_SOM_LEFTMOST) if m else (f & ~hs.FLAG_SOM_LEFTMOST)
        out.append(f)
    return out


def build_pair(exprs, flags, ids=None, mode=hs.MODE_BLOCK):
    db = hs.compile_lit_multi(exprs, flags, ids, mode)
    odb = ohs.compile_lit_multi(exprs, flags, ids)
    return db, odb


def oracle_blob(odb):
    lits = [vsa.HwlmLiteral(t, nc, f, noruns=nr) for t, nc, f, nr in odb.hwlm_literals()]
    return vsa.hwlm_build(lits)


# ------------------------------------------------------------------ CPU ---

COMPILE_ERRORS = [
    # (exprs, flags, ids, mode, message prefix, expression index)
    ([b"abc"], [hs.FLAG_DOTALL], None, hs.MODE_BLOCK, "Only HS_FLAG_CASELESS", 0),
    ([b"abc", b"d"], [0, hs.FLAG_MULTILINE], None, hs.MODE_BLOCK, "Only HS_FLAG_CASELESS", 1),
    ([b"abc"], [hs.FLAG_SINGLEMATCH | hs.FLAG_SOM_LEFTMOST], None, hs.MODE_BLOCK,
     "HS_FLAG_SINGLEMATCH is not supported in combination", 0),
    ([b""], [0], None, hs.MODE_BLOCK, "Pure literal API doesn't support empty string.", 0),
    ([b"\0ab"], [0], None, hs.MODE_BLOCK, "Pure literal API doesn't support empty string.", 0),
    ([b"abc"], [1 << 12], None, hs.MODE_BLOCK, "Unrecognised flag.", 0),
    ([b"a" * 16001], [0], None, hs.MODE_BLOCK, "Pattern length exceeds limit.", 0),
    ([b"abc"], [0], None, hs.MODE_BLOCK | hs.MODE_STREAM, "Invalid parameter: mode must", -1),
    ([b"abc"], [0], None, 0, "Invalid parameter: mode must", -1),
    ([b"abc"], [0], None, 1 << 8, "Invalid parameter: unrecognised mode flags.", -1),
    ([b"abc"], [0], None, hs.MODE_BLOCK | hs.MODE_SOM_HORIZON_LARGE,
     "Invalid parameter: the HS_MODE_SOM_HORIZON_", -1),
    ([b"abc"], [0], None,
     hs.MODE_STREAM | hs.MODE_SOM_HORIZON_LARGE | hs.MODE_SOM_HORIZON_SMALL,
     "Invalid parameter: only one HS_MODE_SOM_HORIZON_", -1),
    ([], None, None, hs.MODE_BLOCK, "Invalid parameter: elements is zero", -1),
    ([b"abc", b"abd"], [hs.FLAG_SINGLEMATCH, 0], [7, 7], hs.MODE_BLOCK,
     "Expression (index 1) with match ID 7 did not specify HS_FLAG_SINGLEMATCH whereas "
     "previous expression (index 0) with the same match ID did.", 1),
]


@pytest.mark.parametrize("case", range(len(COMPILE_ERRORS)))
def test_compile_errors(case):
    exprs, flags, ids, mode, msg, idx = COMPILE_ERRORS[case]
    with pytest.raises(hs.HsError) as ei:
        hs.compile_lit_multi(exprs, flags, ids, mode)
    assert ei.value.code == hs.COMPILER_ERROR
    assert ei.value.message.startswith(msg), ei.value.message
    assert ei.value.expression == idx
    if idx >= 0 and mode == hs.MODE_BLOCK:
        with pytest.raises(ohs.CompileError) as oe:
            ohs.compile_lit_multi(exprs, flags, ids)
        assert oe.value.expression == idx


@pytest.mark.parametrize("seed", range(6))
def test_fragments_match_oracle(seed):
    """The database's HWLM blob is the one built from the oracle's fragment
    list (tails, case, ids, no-runs) — so both runs scan the same literals."""
    rng = random.Random(seed)
    n = [1, 5, 40, 300, 2000, 60][seed]
    exprs, flags = rand_patterns(rng, n, 1, 20, b"abcdAB",
                                 (0, hs.FLAG_CASELESS, hs.FLAG_SINGLEMATCH,
                                  hs.FLAG_SOM_LEFTMOST, hs.FLAG_CASELESS | hs.FLAG_SINGLEMATCH))
    ids = [rng.randrange(0, max(1, n // 2)) for _ in range(n)]
    flags = normalize(flags, ids)
    db, odb = build_pair(exprs, flags, ids)
    _, _, nfrag = db.hwlm()
    assert nfrag == len(odb.frags)
    assert db.hwlm_bytes() == oracle_blob(odb).tobytes()


@pytest.mark.parametrize("seed", range(8))
def test_oracle_equals_brute_force(seed):
    """The oracle's pure-literal run (HWLM + report program) gives exactly
    the brute-force match set, in increasing `to`."""
    rng = random.Random(100 + seed)
    n = [1, 3, 30, 200, 12, 70, 500, 8][seed]
    exprs, flags = rand_patterns(rng, n, 1, 14, b"abcd",
                                 (0, hs.FLAG_CASELESS, hs.FLAG_SINGLEMATCH,
                                  hs.FLAG_SOM_LEFTMOST))
    ids = list(range(n)) if seed % 2 else [rng.randrange(0, n) for _ in range(n)]
    flags = normalize(flags, ids)
    odb = ohs.compile_lit_multi(exprs, flags, ids)
    blob = oracle_blob(odb)
    data = corpus(rng, 3000, exprs, b"abcdABCD")
    got = ohs.scan(odb, blob.ptr, data)
    want = ohs.brute_force(odb, data)
    assert [g[2] for g in got] == sorted(g[2] for g in got)
    assert sorted(got) == sorted(want)
    # split into writes: the same match set
    cuts = sorted(rng.sample(range(1, len(data)), 5))
    parts = np.split(data, cuts)
    assert sorted(ohs.scan_writes(odb, blob.ptr, parts)) == sorted(want)


def test_symbols_exported():
    """every function include/vectorscan_amd_hs.h declares is exported (its
    static inline helpers excepted)"""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "vectorscan_amd_hs.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    inline = set(re.findall(r"static\s+inline\s+\w+\s+(\w+)\s*\(", hdr))
    hdr = re.sub(r"static\s+inline[^{]*\{.*?\n\}", "", hdr, flags=re.S)
    hdr = "\n".join(l for l in hdr.splitlines()
                    if not l.lstrip().startswith(("#", "typedef")))
    names = {n for n in re.findall(r"\b(vsa_hs_\w+)\s*\(", hdr)} - inline
    assert {"vsa_hs_scan", "vsa_hs_corpus_scan_ex", "vsa_hs_database_hwlm"} <= names
    missing = [n for n in sorted(names) if not hasattr(vsa.lib, n)]
    assert not missing, missing


def test_runtime_argument_errors_cpu():
    """Checks that fail before any GPU work (runtime.c:316-336, 1113-1129)."""
    db = hs.compile_lit_multi([b"abc"], [0], [1], hs.MODE_BLOCK)
    vdb = hs.compile_lit_multi([b"abc"], [0], [1], hs.MODE_VECTORED)
    assert hs.scan(db, b"xxabc", None)[0] == hs.INVALID  # NULL scratch
    assert hs.scan_vector(vdb, [b"abc"], None)[0] == hs.INVALID
    with pytest.raises(hs.HsError) as ei:
        hs.Stream(db)  # block database
    assert ei.value.code == hs.DB_MODE_ERROR


# ------------------------------------------------------------------ GPU ---

def gpu_scan(db, scratch, data, stop_after=None):
    seq = []

    def cb(i, f, t, fl):
        seq.append((i, f, t))
        return stop_after is not None and len(seq) >= stop_after
    rc, _ = hs.scan(db, data, scratch, cb)
    return rc, seq


SETS = [
    # (n patterns, len lo, len hi, alphabet, flag mix, dup ids)
    (1, 3, 6, b"abcd", (0,), False),              # noodle
    (1, 12, 20, b"abcd", (0,), False),            # noodle tail + long check
    (20, 2, 8, b"abcd", (0, hs.FLAG_CASELESS), False),      # Teddy
    (48, 1, 8, b"abcdef", (0, hs.FLAG_SOM_LEFTMOST), True),
    (300, 3, 12, b"abcdefgh", (0, hs.FLAG_CASELESS, hs.FLAG_SINGLEMATCH), False),  # FDR
    (2000, 4, 30, b"abcdefghij", (0, hs.FLAG_CASELESS, hs.FLAG_SOM_LEFTMOST), True),
]


def make_set(k, seed=0):
    n, lo, hi, alpha, mix, dup = SETS[k]
    rng = random.Random(1000 * k + seed)
    exprs, flags = rand_patterns(rng, n, lo, hi, alpha, mix)
    ids = [rng.randrange(0, max(1, n // 3)) for _ in range(n)] if dup else list(range(n))
    flags = normalize(flags, ids)
    return rng, exprs, flags, ids, alpha


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(SETS)))
def test_hs_scan_block(k):
    rng, exprs, flags, ids, alpha = make_set(k)
    db, odb = build_pair(exprs, flags, ids)
    blob = oracle_blob(odb)
    scratch = hs.Scratch(db)
    for size in [0, 1, 7, 100, 5000, 70000]:
        data = corpus(rng, size, exprs, alpha + alpha.upper(), plants=max(1, size // 200))
        rc, seq = gpu_scan(db, scratch, data)
        assert rc == hs.SUCCESS
        assert seq == ohs.scan(odb, blob.ptr, data), size
        assert sorted(seq) == sorted(ohs.brute_force(odb, data))


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 4, 5])
def test_hs_scan_terminate(k):
    rng, exprs, flags, ids, alpha = make_set(k, 1)
    db, odb = build_pair(exprs, flags, ids)
    blob = oracle_blob(odb)
    scratch = hs.Scratch(db)
    data = corpus(rng, 20000, exprs, alpha, plants=200)
    full = ohs.scan(odb, blob.ptr, data)
    assert len(full) > 10
    for stop in [1, 2, len(full) // 2, len(full)]:
        rc, seq = gpu_scan(db, scratch, data, stop_after=stop)
        assert rc == hs.SCAN_TERMINATED
        assert seq == full[:stop]


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(SETS)))
def test_hs_scan_vector(k):
    rng, exprs, flags, ids, alpha = make_set(k, 2)
    db, odb = build_pair(exprs, flags, ids, hs.MODE_VECTORED)
    blob = oracle_blob(odb)
    scratch = hs.Scratch(db)
    data = corpus(rng, 40000, exprs, alpha, plants=300)
    for npieces in [1, 2, 7, 40]:
        cuts = sorted(rng.sample(range(0, len(data) + 1), npieces - 1))
        pieces = [np.ascontiguousarray(p) for p in np.split(data, cuts)]
        seq = []
        rc, _ = hs.scan_vector(db, pieces, scratch, lambda i, f, t, fl: seq.append((i, f, t)))
        assert rc == hs.SUCCESS
        assert seq == ohs.scan_writes(odb, blob.ptr, pieces), npieces
        assert sorted(seq) == sorted(ohs.brute_force(odb, data))


@pytest.mark.gpu
def test_hs_scan_vector_null_piece_and_terminate():
    rng, exprs, flags, ids, alpha = make_set(4, 3)
    db, odb = build_pair(exprs, flags, ids, hs.MODE_VECTORED)
    blob = oracle_blob(odb)
    scratch = hs.Scratch(db)
    data = corpus(rng, 9000, exprs, alpha, plants=100)
    pieces = [np.ascontiguousarray(p) for p in np.split(data, [3000, 6000])]
    want = ohs.scan_writes(odb, blob.ptr, pieces[:2])
    seq = []
    rc, _ = hs.scan_vector(db, pieces[:2] + [None, pieces[2]], scratch,
                           lambda i, f, t, fl: seq.append((i, f, t)))
    assert rc == hs.INVALID
    assert seq == want
    full = ohs.scan_writes(odb, blob.ptr, pieces)
    stop = len(full) // 2
    seq = []
    rc, _ = hs.scan_vector(db, pieces, scratch,
                           lambda i, f, t, fl: seq.append((i, f, t)) or len(seq) >= stop)
    assert rc == hs.SCAN_TERMINATED
    assert seq == full[:stop]


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 2, 4, 5])
def test_hs_streams(k):
    rng, exprs, flags, ids, alpha = make_set(k, 4)
    db, odb = build_pair(exprs, flags, ids, hs.MODE_STREAM | hs.MODE_SOM_HORIZON_LARGE)
    blob = oracle_blob(odb)
    scratch = hs.Scratch(db)
    data = corpus(rng, 30000, exprs, alpha, plants=250)
    cuts = sorted(rng.sample(range(0, len(data) + 1), 30))
    writes = [np.ascontiguousarray(p) for p in np.split(data, cuts)]
    st = hs.Stream(db)
    seq = []
    for w in writes:
        rc, _ = st.scan(w, scratch, lambda i, f, t, fl: seq.append((i, f, t)))
        assert rc == hs.SUCCESS
    assert st.close(scratch, lambda *a: 0) == hs.SUCCESS
    assert seq == ohs.scan_writes(odb, blob.ptr, writes)
    # reset: the stream starts over (offset 0, exhaustion cleared)
    st = hs.Stream(db)
    st.scan(writes[0], scratch)
    assert st.reset(scratch, lambda *a: 0) == hs.SUCCESS
    seq2 = []
    for w in writes[:5]:
        st.scan(w, scratch, lambda i, f, t, fl: seq2.append((i, f, t)))
    assert seq2 == ohs.scan_writes(odb, blob.ptr, writes[:5])
    # a terminated stream stays terminated (runtime.c:883-893)
    st = hs.Stream(db)
    rc, _ = st.scan(np.frombuffer(exprs[0], np.uint8).copy(), scratch, lambda *a: 1)
    assert rc == hs.SCAN_TERMINATED
    assert st.scan(exprs[0], scratch)[0] == hs.SCAN_TERMINATED
    st.close()


@pytest.mark.gpu
def test_hs_runtime_errors_gpu():
    db = hs.compile_lit_multi([b"abc", b"bcd"], [0, 0], [1, 2], hs.MODE_BLOCK)
    vdb = hs.compile_lit_multi([b"abc"], [0], [1], hs.MODE_VECTORED)
    other = hs.compile_lit_multi([b"zz"], [0], [3], hs.MODE_BLOCK)
    scratch = hs.Scratch(db)
    assert hs.scan(vdb, b"abc", scratch)[0] == hs.DB_MODE_ERROR
    assert hs.scan_vector(db, [b"abc"], scratch)[0] == hs.DB_MODE_ERROR
    # scratch not allocated for `other` (validScratch)
    assert hs.scan(other, b"zz", scratch)[0] == hs.INVALID
    scratch.grow(other)
    assert hs.scan(other, b"zzz", scratch)[1] == [(3, 0, 2), (3, 0, 3)]
    # shorter than the shortest literal: no scan (runtime.c:346-350)
    assert hs.scan(db, b"ab", scratch) == (hs.SUCCESS, [])
    assert hs.scan(db, b"", scratch) == (hs.SUCCESS, [])
    # re-entrant use from a callback: HS_SCRATCH_IN_USE
    inner = []

    def cb(i, f, t, fl):
        inner.append(hs.scan(db, b"abcd", scratch)[0])
        return 0
    assert hs.scan(db, b"xabcd", scratch, cb)[0] == hs.SUCCESS
    assert inner == [hs.SCRATCH_IN_USE, hs.SCRATCH_IN_USE]
    assert hs.scan(db, b"abcd", scratch)[1] == [(1, 0, 3), (2, 0, 4)]


@pytest.mark.gpu
def test_hs_flood_runs():
    """Long runs of one byte: the flood shortcut's reports (flood_runtime.h)
    and the report program over them, equal to the oracle and the brute
    force."""
    exprs = [b"a", b"aa", b"aaaa", b"aaaaaaaaaaaa", b"ab", b"ba", b"b" * 9]
    flags = [0, hs.FLAG_SOM_LEFTMOST, hs.FLAG_SINGLEMATCH, 0, hs.FLAG_CASELESS, 0, 0]
    for mode in [hs.MODE_BLOCK, hs.MODE_VECTORED]:
        db, odb = build_pair(exprs, flags, list(range(len(exprs))), mode)
        blob = oracle_blob(odb)
        scratch = hs.Scratch(db)
        data = np.frombuffer(b"x" * 40 + b"a" * 3000 + b"b" * 700 + b"aB" * 50 + b"c" * 500,
                             np.uint8).copy()
        if mode == hs.MODE_BLOCK:
            seq = gpu_scan(db, scratch, data)[1]
            assert seq == ohs.scan(odb, blob.ptr, data)
        else:
            pieces = [np.ascontiguousarray(p) for p in np.split(data, [1000, 1001, 3500])]
            seq = []
            hs.scan_vector(db, pieces, scratch, lambda i, f, t, fl: seq.append((i, f, t)))
            assert seq == ohs.scan_writes(odb, blob.ptr, pieces)
        assert sorted(seq) == sorted(ohs.brute_force(odb, data))


# unit/hyperscan/literals.cpp grid (the NDEBUG sizes up to 10000); each
# literal's own text, scanned alone, reports that literal at to = len.
LIT_GRID = [(m, f, n, b) for m in (hs.MODE_BLOCK, hs.MODE_STREAM, hs.MODE_VECTORED)
            for f in (0, hs.FLAG_SINGLEMATCH, hs.FLAG_SOM_LEFTMOST)
            for n in (1, 10, 100, 500, 10000) for b in ((3, 10), (10, 100))]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["caseful", "caseless", "mixed"])
def test_reference_literal_grid(case):
    for mode, all_flags, num, (lo, hi) in LIT_GRID:
        if num == 10000 and (mode != hs.MODE_BLOCK or all_flags):
            continue  # the big size once per case keeps the run short
        rng = random.Random(29785643 + num + lo)
        exprs, flags = [], []
        for i in range(num):
            ln = rng.randint(lo, hi)
            exprs.append(bytes(rng.randint(97, 122) for _ in range(ln)))
            f = all_flags
            if case == "caseless" or (case == "mixed" and i % 2):
                f |= hs.FLAG_CASELESS
            flags.append(f)
        m = mode | (hs.MODE_SOM_HORIZON_LARGE
                    if mode == hs.MODE_STREAM and all_flags & hs.FLAG_SOM_LEFTMOST else 0)
        db, odb = build_pair(exprs, flags, list(range(num)), m)
        blob = oracle_blob(odb)
        scratch = hs.Scratch(db)
        step = max(1, num // 50)
        for i in range(0, num, step):
            text = np.frombuffer(exprs[i], np.uint8).copy()
            seq = []

            def cb(a, f, t, fl):
                seq.append((a, f, t))
                return 0
            if mode == hs.MODE_BLOCK:
                rc, _ = hs.scan(db, text, scratch, cb)
            elif mode == hs.MODE_VECTORED:
                rc, _ = hs.scan_vector(db, [text], scratch, cb)
            else:
                st = hs.Stream(db)
                rc, _ = st.scan(text, scratch, cb)
                assert st.close(scratch, lambda *a: 0) == hs.SUCCESS
            assert rc == hs.SUCCESS
            assert (i, 0, len(exprs[i])) in seq, (mode, all_flags, num, i)
            assert seq == ohs.scan(odb, blob.ptr, text)


@pytest.mark.gpu
def test_hs_block_limit_is_invalid():
    """one launch takes at most VSA_MAX_BLOCKS blocks (the records carry a
    20-bit block index): an hs_scan_vector call with more non-empty pieces
    is scanned as consecutive launches of one stream (the reference has no
    such limit), empty pieces do not count, and a larger prepared hs corpus
    is refused with HS_INVALID, not a misleading NOMEM / UNKNOWN_ERROR"""
    limit = 1 << 20
    db = hs.compile_lit_multi([b"abcd"], [0], [1], hs.MODE_VECTORED)
    scratch = hs.Scratch(db)
    try:
        one = b"abcd"
        rc, out = hs.scan_vector(db, [one] * (limit + 1), scratch)
        assert rc == hs.SUCCESS and len(out) == limit + 1
        assert out[0] == (1, 0, 4) and out[-1] == (1, 0, 4 * (limit + 1))
        assert all(out[k][2] == 4 * (k + 1) for k in range(0, limit + 1, 4099))
        rc, out = hs.scan_vector(db, [b""] * (limit + 5) + [one], scratch)
        assert rc == hs.SUCCESS and out == [(1, 0, 4)]
        # a match across the launch boundary: "ab" ends the first launch's
        # last piece, "cd" starts the next launch
        rc, out = hs.scan_vector(db, [b"xxxx"] * (limit - 1) + [b"xxab", b"cdxx"], scratch)
        assert rc == hs.SUCCESS and out == [(1, 0, 4 * limit + 2)]
        rc, out = hs.scan_vector(db, [one] * 4, scratch)
        assert rc == hs.SUCCESS and len(out) == 4
    finally:
        scratch.close()
        db.close()
    bdb = hs.compile_lit_multi([b"abcd"], [0], [1], hs.MODE_BLOCK)
    bs = hs.Scratch(bdb)
    ctx = vsa.Context(0)
    d = ctx.malloc(16)
    try:
        n = limit + 1
        with pytest.raises(hs.HsError) as e:
            hs.Corpus(bdb, bs, d, np.zeros(n, np.uint64), np.ones(n, np.uint64))
        assert e.value.code == hs.INVALID
    finally:
        ctx.free(d)
        bs.close()
        bdb.close()
