"""CPU tests: the oracle against the reference's own known answers
(tests/golden, restated from unit/internal/*.cpp), the oracle against a
brute-force matcher on random inputs, and the bytecode builder's layout.

No GPU is touched here: the builder is host code in the library and the
oracle is plain C.
"""
import ctypes
import json
import os
import random

import numpy as np
import pytest

import oracle
import vectorscan_amd as vsa

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FDR_HINTS = [0, 11, 12, 13, 14, 15, 16, 17, 18, 3, 4, 5, 6, 7, 8, 9, 10]


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def lits_of(case):
    return [vsa.HwlmLiteral(bytes.fromhex(l["s"]), l["nocase"], l["id"], noruns=l["noruns"])
            for l in case["lits"]]


def build_or_none(lits, hint):
    try:
        return vsa.hwlm_build(lits, engine_hint=hint)
    except vsa.BuildError:
        return None


# ------------------------------------------------------------- golden ---

def test_golden_noodle_oracle():
    for c in load("noodle.json"):
        blob = vsa.hwlm_build([vsa.HwlmLiteral(bytes.fromhex(c["lit"]), c["nocase"], 1000)])
        assert blob.is_noodle
        st, m = oracle.nood_exec(vsa.engine_blob(blob), bytes.fromhex(c["data"]))
        assert st == 0
        assert [e for e, _ in m] == c["expected"], c["src"]
        assert all(i == 1000 for _, i in m)


@pytest.mark.parametrize("hint", FDR_HINTS)
def test_golden_fdr_oracle(hint):
    ran = 0
    for c in load("fdr.json"):
        blob = build_or_none(lits_of(c), hint)
        if blob is None:
            continue  # CHECK_WITH_TEDDY_OK_TO_FAIL (fdr.cpp:75-84)
        ran += 1
        st, m = oracle.fdr_exec(vsa.engine_blob(blob), bytes.fromhex(c["data"]),
                                start=c["start"], term_after=c["term_after"])
        if c["expected"] is None:
            assert len(m) == c["expected_len"], c["src"]
            assert st == 1
            continue
        assert st == 0
        assert [list(x) for x in m] == c["expected"], (c["src"], hint)
    assert ran > 0


@pytest.mark.parametrize("hint", [0, 11, 17, 3, 9])
def test_golden_short_writings_oracle(hint):
    """fdr.cpp:594-692 on the first alphabet (all alphabets: slow test)."""
    spec = load("fdr_shortwritings.json")[0]
    _short_writings(spec, hint, oracle_run)


def oracle_run(blob, bufs):
    out = []
    for b in bufs:
        st, m = oracle.fdr_exec(vsa.engine_blob(blob), b)
        assert st == 0
        out.append(m)
    return out


def _short_writings(spec, hint, run):
    bufs = [bytes.fromhex(x) for x in spec["bufs"]]
    pats = [bytes.fromhex(x) for x in spec["pats"]]
    for g in range(0, len(pats), 32):
        group = pats[g:g + 32]
        lits = [vsa.HwlmLiteral(p, False, g + i) for i, p in enumerate(group)]
        blob = build_or_none(lits, hint)
        if blob is None:
            continue
        got = run(blob, bufs)
        for b, m in zip(bufs, got):
            exp = sorted((j + len(p) - 1, g + i) for i, p in enumerate(group)
                         for j in range(len(b) - len(p) + 1) if b[j:j + len(p)] == p)
            assert sorted(m) == exp


@pytest.mark.slow
@pytest.mark.parametrize("alpha", [1, 2, 3])
def test_golden_short_writings_oracle_all(alpha):
    spec = load("fdr_shortwritings.json")[alpha]
    for hint in (0, 11, 17, 3):
        _short_writings(spec, hint, oracle_run)


def accel_expected_oracle(c):
    data = bytes.fromhex(c["data"])
    k = c["kind"]
    if k in ("shufti", "rshufti"):
        lo, hi = vsa.shufti_build_masks(c["chars"])
        return oracle.shufti(lo, hi, data, reverse=(k == "rshufti"))
    if k in ("truffle", "rtruffle"):
        m1, m2 = vsa.truffle_build_masks(c["chars"])
        return oracle.truffle(m1, m2, data, reverse=(k == "rtruffle"))
    if k in ("verm", "nverm", "rverm", "rnverm"):
        return oracle.verm(c["c"], c["nocase"], data, negate=k in ("nverm", "rnverm"),
                           reverse=k in ("rverm", "rnverm"))
    if k == "dverm":
        return oracle.dverm(c["c1"], c["c2"], c["nocase"], data)
    if k == "rdverm":
        return oracle.rdverm(c["c1"], c["c2"], c["nocase"], data)
    raise AssertionError(k)


def test_golden_accel_oracle():
    for c in load("accel.json"):
        assert accel_expected_oracle(c) == c["expected"], c["src"]


# -------------------------------------------------- random differential --

def rand_lits(rng, n, minlen=1, maxlen=8, alphabet=b"abcdefgh", nocase_frac=0.2,
              msk_frac=0.0):
    lits = []
    for i in range(n):
        ln = rng.randint(minlen, maxlen)
        s = bytes(rng.choice(alphabet) for _ in range(ln))
        nc = rng.random() < nocase_frac
        msk = cmp = b""
        if rng.random() < msk_frac:
            ml = rng.randint(1, 8)
            m = bytearray(ml)
            v = bytearray(ml)
            # constrain one byte before (or inside) the literal
            k = rng.randrange(ml)
            m[k] = 0xF0
            v[k] = rng.choice(alphabet) & 0xF0
            # keep consistent with s where overlapping
            for q in range(ml):
                si = len(s) - ml + q
                if 0 <= si and m[q]:
                    c = s[si]
                    if nc and (0x41 <= (c & 0xDF) <= 0x5A):
                        c &= 0xDF
                        m[q] &= 0xDF
                    v[q] = c & m[q]
            msk, cmp = bytes(m), bytes(v)
        lits.append(vsa.HwlmLiteral(s, nc, i, msk=msk, cmp=cmp))
    return lits


def rand_data(rng, n, alphabet=b"abcdefghABCDEFGH"):
    return bytes(rng.choice(alphabet) for _ in range(n))


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("nlits", [1, 5, 30, 60, 200])
def test_oracle_vs_bruteforce(seed, nlits):
    rng = random.Random(seed * 1000 + nlits)
    lits = rand_lits(rng, nlits, msk_frac=0.2)
    blob = vsa.hwlm_build(lits)
    for ln in (0, 1, 7, 15, 16, 17, 33, 100, 999):
        data = rand_data(rng, ln)
        for start in sorted({0, 1, min(5, ln), ln // 2}):
            if ln and start >= ln:
                continue
            st, m = oracle.hwlm_exec(blob.ptr, data, start=start)
            got = set(m)
            exp = oracle.brute_force(lits, data)
            if start == 0 or blob.is_noodle:
                if blob.is_noodle:
                    # noodle needs the whole window at or after start
                    w = max(len(lits[0].s), len(lits[0].msk))
                    exp = {(e, i) for e, i in exp if e - w + 1 >= start}
                assert got == exp, (nlits, ln, start)
            else:
                # FDR/Teddy may report literals that begin before `start`
                # (zone semantics, fdr.c:625-659); every report is real and
                # every occurrence fully after start is reported
                assert got <= {(e, i) for e, i in exp if e >= start}
                lens = {l.id: max(len(l.s), len(l.msk)) for l in lits}
                need = {(e, i) for e, i in exp if e - lens[i] + 1 >= start}
                assert need <= got
            # callback order: non-decreasing end
            ends = [e for e, _ in m]
            assert ends == sorted(ends)


# ----------------------------------------------------------- builder ----

def test_builder_engine_choice():
    rng = random.Random(7)
    pr = bytes(range(0x20, 0x7F))
    def lits_n(n, seed):
        r = random.Random(seed)
        return [vsa.HwlmLiteral(bytes(r.choice(pr) for _ in range(r.randint(4, 8))), False, i)
                for i in range(n)]
    assert vsa.hwlm_build(lits_n(1, 1)).is_noodle
    e48 = vsa.hwlm_build(lits_n(48, 55)).engine_id
    assert 11 <= e48 <= 18 or 3 <= e48 <= 10
    e64 = vsa.hwlm_build(lits_n(64, 71)).engine_id
    assert 3 <= e64 <= 10  # fat teddy (16 buckets) on this target
    b5k = vsa.hwlm_build(lits_n(5000, 12))
    assert b5k.engine_id == 0
    raw = b5k.tobytes()
    fdr = raw[vsa.HWLM_HEADER:]
    domain = fdr[25]
    stride = fdr[24]
    assert domain == 13 and stride == 1
    assert int.from_bytes(fdr[26:28], "little") == (1 << domain) - 1
    assert rng  # silence


def test_builder_layout_offsets():
    blob = vsa.hwlm_build([vsa.HwlmLiteral(b"abc", False, 1), vsa.HwlmLiteral(b"xyz", True, 2)],
                          engine_hint=0)
    raw = blob.tobytes()
    assert raw[0] == 12  # HWLM_ENGINE_FDR
    fdr = raw[192:]
    size, = np.frombuffer(fdr[4:8], np.uint32)
    conf_off, flood_off = np.frombuffer(fdr[16:24], np.uint32)
    assert 192 + size == len(raw)
    assert conf_off % 64 == 0 and flood_off % 64 == 0
    assert conf_off == 64 + (1 << 9) * 8  # header, then the domain-9 table


def test_shufti_truffle_masks():
    chars = [1, 0x7F, 0x80, 0xFE, ord("<"), ord(">"), ord('"'), ord("'")]
    lo, hi = vsa.shufti_build_masks(chars)
    member = {c for c in range(256) if lo[c & 15] & hi[c >> 4]}
    assert member == set(chars)
    m1, m2 = vsa.truffle_build_masks(range(0, 256, 3))
    mem = {c for c in range(256) if ((m2 if c & 0x80 else m1)[c & 15] >> ((c >> 4) & 7)) & 1}
    assert mem == set(range(0, 256, 3))
    big = random.Random(5).sample(range(256), 100)
    assert vsa.shufti_build_masks(big) is None  # needs truffle (SURVEY §8d cfg 2)


# ------------------------------------------------------------ C ABI -----

def test_library_exports_header_symbols():
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "vectorscan_amd.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    hdr = "\n".join(l for l in hdr.splitlines()
                    if not l.lstrip().startswith(("#", "typedef")))
    names = set(re.findall(r"\b(\w+)\s*\(", hdr))
    names -= {"if", "while", "sizeof", "defined", "HWLMCallback"}
    assert "hwlmExec" in names and "vsa_scan_blocks" in names
    lib = ctypes.CDLL(vsa.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


@pytest.mark.parametrize("nlits,lo", [(300, 6), (200, 8), (1000, 4)])
def test_oracle_vs_bruteforce_long_literals(nlits, lo):
    """Stride 2 / 4 FDR engines (long literal sets, fdr_compile.cpp
    chooseEngine) against brute force."""
    rng = random.Random(nlits * 31 + lo)
    lits = rand_lits(rng, nlits, minlen=lo, maxlen=8, nocase_frac=0.1)
    blob = vsa.hwlm_build(lits)
    assert blob.engine_id == 0
    for ln in (0, 5, 16, 17, 40, 300, 5000):
        data = rand_data(rng, ln, alphabet=b"abcdefgh")
        for start in sorted({0, 1, 3, ln // 2}):
            if ln and start >= ln:
                continue
            st, m = oracle.hwlm_exec(blob.ptr, data, start=start, cap=1 << 16)
            got = set(m)
            exp = oracle.brute_force(lits, data)
            if start == 0:
                assert got == exp, (nlits, ln)
            else:
                assert got <= {(e, i) for e, i in exp if e >= start}
                lens = {l.id: len(l.s) for l in lits}
                assert {(e, i) for e, i in exp if e - lens[i] + 1 >= start} <= got


# ------------------------------------------------------ double shufti ----

def placed(data, mis, align=64):
    """Copy data to host memory whose address is `mis` mod `align`;
    returns (keepalive, address)."""
    import ctypes
    buf = ctypes.create_string_buffer(len(data) + 2 * align)
    addr = ctypes.addressof(buf)
    addr += (mis - addr) % align
    ctypes.memmove(addr, bytes(data), len(data))
    return buf, addr


def dshufti_expect_ok(c, r, base_mis):
    """r = result index relative to the scanned buffer t[start:end]."""
    base = 4096 + base_mis
    rv = base + c["start"] + r
    if c["kind"] == "eq":
        return rv == base + c["value"]
    if c["kind"] == "ge":
        return rv >= base + c["value"]
    assert c["kind"] == "ge_end16"
    return rv >= (base + c["end"]) & ~15


def dshufti_masks(c):
    return vsa.shufti_build_double_masks([tuple(p) for p in c["pairs"]], bytes(c["onechar"]))


def test_golden_dshufti_build():
    spec = load("dshufti.json")
    for c in spec["build"]:
        m = dshufti_masks(c)
        assert (m is not None) == c["ok"], c["src"]
        if m is None:
            continue
        lo1, hi1, lo2, hi2 = m
        if c["exact"]:
            assert list(lo1) == c["exact"]["lo1"] and list(hi1) == c["exact"]["hi1"]
            assert list(lo2) == c["exact"]["lo2"] and list(hi2) == c["exact"]["hi2"]
        for a, b, rel in c["checks"]:
            v = lo1[a % 16] | hi1[a >> 4] | lo2[b % 16] | hi2[b >> 4]
            assert (v != 0xFF) if rel == "ne" else (v == 0xFF), (c["src"], chr(a), chr(b))


@pytest.mark.parametrize("vsize", [16, 32, 64])
def test_golden_dshufti_oracle(vsize):
    """shufti.cpp:482-890 known answers hold for the restated
    shuftiDoubleExec at every alignment of the test array."""
    spec = load("dshufti.json")
    for c in spec["exec"]:
        m = dshufti_masks(c)
        data = bytes.fromhex(c["data"])[c["start"]:c["end"]]
        for base_mis in (0, 1, 5, 8, 15, 16, 33, 63):
            mis = (base_mis + c["start"]) % vsize
            r = oracle.shufti_double(*m, data, vector_size=vsize, mis=mis)
            assert dshufti_expect_ok(c, r, base_mis), (c["src"], vsize, base_mis, r)


# ---------------------------------------------------------- streaming ----

def stream_lits(c):
    return [vsa.HwlmLiteral(bytes.fromhex(l["s"]), l["nocase"], l["id"], noruns=l["noruns"])
            for l in c["lits"]]


@pytest.mark.parametrize("hint", FDR_HINTS)
def test_golden_fdr_stream_oracle(hint):
    """fdr.cpp SmallStreaming / SmallStreaming2 / Stream1 / FDRTermS."""
    for c in load("fdr_stream.json"):
        lits = stream_lits(c)
        blob = build_or_none(lits, hint) if c["hinted"] else vsa.hwlm_build(lits)
        if blob is None or blob.is_noodle:
            continue
        st, m = oracle.fdr_exec_stream(vsa.engine_blob(blob), bytes.fromhex(c["hist"]),
                                       bytes.fromhex(c["data"]), start=c["start"],
                                       term_after=c["term_after"])
        assert st == c["status"], c["src"]
        if c["expected"] is not None:
            assert m == [tuple(x) for x in c["expected"]], (c["src"], hint)
        if "expected_len" in c:
            assert len(m) == c["expected_len"], c["src"]


def stream_expected(lits, hist, data, start):
    """Streaming semantics (fdr.c:827 with len_history > 0): every
    occurrence in hist + data ending at or after `start` (relative to data)
    whose overhang into the history is at most len(hist)."""
    h = len(hist)
    occ = oracle.brute_force(lits, bytes(hist) + bytes(data))
    return {(e - h, i) for e, i in occ if e - h >= start}


@pytest.mark.parametrize("seed", range(8))
def test_oracle_stream_semantics(seed):
    rng = random.Random(4242 + seed)
    for nl in (1, 3, 30, 200, 800):
        lits = rand_lits(rng, nl, minlen=1, maxlen=8, msk_frac=0.0)
        for l in lits:
            l.noruns = False
        blob = vsa.hwlm_build(lits)
        for trial in range(6):
            hist = rand_data(rng, rng.choice([1, 2, 5, 8, 15, 16, 17, 40]))
            data = rand_data(rng, rng.choice([1, 3, 9, 16, 17, 31, 100, 700]))
            start = rng.choice([0, 0, 1, 3, len(data) // 2])
            if start >= len(data):
                start = 0
            st, m = oracle.hwlm_exec_stream(blob.ptr, hist, data, start=start, cap=1 << 16)
            got = set(m)
            if blob.is_noodle and start:
                # hwlmExecStreaming falls back to a block scan from start
                w = max(len(lits[0].s), len(lits[0].msk))
                exp = {(e, i) for e, i in oracle.brute_force(lits, data) if e - w + 1 >= start}
            else:
                exp = stream_expected(lits, hist, data, start)
            assert got == exp, (seed, nl, trial, len(hist), len(data), start)
            ends = [e for e, _ in m]
            assert ends == sorted(ends)


def test_oracle_accel_correct_schemes_keep_matches():
    """An accel scheme whose stop condition every match satisfies (the
    literal's byte at `offset` from its start) never changes the match set
    (hwlm.c:85-105 block, 114-175 streaming)."""
    rng = random.Random(77)
    for trial in range(20):
        s = rand_data(rng, rng.randint(2, 5), b"abcdefgh")
        lits = [vsa.HwlmLiteral(s + t, False, i)
                for i, t in enumerate([b"", b"a", b"bb", b"cde"][:rng.randint(2, 4)])]
        blob = vsa.hwlm_build(lits)
        if blob.is_noodle:
            continue
        k = rng.randrange(len(s))
        kind = rng.choice(["verm", "shufti", "truffle"] + (["dverm"] if k + 1 < len(s) else []))
        if kind == "verm":
            aux = vsa.accel_aux("verm", k, s[k])
        elif kind == "dverm":
            aux = vsa.accel_aux("dverm", k, s[k], s[k + 1])
        elif kind == "shufti":
            aux = vsa.accel_aux("shufti", k, masks=vsa.shufti_build_masks(bytes([s[k]])))
        else:
            aux = vsa.accel_aux("truffle", k, masks=vsa.truffle_build_masks(bytes([s[k]])))
        blob.set_accel(aux)
        data = rand_data(rng, rng.choice([20, 100, 3000]), b"abcdefgh")
        st, m = oracle.hwlm_exec(blob.ptr, data, cap=1 << 16)
        assert set(m) == oracle.brute_force(lits, data), (trial, kind)
        hist = rand_data(rng, rng.choice([0, 3, 30]), b"abcdefgh")
        st, m = oracle.hwlm_exec_stream(blob.ptr, hist, data, cap=1 << 16)
        assert set(m) == stream_expected(lits, hist, data, 0), (trial, kind, len(hist))


# ------------------------------------------------- derived first stages ---

def _first_stage_candidates(table, key_bits, field_bits, data):
    """numpy restatement of the kernels' first stage: candidate ends (any
    bucket) from the derived table; positions before the buffer pass."""
    b = np.frombuffer(bytes(data), np.uint8).astype(np.uint64)
    n = len(b)
    assert key_bits == 8  # Teddy / Fat Teddy: the byte itself
    x = table[b.astype(np.int64)]
    nfields = 64 // field_bits
    fmask = np.uint64((1 << field_bits) - 1)
    conf = np.zeros(n, np.uint64)
    for k in range(nfields):
        f = (x >> np.uint64(field_bits * k)) & fmask
        conf[k:] |= f[:n - k]
    return np.nonzero((~conf) & fmask)[0]


@pytest.mark.parametrize("nlits,hint,minlen", [(40, 11, 1), (40, 17, 4), (60, 3, 1),
                                                (60, 8, 4)])
def test_derived_first_stage_no_false_negatives(nlits, hint, minlen):
    """The first stage the engine derives from the confirm records (Teddy /
    Fat Teddy exact byte tables; FDR: the next test)
    passes every end the reference's confirm accepts, and (literals of 4+
    bytes) stays selective."""
    import bench
    rng = random.Random(900 + nlits + hint + minlen)
    lits = [vsa.HwlmLiteral(bytes(rng.randint(0x20, 0x7E)
                                  for _ in range(rng.randint(minlen, 8))),
                            rng.random() < 0.1, i) for i in range(nlits)]
    blob = build_or_none(lits, hint)
    if blob is None:
        pytest.skip("engine not buildable for this set")
    table, kb, fb = vsa.derive_first_stage(blob)
    data = bench.make_corpus(1 << 20, lits, seed=nlits + hint, plant_every=512)
    st, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 20)
    assert st == 0 and len(m) > 1000
    cand = set(_first_stage_candidates(table, kb, fb, data).tolist())
    missing = [e for e, _ in m if e not in cand]
    assert not missing, missing[:10]
    if minlen >= 4:
        assert len(cand) < 0.05 * len(data), len(cand)


def _fdr4_candidates(table, data):
    """numpy restatement of the FDR4 first stage (kernels.hip fdr4_conf):
    key of position p = vsa_fdr4_key (kernels.h): b[p-1] & 0x7f, bit 0 of
    b[p-2] at bit 7, b[p] & 0x7f at bits 8..14; field f of T[key] on end
    p + f; bytes before the buffer are 0."""
    b = np.frombuffer(bytes(data), np.uint8).astype(np.uint64)
    n = len(b)
    p1 = np.concatenate([np.zeros(1, np.uint64), b[:-1]])
    p2 = np.concatenate([np.zeros(2, np.uint64), b[:-2]])
    key = ((p1 & np.uint64(0x7F)) | ((p2 & np.uint64(1)) << np.uint64(7)) |
           ((b & np.uint64(0x7F)) << np.uint64(8)))
    x = table[key.astype(np.int64)].astype(np.uint64)
    conf = np.zeros(n, np.uint64)
    for f in range(4):
        conf[f:] |= (x[:n - f] >> np.uint64(8 * f)) & np.uint64(0xFF)
    return np.nonzero((~conf) & np.uint64(0xFF))[0]


@pytest.mark.parametrize("nlits,minlen", [(2000, 1), (2000, 4), (300, 2), (5000, 4)])
def test_fdr4_first_stage_no_false_negatives(nlits, minlen):
    """The 4-field FDR first stage (derive_fdr4_table, the scan table of
    every FDR engine) passes every end the reference's confirm accepts, and
    (literals of 4+ bytes) stays selective: at most 0.3 % of the ends of a
    printable corpus with a literal planted every 512 bytes."""
    import bench
    rng = random.Random(700 + nlits + minlen)
    lits = [vsa.HwlmLiteral(bytes(rng.randint(0x20, 0x7E)
                                  for _ in range(rng.randint(minlen, 8))),
                            rng.random() < 0.1, i) for i in range(nlits)]
    blob = build_or_none(lits, 0)
    if blob is None:
        pytest.skip("FDR not buildable for this set")
    table = vsa.derive_fdr4_table(blob, 15)
    data = bench.make_corpus(1 << 20, lits, seed=nlits + 15, plant_every=512)
    st, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 20)
    assert st == 0 and len(m) > 1000
    cand = set(_fdr4_candidates(table, data).tolist())
    missing = [e for e, _ in m if e not in cand]
    assert not missing, missing[:10]
    if minlen >= 4:
        assert len(cand) < 0.003 * len(data), len(cand)


@pytest.mark.parametrize("nlits,minlen,msk", [(2000, 1, 0.0), (3000, 4, 0.0), (800, 2, 0.3)])
def test_fdr4_split_passes_no_false_negatives(nlits, minlen, msk):
    """Split passes (runtime.hip, large sets): pass `par` keeps the ends
    whose byte has bit 0 == par and scans them with the table of the
    literals whose last byte can have that bit (vsa_derive_fdr4_pass).
    Every end the reference's confirm accepts is a candidate of exactly the
    pass its byte belongs to, and each pass table is at least as selective
    on its ends as the one-pass table."""
    import bench
    rng = random.Random(910 + nlits + minlen)
    lits = (rand_lits(rng, nlits, minlen=minlen, maxlen=8, msk_frac=msk) if msk else
            [vsa.HwlmLiteral(bytes(rng.randint(0x20, 0x7E) for _ in range(rng.randint(minlen, 8))),
                             rng.random() < 0.1, i) for i in range(nlits)])
    blob = build_or_none(lits, 0)
    if blob is None or blob.is_noodle or blob.engine_id != 0:
        pytest.skip("FDR not buildable for this set")
    data = (bench.make_corpus(1 << 20, lits, seed=nlits, plant_every=512) if not msk else
            np.frombuffer(rand_data(rng, 1 << 20, alphabet=bytes(range(0x61, 0x6b))), np.uint8))
    st, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 21)
    assert st == 0 and len(m) > 100
    full, _ = vsa.derive_fdr4_pass(blob, -1)
    assert np.array_equal(full, vsa.derive_fdr4_table(blob, 15))
    b = np.frombuffer(bytes(data), np.uint8)
    ends = np.array(sorted({e for e, _ in m}), np.int64)
    one = set(_fdr4_candidates(full, data).tolist())
    for par in (0, 1):
        t, _ = vsa.derive_fdr4_pass(blob, par)
        c = _fdr4_candidates(t, data)
        c = c[(b[c] & 1) == par]
        mine = ends[(b[ends] & 1) == par]
        assert set(mine.tolist()) <= set(c.tolist()), par
        assert set(c.tolist()) <= one


def test_fdr4_split_rule():
    """The split rule (runtime.hip split_passes: estimated text rate of the
    one-pass table > 0.015, the measured crossover): one pass for the
    20k-literal cfg-4 set, split passes for 30k and 50k, whose pass tables
    estimate well under the one-pass rate."""
    import bench
    r20 = vsa.derive_fdr4_pass(vsa.hwlm_build(bench.make_literals(20000, seed=12)), -1)[1]
    b50 = vsa.hwlm_build(bench.make_literals(50000, seed=12))
    r30 = vsa.derive_fdr4_pass(vsa.hwlm_build(bench.make_literals(30000, seed=12)), -1)[1]
    r50 = vsa.derive_fdr4_pass(b50, -1)[1]
    p0, p1 = (vsa.derive_fdr4_pass(b50, p)[1] for p in (0, 1))
    assert r20 < 0.015 < r30 < r50
    assert (p0 + p1) / 2 < r50 / 3


# ------------------------------------------------- SIMD CPU baseline ---

@pytest.mark.parametrize("hint", [0, -1])
def test_simd_fdr_equals_scalar_oracle(hint):
    """oracle.c's SSE2 get_conf_stride_1 port (bench.py's cpu_baseline
    engine) == the scalar restatement: the reference's known answers
    (fdr.cpp fixtures, FDR engine) and random sets / buffers / starts."""
    for c in load("fdr.json"):
        blob = build_or_none(lits_of(c), 0)
        if blob is None or blob.engine_id != 0 or c["expected"] is None:
            continue
        data = bytes.fromhex(c["data"])
        st, m = oracle.fdr_exec_simd(vsa.engine_blob(blob), data, start=c["start"])
        assert st == 0 and [list(x) for x in m] == c["expected"], c["src"]
    rng = random.Random(77 + hint)
    for trial in range(12):
        lits = rand_lits(rng, rng.choice([50, 300, 2000]), minlen=rng.choice([1, 3, 5]),
                         msk_frac=0.1)
        blob = build_or_none(lits, hint)
        if blob is None or blob.is_noodle or blob.engine_id != 0:
            continue
        for ln in (17, 40, 300, 5000, 70000):
            data = rand_data(rng, ln, alphabet=b"abcdefgh" + bytes([rng.randrange(256)]) * 4)
            for start in (0, 5, ln // 3):
                a = oracle.fdr_exec(vsa.engine_blob(blob), data, start=start, cap=1 << 18)
                b = oracle.fdr_exec_simd(vsa.engine_blob(blob), data, start=start, cap=1 << 18)
                assert a == b, (trial, ln, start)


@pytest.mark.parametrize("kind", ["shufti", "truffle"])
def test_class_bitmap_of_masks(kind):
    """oracle.class_bitmap_of_masks (the cfg-2 full-buffer check) agrees with
    the oracle's own first / last scans over the same masks and with
    membership of the class the masks were built from."""
    rng = np.random.default_rng(7)
    for nchars in (0, 1, 8, 60, 200):
        chars = bytes(rng.choice(256, nchars, replace=False).astype(np.uint8))
        data = rng.integers(0, 256, 20000 + nchars, dtype=np.uint8)
        if kind == "shufti":
            m = vsa.shufti_build_masks(chars) if chars else (bytes(16), bytes(16))
            if m is None:
                continue
            first, last = oracle.shufti(*m, data), oracle.shufti(*m, data, reverse=True)
        else:
            m = vsa.truffle_build_masks(chars)
            first, last = oracle.truffle(*m, data), oracle.truffle(*m, data, reverse=True)
        bits, n = oracle.class_bitmap_of_masks(kind, m[0], m[1], data)
        member = np.isin(data, np.frombuffer(chars, np.uint8))
        assert np.array_equal(bits.view(np.uint8)[:(len(data) + 7) // 8],
                              np.packbits(member, bitorder="little"))
        idx = np.flatnonzero(member)
        assert n == len(idx)
        assert first == (idx[0] if len(idx) else len(data))
        assert last == (idx[-1] if len(idx) else -1)
