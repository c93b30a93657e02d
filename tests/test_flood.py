"""Flood detection (src/fdr/flood_runtime.h:41-335) with the
reference's default Grey (fdrAllowFlood, grey.cpp:68): the known answers of
unit/internal/fdr_flood.cpp (restated in tests/golden/fdr_flood.json) for the
oracle's restatement and the GPU drop-in, and exact callback sequences GPU ==
oracle on flood-heavy inputs (the flood shortcut reports its ids in its own
order, without NOREPEAT, and skips the main loop over the run)."""
import ctypes
import random
from collections import Counter

import numpy as np
import pytest

import oracle
import vectorscan_amd as vsa
from test_cpu_oracle import load, rand_lits

HINTS = [0, 11, 12, 15, 17, 18, 3, 4, 7, 9]


def flood_lits(case):
    return [vsa.HwlmLiteral(bytes.fromhex(s), bool(nc), i, msk=bytes.fromhex(m),
                            cmp=bytes.fromhex(cm))
            for s, nc, i, m, cm in case["lits"]]


def build(lits, hint, flood=True):
    try:
        return vsa.hwlm_build(lits, engine_hint=hint, allow_flood=flood)
    except vsa.BuildError:
        return None


def check_counts(seq, expected, what):
    got = Counter(i for _, i in seq)
    for k, v in expected.items():
        assert got.get(int(k), 0) == v, (what, int(k), got.get(int(k), 0), v)


def placed(data, mis):
    """bytes at an address = mis (mod 64): the flood probes are 8-byte
    aligned loads, so the buffer address matters (flood_runtime.h:50-62)"""
    raw = ctypes.create_string_buffer(len(data) + 128)
    addr = (ctypes.addressof(raw) + 63) & ~63
    addr += mis
    ctypes.memmove(addr, bytes(data), len(data))
    return raw, addr


def oracle_fdr(blob, addr, n, **kw):
    """oracle fdrExec on host memory at `addr` (no copy: alignment kept)"""
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(addr))[:n]
    return oracle.fdr_exec(vsa.engine_blob(blob), arr, **kw)


def gpu_fdr(blob, addr, n, start=0, groups=vsa.HWLM_ALL_GROUPS, cb_ret=None, term_after=-1):
    seq = []

    def cb(end, id_, scr):
        seq.append((end, id_))
        if term_after >= 0 and len(seq) >= term_after:
            return 0
        return vsa.HWLM_ALL_GROUPS if cb_ret is None else cb_ret

    ccb = vsa.HWLMCallback(cb)
    rc = vsa.lib.fdrExec(vsa.engine_blob(blob), addr, n, start, ccb, None, groups)
    return rc, seq


# ----------------------------------------------------------- CPU oracle --

@pytest.mark.parametrize("hint", HINTS)
def test_oracle_fdr_flood_known_answers(hint):
    """fdr_flood.cpp NoMask / WithMask: per-id counts over 1024 bytes of c
    and of cAlt, every c, flood detection on."""
    changed = 0
    for case in load("fdr_flood.json"):
        lits = flood_lits(case)
        blob = build(lits, hint)
        if blob is None:
            continue
        plain = build(lits, hint, flood=False)
        for run in case["runs"]:
            data = bytes([run["fill"]]) * 1024
            st, m = oracle.fdr_exec(vsa.engine_blob(blob), data, cap=1 << 16)
            assert st == 0
            check_counts(m, run["expected"], (case["src"], case["c"], hint))
            _, m0 = oracle.fdr_exec(vsa.engine_blob(plain), data, cap=1 << 16)
            assert Counter(m) == Counter(m0)
            changed += m != m0
    # the flood path ran: its report order differs from the confirm order
    assert changed > 0


@pytest.mark.parametrize("hint", [0, 17, 3])
def test_oracle_fdr_flood_streaming_mask(hint):
    """fdr_flood.cpp StreamingMask :404-558: the buffer of c fed as
    streaming calls of 1..16 bytes with 8 (or j < 16) bytes of history."""
    for case in load("fdr_flood.json")[1::2][::9]:
        lits = flood_lits(case)
        blob = build(lits, hint)
        if blob is None:
            continue
        c = case["c"]
        eng = vsa.engine_blob(blob)
        for chunk in (1, 2, 4, 8, 16):
            seq = []
            _, m = oracle.fdr_exec_stream(eng, b"", bytes([c]) * chunk, cap=1 << 12)
            seq += m
            for j in range(chunk, 1024, chunk):
                hist = bytes([c]) * (j if j < 16 else 8)
                _, m = oracle.fdr_exec_stream(eng, hist, bytes([c]) * chunk, cap=1 << 12,
                                              filler=bytes([c]) * 16)
                seq += m
            check_counts(seq, case["runs"][0]["expected"], (case["src"], c, hint, chunk))


def flood_text(rng, n, alphabet=b"abcdxyzAB"):
    """random text with long runs of one byte (floods) of random lengths"""
    out = bytearray()
    while len(out) < n:
        if rng.random() < 0.3:
            out += bytes([rng.choice(alphabet)]) * rng.randint(16, 900)
        else:
            out += bytes(rng.choice(alphabet) for _ in range(rng.randint(1, 60)))
    return bytes(out[:n])


# ------------------------------------------------------------------ GPU --

@pytest.mark.gpu
@pytest.mark.parametrize("hint", [0, 11, 17, 3, 9])
def test_gpu_fdr_flood_known_answers(hint):
    """The drop-in on flood-enabled engines: the fdr_flood.cpp counts, and
    the exact oracle sequence (flood reports in place of confirm order)."""
    for case in load("fdr_flood.json"):
        lits = flood_lits(case)
        blob = build(lits, hint)
        if blob is None:
            continue
        for run in case["runs"]:
            keep, addr = placed(bytes([run["fill"]]) * 1024, 0)
            _, want = oracle_fdr(blob, addr, 1024, cap=1 << 16)
            rc, got = gpu_fdr(blob, addr, 1024)
            assert rc == 0
            check_counts(got, run["expected"], (case["src"], case["c"], hint))
            assert got == want, (case["src"], case["c"], hint)


@pytest.mark.gpu
@pytest.mark.parametrize("vsize", [16, 32, 64])
@pytest.mark.parametrize("seed", range(6))
def test_gpu_flood_random_sequences(seed, vsize):
    """Random literal sets rich in single-byte runs (so the flood tables
    hold ids), flood-heavy text, every engine kind, several buffer
    alignments and starts, group masks, NOREPEAT, early termination: the
    drop-in's callback sequence == the oracle's, Teddy under the loop shape
    of each emulated build."""
    rng = random.Random(seed * 101 + vsize)
    vsa.set_accel_vector_size(vsize)
    oracle.set_vector_size(vsize)
    try:
        for trial in range(6):
            lits = rand_lits(rng, rng.randint(2, 60), minlen=1, maxlen=8, alphabet=b"abcdxyz",
                             msk_frac=0.1)
            for l in lits:
                if rng.random() < 0.4:  # runs of one byte: flood-table ids
                    l.s = bytes([rng.choice(b"abcdxyz")]) * len(l.s)
                    l.msk = l.cmp = b""
                l.noruns = rng.random() < 0.3
                l.groups = rng.choice([1, 2, 3, vsa.HWLM_ALL_GROUPS])
            hint = rng.choice([-1, 0, 0, 11, 13, 15, 17, 18, 3, 5, 7, 9, 10])
            blob = build(lits, hint)
            if blob is None or blob.is_noodle:
                continue
            for ln in (255, 256, 300, 1000, 5000, 40000):
                data = flood_text(rng, ln)
                mis = rng.randrange(64)
                keep, addr = placed(data, mis)
                for start in sorted({0, 1, 17, ln // 3}):
                    for kw in ({}, {"groups": 1}, {"cb_ret": 2}, {"term_after": 7}):
                        so, want = oracle_fdr(blob, addr, ln, start=start, cap=1 << 20, **kw)
                        sg, got = gpu_fdr(blob, addr, ln, start=start, **kw)
                        assert (sg, got) == (so, want), (seed, vsize, trial, hint, ln, mis,
                                                         start, kw, blob.engine_id)
    finally:
        vsa.set_accel_vector_size(64)
        oracle.set_vector_size(64)
