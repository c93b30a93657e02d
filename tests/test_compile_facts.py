"""CPU: the compile-side facts the reference's own FDR / Teddy unit tests
depend on, asserted on the product's builder (csrc/compile.cpp).

The reference unit tests (unit/internal/fdr.cpp, fdr_flood.cpp) run every
literal set once per engine id that getValidFdrEngines() returns
(fdr.cpp:114-137) and skip a Teddy id whose hinted build fails
(CHECK_WITH_TEDDY_OK_TO_FAIL, fdr.cpp:61-69).  What those tests therefore
rely on from the compile side:

  * the engine table: FDR id 0 (fdr_engine_description.cpp:55-59) and Teddy
    ids 3-18 with their mask count, bucket count and packing
    (teddy_engine_description.cpp:53-71);
  * which (literal set, engine id) pairs build: a hinted Teddy build fails
    only past TEDDY_BUCKET_LOAD literals per bucket or when packing cannot
    fit the buckets (teddy_compile.cpp:622-650, 661-681); a hinted FDR build
    always builds, at domain 9 stride 1 (fdr_compile.cpp:855-866);
  * the unhinted choice: noodle for one literal (hwlm_build.cpp:104-118),
    else the best-scored allowed Teddy (teddy_engine_description.cpp:95-200),
    else FDR at chooseEngine's domain / stride (fdr_engine_description.cpp:
    61-199).

The scoring rules are restated below from those lines and compared with
the blobs the builder emits, on every literal set of the golden fixtures and
on random sets.  Byte identity of whole blobs with reference-built ones stays
unpinned (nothing reference-built runs here): DESIGN.md says so.
"""
import json
import os
import random

import numpy as np
import pytest

import vectorscan_amd as vsa

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HDR = vsa.HWLM_HEADER

# teddy_engine_description.cpp:54-71: (id, avx2, numMasks, numBuckets, packed)
REF_TEDDY = [(3, True, 1, 16, False), (4, True, 1, 16, True), (5, True, 2, 16, False),
             (6, True, 2, 16, True), (7, True, 3, 16, False), (8, True, 3, 16, True),
             (9, True, 4, 16, False), (10, True, 4, 16, True), (11, False, 1, 8, False),
             (12, False, 1, 8, True), (13, False, 2, 8, False), (14, False, 2, 8, True),
             (15, False, 3, 8, False), (16, False, 3, 8, True), (17, False, 4, 8, False),
             (18, False, 4, 8, True)]
TEDDY = {t[0]: t for t in REF_TEDDY}
TEDDY_BUCKET_LOAD = 6                      # teddy_engine_description.h:40
RTABLE_SIZE = (256 + 1) * 8                # teddy_compile.cpp:324-327


def rucl(x):
    return (x + 63) & ~63


def u32(b, off):
    return int.from_bytes(b[off:off + 4], "little")


def build(lits, hint=-1):
    try:
        return vsa.hwlm_build(lits, engine_hint=hint)
    except vsa.BuildError:
        return None


def golden_sets():
    """every literal set the golden fixtures hold (fdr.cpp, fdr_flood.cpp,
    the streaming cases, ShortWritings' pattern sets)"""
    out = []
    for name in ("fdr.json", "fdr_stream.json"):
        with open(os.path.join(GOLD, name)) as f:
            for c in json.load(f):
                out.append([vsa.HwlmLiteral(bytes.fromhex(l["s"]), l["nocase"], l["id"],
                                            noruns=l["noruns"]) for l in c["lits"]])
    with open(os.path.join(GOLD, "fdr_flood.json")) as f:
        for c in json.load(f):
            out.append([vsa.HwlmLiteral(bytes.fromhex(t), bool(nc), i, msk=bytes.fromhex(m),
                                        cmp=bytes.fromhex(cm))
                        for t, nc, i, m, cm in c["lits"]])
    with open(os.path.join(GOLD, "fdr_shortwritings.json")) as f:
        for spec in json.load(f):
            out.append([vsa.HwlmLiteral(bytes.fromhex(p), False, i)
                        for i, p in enumerate(spec["pats"])])
    # dedupe (the flood fixtures repeat shapes per byte value)
    seen, uniq = set(), []
    for s in out:
        k = tuple((l.s, l.nocase, l.id, l.msk) for l in s)
        if k not in seen:
            seen.add(k)
            uniq.append(s)
    return uniq


# --------------------------------------------------- restated choices ---

def ref_choose_teddy(lits):
    """chooseTeddyEngine + isAllowed (teddy_engine_description.cpp:95-200)
    on an AVX2 target: the chosen id or None"""
    max_len = max(len(l.s) for l in lits)
    tail = 0
    for l in lits:
        s = l.s
        j = 1
        while j < len(s) and s[len(s) - j - 1] == s[-1]:
            j += 1
        tail = max(tail, j)
    best, best_score = None, 0
    for tid, _, masks, buckets, packed in REF_TEDDY:
        n = len(lits)
        if buckets < n and not packed:
            continue
        if buckets * TEDDY_BUCKET_LOAD < n:
            continue
        if masks > max_len:
            continue
        if n > 40 and sum(len(l.s) < masks for l in lits) * 5 > n:
            continue
        score = (100 if not packed else 0)
        score += masks * 4 if n > 4 * buckets else 100
        score += 50 if masks > tail else 0
        score += 6 // (abs(3 - masks) + 1)
        score += 16 // buckets
        if best is None or score > best_score:
            best, best_score = tid, score
    return best


def ref_choose_fdr(lits):
    """chooseEngine (fdr_engine_description.cpp:61-199), 64-bit scheme,
    8 buckets, not an atom-class target, make_small off: (domain, stride)"""
    lens = [len(l.s) for l in lits]
    msl = min(lens)
    cnt = lens.count(msl)
    n = len(lits)
    want = 1
    if msl > 1:
        if n < 250:
            want = msl
        elif n < 800:
            want = msl - 1
        elif n < 5000:
            want = min(msl - 1, 2)
    if msl == 4 and want == 4 and cnt > 2:
        want = 2
    best, best_score = None, 0
    for domain in range(9, 16):
        for stride in (1, 2, 4):
            if domain > 13 and stride > 1:
                continue
            if msl < stride:
                continue
            score = 100 - abs(want - stride)
            if stride <= want:
                score += stride
            if n < 8:
                ideal = 8 if stride == 1 else 10
            elif n < 20:
                ideal = 10
            elif n < 100:
                ideal = 11
            elif n < 1000:
                ideal = 12
            elif n < 10000:
                ideal = 13
            else:
                ideal = 15
            if stride > 1:
                ideal += 1
            score -= abs(ideal - domain)
            if best is None or score > best_score:
                best, best_score = (domain, stride), score
    return best


def fdr_fields(blob):
    raw = blob.tobytes()
    e = raw[HDR:]
    return {"engine": u32(e, 0), "size": u32(e, 4), "max_len": u32(e, 8), "n": u32(e, 12),
            "conf_off": u32(e, 16), "flood_off": u32(e, 20), "stride": e[24], "domain": e[25],
            "raw_len": len(raw)}


# ----------------------------------------------------------- tests ------

def test_engine_table_layout():
    """each Teddy id builds as itself with the reference's mask count and
    bucket width: the confirm table starts after the header, the nibble
    masks (numMasks * 32 * maskWidth) and the reinforcement table (Teddy) or
    duplicated masks (Fat Teddy), each cacheline-rounded
    (teddy_compile.cpp:555-600)"""
    lits = [vsa.HwlmLiteral(b"abcdefgh", False, 1), vsa.HwlmLiteral(b"zyxwvuts", True, 2)]
    for tid, avx2, masks, buckets, _ in REF_TEDDY:
        b = build(lits, tid)
        assert b is not None, tid
        f = fdr_fields(b)
        mw = buckets // 8
        assert avx2 == (mw == 2), tid  # the 16-bucket engines are the AVX2 ones
        mask_len = masks * 16 * 2 * mw
        extra = RTABLE_SIZE * mw if mw == 1 else mask_len * 2
        assert (f["engine"], f["n"], f["max_len"]) == (tid, 2, 8), tid
        assert f["conf_off"] == rucl(24) + rucl(mask_len) + rucl(extra), tid
        assert HDR + f["size"] == f["raw_len"]
    # FDR id 0, hinted: domain 9, stride 1 (fdr_compile.cpp:862-866)
    f = fdr_fields(build(lits, 0))
    assert (f["engine"], f["domain"], f["stride"]) == (0, 9, 1)
    # ids outside the table do not build
    for bad in (1, 2, 19, 40):
        assert build(lits, bad) is None, bad


def test_hinted_buildability_golden_sets():
    """for every golden literal set and every valid engine id: FDR always
    builds (domain 9, stride 1); Teddy builds whenever the set fits the
    buckets unpacked, never past TEDDY_BUCKET_LOAD per bucket, and when it
    builds it carries the set's string count and maximum length"""
    sets = golden_sets()
    assert len(sets) > 20
    for lits in sets:
        n = len(lits)
        mx = max(len(l.s) for l in lits)
        f = fdr_fields(build(lits, 0))
        assert (f["engine"], f["domain"], f["stride"], f["n"], f["max_len"]) == (0, 9, 1, n, mx)
        for tid, _, masks, buckets, _ in REF_TEDDY:
            b = build(lits, tid)
            if n > buckets * TEDDY_BUCKET_LOAD:
                assert b is None, (tid, n)
                continue
            if n <= buckets:
                assert b is not None, (tid, n)
            if b is not None:
                f = fdr_fields(b)
                assert (f["engine"], f["n"], f["max_len"]) == (tid, n, mx), (tid, n)


def _random_set(rng, n, lo, hi, nocase_frac=0.0, alpha=None):
    alpha = alpha or bytes(range(0x20, 0x7F))
    while sum(len(alpha) ** k for k in range(lo, hi + 1)) < 2 * n:
        hi += 1  # room for n distinct strings
    out, seen = [], set()
    while len(out) < n:
        s = bytes(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))
        if s in seen:
            continue
        seen.add(s)
        out.append(vsa.HwlmLiteral(s, rng.random() < nocase_frac, len(out)))
    return out


@pytest.mark.parametrize("seed", range(6))
def test_unhinted_choice_matches_reference_rules(seed):
    """unhinted builds of random sets (1 - 12000 literals, minimum lengths
    1 - 8): noodle for one literal; the reference-scored Teddy when one is
    allowed (or FDR when that Teddy cannot pack, which a hinted build then
    confirms); otherwise FDR at the reference-scored domain and stride"""
    rng = random.Random(9000 + seed)
    sizes = [1, 2, 5, 8, 9, 16, 30, 41, 48, 60, 96, 97, 200, 300, 900, 2000]
    if seed < 2:
        sizes += [5000, 12000]
    for n in sizes:
        lo = rng.randint(1, 8)
        lits = _random_set(rng, n, lo, min(8, lo + rng.randint(0, 6)), nocase_frac=0.1,
                           alpha=b"abcdefgh" if lo <= 2 and n <= 48 else None)
        n = len(lits)
        b = build(lits)
        assert b is not None
        if n == 1:
            assert b.is_noodle
            continue
        f = fdr_fields(b)
        want_t = ref_choose_teddy(lits)
        if want_t is not None and f["engine"] == want_t:
            continue
        if want_t is not None:
            # the chosen Teddy could not pack: the reference falls to FDR too
            # (fdr_compile.cpp:844-853)
            assert f["engine"] == 0 and build(lits, want_t) is None, (n, want_t, f["engine"])
        assert f["engine"] == 0, (n, lo)
        assert (f["domain"], f["stride"]) == ref_choose_fdr(lits), (n, lo)
        assert f["n"] == n


def test_cfg4_set_facts():
    """the headline set (bench.make_literals(5000)): FDR, domain 13, stride
    1, 8 buckets, as chooseEngine scores it"""
    import bench
    lits = bench.make_literals(5000, seed=12)
    assert ref_choose_teddy(lits) is None
    f = fdr_fields(build(lits))
    assert (f["engine"], f["domain"], f["stride"]) == (0, 13, 1) == (0,) + ref_choose_fdr(lits)
    assert np.uint32(f["n"]) == 5000
