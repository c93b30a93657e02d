"""The reference's own hs-level known answers for pure literals
(unit/hyperscan/behaviour.cpp, restated as data in
tests/golden/hs_behaviour.json by tests/golden/make_golden.py):

* HyperscanScanGigabytesMatch BlockMatch (:241-303, allocAndScanBlock
  :211-235): a zero-filled block with a pre-block at 0 and a post-block at
  the end, 1 KiB .. 1 MiB (+4, +len(post)); the last match's `to` is the
  block length.  The BIG_BLOCKS sizes (:266-273: 4 MiB .. 3 GiB) run on the
  GPU only.
* StreamingMatch (:137-208): pre-block, gb x 1024 writes of 1 MiB of 'X',
  post-block, close; no match until the post-block, then `to` = the stream
  length.
* LiteralLength FloatingBlock (:404-440, :481-483): 'a' * L in 'a' * (L + 4)
  matches 5 times, and 0 times from 5 bytes in.
* CallbackReturnStop (:494-599) pure-literal rows: exactly one match and
  HS_SCAN_TERMINATED in block, stream and vectored mode.
* SerializedDogfood1 (:613-662): a deserialized database has the same size
  and matches "delicious puppy treats!" at its end.

The CPU tests check oracle/hs_lit.py (the restatement the rest of the hs
tests compare the GPU with) against these answers; the GPU tests run the
product (vsa_hs_* through the C ABI) on them at full size.
"""
import json
import os

import numpy as np
import pytest

from oracle import hs_lit as ohs
import vectorscan_amd as vsa
from vectorscan_amd import hs

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "hs_behaviour.json")) as _f:
    G = json.load(_f)


def block_of(case, n):
    """allocAndScanBlock (behaviour.cpp:216-225): calloc(len), pre-block at
    0, post-block at len - strlen(post)"""
    a = np.zeros(n, np.uint8)
    pre, post = case["pre"].encode(), case["post"].encode()
    a[:len(pre)] = np.frombuffer(pre, np.uint8)
    a[n - len(post):] = np.frombuffer(post, np.uint8)
    return a


def oracle_pair(patterns, flags):
    odb = ohs.compile_lit_multi([p.encode() for p in patterns], flags)
    lits = [vsa.HwlmLiteral(t, nc, f, noruns=nr) for t, nc, f, nr in odb.hwlm_literals()]
    blob = vsa.hwlm_build(lits)
    return odb, blob


# ------------------------------------------------------------------ CPU ---

def test_fixture_shape():
    assert len(G["block_gigabytes"]) == 2 and len(G["block_gigabytes"][0]["lens"]) == 30
    assert [c["literal_len"] for c in G["literal_length_floating"]][-1] == 15999
    assert {c["corpus"] for c in G["callback_stop"]} == {
        "xxxfoobarxxxfoobarxxxfoobar", "xxxaaaaaaaaaaaaaaaaaaa", "xxxAaAaAaAa"}


@pytest.mark.parametrize("ci", range(2))
def test_oracle_block_gigabytes(ci):
    case = G["block_gigabytes"][ci]
    odb, blob = oracle_pair([case["pattern"]], [case["flags"]])
    for n, want in zip(case["lens"], case["expected_last_to"]):
        out = ohs.scan(odb, blob.ptr, block_of(case, n))
        assert out and out[-1][2] == want, (case["pattern"], n)


@pytest.mark.parametrize("case", [c for c in G["stream_gigabytes"] if c["chunks"] == 1024],
                         ids=lambda c: c["pattern"][:8])
def test_oracle_stream_gigabytes(case):
    """the same stream rule with 16 writes of 1 MiB (the GPU test writes the
    reference's 1 and 2 GiB)"""
    odb, blob = oracle_pair([case["pattern"]], [case["flags"]])
    chunks = 16
    fill = np.full(case["chunk"], ord(case["fill"]), np.uint8)
    writes = [case["pre"].encode()] + [fill] * chunks
    assert ohs.scan_writes(odb, blob.ptr, writes) == []
    out = ohs.scan_writes(odb, blob.ptr, writes + [case["post"].encode()])
    total = len(case["pre"]) + chunks * case["chunk"] + len(case["post"])
    assert out and out[-1][2] == total


def test_oracle_literal_length():
    for c in G["literal_length_floating"]:
        odb, blob = oracle_pair(["a" * c["literal_len"]], [0])
        data = b"a" * c["data_len"]
        assert len(ohs.scan(odb, blob.ptr, data)) == c["expected_count"], c["literal_len"]
        assert len(ohs.scan(odb, blob.ptr, data[5:])) == c["expected_count_from5"]


def test_oracle_callback_stop():
    for c in G["callback_stop"]:
        odb, blob = oracle_pair([c["pattern"]], [c["flags"]])
        data = c["corpus"].encode()
        assert len(ohs.scan(odb, blob.ptr, data, stop_after=1)) == c["expected_count"]
        assert len(ohs.scan_writes(odb, blob.ptr, [data], stop_after=1)) == c["expected_count"]


def test_serialized_dogfood_size():
    """hs_database_size before serialization == after deserialization
    (behaviour.cpp:619-646); no scan, so no GPU"""
    c = G["serialized_dogfood"][0]
    db = hs.compile_lit_multi([c["pattern"].encode()], [c["flags"]], None, hs.MODE_BLOCK)
    size0 = db.size()
    blob = db.serialize()
    db.close()
    db2 = hs.deserialize(blob)
    assert (db2.size() == size0) == c["expected_size_equal"]
    assert hs.serialized_size(blob) == size0


# ------------------------------------------------------------------ GPU ---

def _last_to(matches):
    return matches[-1][2] if matches else 0


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(2))
def test_gpu_block_gigabytes(ci):
    case = G["block_gigabytes"][ci]
    db = hs.compile_lit_multi([case["pattern"].encode()], [case["flags"]], None, hs.MODE_BLOCK)
    s = hs.Scratch(db)
    for n, want in zip(case["lens"], case["expected_last_to"]):
        rc, out = hs.scan(db, block_of(case, n), s)
        assert rc == case["expected_status"] and _last_to(out) == want, (n, rc, out[-3:])


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(2))
def test_gpu_big_blocks(ci):
    """BIG_BLOCKS (behaviour.cpp:266-273): up to 3 GiB in one hs_scan"""
    case = G["big_block"][ci]
    db = hs.compile_lit_multi([case["pattern"].encode()], [case["flags"]], None, hs.MODE_BLOCK)
    s = hs.Scratch(db)
    for n, want in zip(case["lens"], case["expected_last_to"]):
        for m in (n, n + 4, n + len(case["post"])):
            rc, out = hs.scan(db, block_of(case, m), s)
            assert rc == case["expected_status"] and _last_to(out) == m, (m, rc, out[-3:])


@pytest.mark.gpu
@pytest.mark.parametrize("ci", range(4))
def test_gpu_stream_gigabytes(ci):
    case = G["stream_gigabytes"][ci]
    db = hs.compile_lit_multi([case["pattern"].encode()], [case["flags"]], None,
                              hs.MODE_STREAM)
    s = hs.Scratch(db)
    st = hs.Stream(db)
    seen = []
    cb = lambda i, f, t, fl: seen.append(t) and False  # noqa: E731
    assert st.scan(case["pre"].encode(), s, cb)[0] == case["expected_status"]
    fill = np.full(case["chunk"], ord(case["fill"]), np.uint8)
    for _ in range(case["chunks"]):
        assert st.scan(fill, s, cb)[0] == case["expected_status"]
    assert (seen[-1] if seen else 0) == case["expected_last_to_before_post"]
    assert st.scan(case["post"].encode(), s, cb)[0] == case["expected_status"]
    assert st.close(s, cb) == hs.SUCCESS
    assert seen and seen[-1] == case["expected_last_to_after_close"]


@pytest.mark.gpu
def test_gpu_literal_length():
    for c in G["literal_length_floating"]:
        db = hs.compile_lit_multi([b"a" * c["literal_len"]], [0], None, hs.MODE_BLOCK)
        s = hs.Scratch(db)
        data = b"a" * c["data_len"]
        rc, out = hs.scan(db, data, s)
        assert rc == hs.SUCCESS and len(out) == c["expected_count"], (c["literal_len"], out)
        rc, out = hs.scan(db, data[5:], s)
        assert rc == hs.SUCCESS and len(out) == c["expected_count_from5"], c["literal_len"]


@pytest.mark.gpu
def test_gpu_callback_stop():
    for c in G["callback_stop"]:
        data = c["corpus"].encode()
        cnt = []

        def stop(i, f, t, fl):
            cnt.append(t)
            return True

        # Block (:494-522)
        db = hs.compile_lit_multi([c["pattern"].encode()], [c["flags"]], None, hs.MODE_BLOCK)
        s = hs.Scratch(db)
        rc, _ = hs.scan(db, data, s, stop)
        assert rc == c["expected_status"] and len(cnt) == c["expected_count"], c
        # Streaming (:524-561): the close after termination succeeds
        cnt.clear()
        db = hs.compile_lit_multi([c["pattern"].encode()], [c["flags"]], None, hs.MODE_STREAM)
        s = hs.Scratch(db)
        st = hs.Stream(db)
        rc, _ = st.scan(data, s, stop)
        assert rc == c["expected_status"] and len(cnt) == c["expected_count"], c
        assert st.close(s, stop) == c["expected_close_status"]
        # Vectored (:563-594)
        cnt.clear()
        db = hs.compile_lit_multi([c["pattern"].encode()], [c["flags"]], None,
                                  hs.MODE_VECTORED)
        s = hs.Scratch(db)
        rc, _ = hs.scan_vector(db, [data], s, stop)
        assert rc == c["expected_status"] and len(cnt) == c["expected_count"], c


@pytest.mark.gpu
def test_gpu_serialized_dogfood():
    c = G["serialized_dogfood"][0]
    db = hs.compile_lit_multi([c["pattern"].encode()], [c["flags"]], None, hs.MODE_BLOCK)
    size0 = db.size()
    blob = db.serialize()
    db.close()
    db2 = hs.deserialize(blob)
    assert db2.size() == size0
    s = hs.Scratch(db2)
    rc, out = hs.scan(db2, c["data"].encode(), s)
    assert rc == hs.SUCCESS and _last_to(out) == c["expected_last_to"]
