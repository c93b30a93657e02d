"""hsbench-compatible driver: the reference's expression-file
and sqlite corpus formats (tools/hsbench: util/expressions.cpp,
ExpressionParser.rl, data_corpus.cpp, scripts/CorpusBuilder.py), and
vsa_hs_scan_corpus — the corpus loop as one launch — against per-block
vsa_hs_scan calls and the oracle's pure-literal restatement (block,
streaming, vectored)."""
import os
import random

import numpy as np
import pytest

from oracle import hs_lit as ohs
import vectorscan_amd as vsa
from vectorscan_amd import hs, hsbench


def test_read_expression():
    assert hsbench.read_expression("/foobar/") == ("foobar", 0)
    assert hsbench.read_expression("/foo/bar/iH") == ("foo/bar", hs.FLAG_CASELESS |
                                                      hs.FLAG_SINGLEMATCH)
    assert hsbench.read_expression("/a.b\\x41/L") == ("a.b\\x41", hs.FLAG_SOM_LEFTMOST)
    for bad in ["foo", "/", "/abc/q", ""]:
        with pytest.raises(hsbench.ExpressionError):
            hsbench.read_expression(bad)
    with pytest.raises(hsbench.ExpressionError):
        hsbench.read_expression("/abc/{min_offset=3}")


def test_load_expressions(tmp_path):
    f = tmp_path / "sigs"
    f.write_text("# comment\n\n10:/abc/i\n  7:/xyz/ \n3:/q/H\n")
    m = hsbench.load_expressions(str(f))
    assert m == {10: "/abc/i", 7: "/xyz/", 3: "/q/H"}
    exprs, ids, flags = hsbench.build_set(m)
    assert ids == [3, 7, 10] and exprs == [b"q", b"xyz", b"abc"]
    assert flags == [hs.FLAG_SINGLEMATCH, 0, hs.FLAG_CASELESS]
    exprs, ids, _ = hsbench.build_set(m, [10, 3])
    assert ids == [3, 10]
    d = tmp_path / "dir"
    d.mkdir()
    (d / "a").write_text("1:/aa/\n")
    (d / "b~").write_text("2:/bb/\n")
    (d / ".c").write_text("3:/cc/\n")
    (d / "d").write_text("4:/dd/\n")
    assert hsbench.load_expressions(str(d)) == {1: "/aa/", 4: "/dd/"}
    (d / "e").write_text("4:/ee/\n")
    with pytest.raises(hsbench.ExpressionError):
        hsbench.load_expressions(str(d))
    (d / "e").write_text("x:/ee/\n")
    with pytest.raises(hsbench.ExpressionError):
        hsbench.load_expressions(str(d / "e"))


def test_corpus_roundtrip_and_layout(tmp_path):
    chunks = [(0, b"alpha"), (1, b"beta"), (0, b"gamma"), (2, b"d"), (1, b"eps")]
    path = str(tmp_path / "c.db")
    hsbench.write_corpus(path, chunks)
    blocks = hsbench.read_corpus(path)
    assert blocks == [(i, s, d) for i, (s, d) in enumerate(chunks)]
    img, offs, lens, sids = hsbench.layout(blocks, hs.MODE_BLOCK)
    assert img.tobytes() == b"alphabetagammadeps" and list(sids) == [0, 1, 0, 2, 1]
    img, offs, lens, sids = hsbench.layout(blocks, hs.MODE_STREAM)
    assert img.tobytes() == b"alphagammabetaepsd"
    assert list(sids) == [0, 0, 1, 1, 2] and list(offs) == [0, 5, 10, 14, 17]
    with pytest.raises(IOError):
        hsbench.read_corpus(str(tmp_path / "missing.db"))


def test_calc_mbps():
    assert hsbench.calc_mbps(1.0, 125000) == 1.0
    assert hsbench.calc_mbps(0.5, 1 << 30) == (1 << 30) / 62500.0


def make_corpus(rng, exprs, nstreams, nchunks, lo, hi, alpha):
    chunks = []
    for c in range(nchunks):
        ln = rng.randint(lo, hi)
        b = bytearray(rng.choice(alpha) for _ in range(ln))
        for _ in range(max(1, ln // 300)):
            e = rng.choice(exprs)
            if len(e) < ln:
                p = rng.randrange(0, ln - len(e))
                b[p:p + len(e)] = e
        if ln > 400 and c % 3 == 0:
            p = rng.randrange(0, ln - 300)
            b[p:p + 280] = bytes([alpha[0]]) * 280
        chunks.append((rng.randrange(nstreams), bytes(b)))
    return chunks


CASES = [
    # (n, len lo, hi, alphabet, flag mix, dup ids)
    (40, 2, 8, b"abcdef", (0, hs.FLAG_CASELESS), False),              # Teddy, simple
    (600, 3, 8, b"abcdefgh", (0,), False),                            # FDR, simple
    (300, 2, 24, b"abcdefgh", (0, hs.FLAG_CASELESS, hs.FLAG_SINGLEMATCH,
                              hs.FLAG_SOM_LEFTMOST), True),           # replay path
]


def make_case(k, seed):
    n, lo, hi, alpha, mix, dup = CASES[k]
    rng = random.Random(77 * k + seed)
    exprs = [bytes(rng.choice(alpha) for _ in range(rng.randint(lo, hi))) for _ in range(n)]
    flags = [rng.choice(mix) for _ in range(n)]
    ids = [rng.randrange(max(1, n // 3)) for _ in range(n)] if dup else list(range(n))
    single, som = {}, {}
    for i, f in enumerate(flags):
        s = single.setdefault(ids[i], bool(f & hs.FLAG_SINGLEMATCH))
        f = ((f | hs.FLAG_SINGLEMATCH) & ~hs.FLAG_SOM_LEFTMOST) if s else \
            (f & ~hs.FLAG_SINGLEMATCH)
        m = som.setdefault(ids[i], bool(f & hs.FLAG_SOM_LEFTMOST))
        flags[i] = (f | hs.FLAG_SOM_LEFTMOST) if m else (f & ~hs.FLAG_SOM_LEFTMOST)
    return rng, exprs, flags, ids, alpha


def oracle_counts(exprs, flags, ids, blocks, mode):
    """per-chunk counts from the oracle's pure-literal restatement, in the
    layout's scan order"""
    odb = ohs.compile_lit_multi(exprs, flags, ids)
    lits = [vsa.HwlmLiteral(t, nc, f, noruns=nr) for t, nc, f, nr in odb.hwlm_literals()]
    blob = vsa.hwlm_build(lits)
    img, offs, lens, sids = hsbench.layout(blocks, mode)
    counts = []
    if mode == hs.MODE_BLOCK:
        for o, ln in zip(offs, lens):
            counts.append(len(ohs.scan(odb, blob.ptr, img[int(o):int(o + ln)].copy())))
        return counts
    # streams: count per write through the shared run state
    runs = {}
    for o, ln, s in zip(offs, lens, sids):
        r = runs.setdefault(int(s), ohs._Run(odb))
        out = []
        r.write(blob.ptr, img[int(o):int(o + ln)].copy(), out)
        counts.append(len(out))
    return counts


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(CASES)))
@pytest.mark.parametrize("mode", [hs.MODE_BLOCK, hs.MODE_STREAM, hs.MODE_VECTORED])
def test_scan_corpus_counts(k, mode):
    rng, exprs, flags, ids, alpha = make_case(k, 1)
    chunks = make_corpus(rng, exprs, 7, 60, 1, 3000, alpha)
    blocks = [(i, s, d) for i, (s, d) in enumerate(chunks)]
    g = hsbench.GpuCorpus(exprs, ids, flags, blocks, mode)
    try:
        want = oracle_counts(exprs, flags, ids, blocks, mode)
        total, counts = g.scan(counts=True)
        assert list(counts) == want
        assert total == sum(want)
        t2, _ = g.scan()  # fast path (simple sets) or replay without counts
        assert t2 == total
        t3, _ = g.scan(threads=1)
        assert t3 == total
        if mode == hs.MODE_BLOCK:  # per-block hs_scan calls agree
            per = [len(hs.scan(g.db, d, g.scratch)[1]) for _, _, d in blocks]
            assert per == want
    finally:
        g.close()


@pytest.mark.gpu
def test_scan_corpus_errors():
    db = hs.compile_lit_multi([b"abc"], [0], [1], hs.MODE_STREAM)
    scratch = hs.Scratch(db)
    ctx = vsa.Context(0)
    d = ctx.malloc(64)
    try:
        # the second block of stream 0 does not follow the first: invalid
        rc, _, _ = hs.scan_corpus(db, scratch, d, [0, 20], [10, 10], [0, 0])
        assert rc == hs.INVALID
        rc, total, _ = hs.scan_corpus(db, scratch, d, [0, 10], [10, 10], [0, 0])
        assert rc == hs.SUCCESS
        long_db = hs.compile_lit_multi([b"abcdefghijk"], [0], [1], hs.MODE_BLOCK)
        scratch.grow(long_db)
        rc, _, _ = hs.scan_corpus(long_db, scratch, d, [0], [10])  # needs h_data
        assert rc == hs.INVALID
    finally:
        ctx.free(d)


@pytest.mark.gpu
@pytest.mark.parametrize("mode_flag", ["-N", "-V", None])
def test_hsbench_main(tmp_path, capsys, mode_flag):
    rng, exprs, flags, ids, alpha = make_case(1, 2)
    chunks = make_corpus(rng, exprs, 5, 40, 100, 4000, alpha)
    corpus = str(tmp_path / "corpus.db")
    hsbench.write_corpus(corpus, chunks)
    sig = tmp_path / "sigs"
    sig.write_text("".join("%d:/%s/\n" % (i, e.decode()) for i, e in zip(ids, exprs)))
    argv = ["-e", str(sig), "-c", corpus, "-n", "3", "--literal-on", "--json"]
    if mode_flag:
        argv.append(mode_flag)
    assert hsbench.main(argv) == 0
    out = capsys.readouterr().out
    import json
    res = json.loads(out.strip().splitlines()[-1])
    mode = {"-N": hs.MODE_BLOCK, "-V": hs.MODE_VECTORED, None: hs.MODE_STREAM}[mode_flag]
    blocks = [(i, s, d) for i, (s, d) in enumerate(chunks)]
    assert res["matches"] == sum(oracle_counts(exprs, [0] * len(exprs), ids, blocks, mode))
    assert "Mean throughput (overall):" in out and "WARNING" not in out


def cfg5_case(nbytes, nstreams=8, chunk=16 << 10):
    """the cfg-5-shaped pure-literal set (bench.make_mixed_set: 10k
    literals, length 4-16, CASELESS / SINGLEMATCH / SOM_LEFTMOST mixed, shared
    ids) planted once per 4 KiB in printable bytes, cut into `chunk`-byte
    chunks dealt round-robin over `nstreams` streams"""
    import bench
    exprs, flags, ids = bench.make_mixed_set(10000)
    lits = [vsa.HwlmLiteral(e, False, i) for i, e in enumerate(exprs)]
    data = bench.make_corpus(nbytes, lits, seed=9, plant_every=4 << 10)
    chunks = [(k % nstreams, data[o:o + chunk].tobytes())
              for k, o in enumerate(range(0, nbytes, chunk))]
    return exprs, flags, ids, [(i, s, d) for i, (s, d) in enumerate(chunks)]


def oracle_sequences(exprs, flags, ids, blocks, mode):
    """per-chunk callback sequences [(id, from, to)] from the oracle's
    pure-literal restatement (runtime.c:204-230 block, :802-831 streams:
    each stream's writes in order through one run state), indexed like
    `blocks`"""
    odb = ohs.compile_lit_multi(exprs, flags, ids)
    lits = [vsa.HwlmLiteral(t, nc, f, noruns=nr) for t, nc, f, nr in odb.hwlm_literals()]
    blob = vsa.hwlm_build(lits)
    seqs = [None] * len(blocks)
    runs = {}
    for i, s, d in blocks:
        data = np.frombuffer(d, np.uint8)
        if mode == hs.MODE_BLOCK:
            seqs[i] = ohs.scan(odb, blob.ptr, data)
            continue
        r = runs.setdefault(s, ohs._Run(odb))
        out = []
        r.write(blob.ptr, data, out)
        seqs[i] = out
    return seqs


def test_cfg5_set_blob_and_oracle():
    """CPU: the product's HWLM blob for the cfg-5-shaped set is the one built
    from the oracle's fragment list, and the oracle's run over a chunk equals
    the engine-free brute force"""
    exprs, flags, ids, blocks = cfg5_case(64 << 10)
    db = hs.compile_lit_multi(exprs, flags, ids, hs.MODE_BLOCK)
    odb = ohs.compile_lit_multi(exprs, flags, ids)
    lits = [vsa.HwlmLiteral(t, nc, f, noruns=nr) for t, nc, f, nr in odb.hwlm_literals()]
    blob = vsa.hwlm_build(lits)
    assert db.hwlm_bytes() == blob.tobytes()
    data = np.frombuffer(blocks[1][2], np.uint8).copy()
    got = ohs.scan(odb, blob.ptr, data)
    assert len(got) > 0
    assert sorted(got) == sorted(ohs.brute_force(odb, data))


def test_seq_digest_matches_c():
    """the Python fold of the sequence digest equals the C one (through a
    one-block corpus would need a GPU; here the formula on known values)"""
    assert hs.seq_digest([]) == 0
    a = hs.seq_digest([(1, 0, 5), (2, 3, 9)])
    b = hs.seq_digest([(2, 3, 9), (1, 0, 5)])
    assert a != b and a == hs.seq_digest([(2, 3, 9)], hs.seq_digest([(1, 0, 5)]))


def _check_sequences(g, exprs, flags, ids, blocks, mode):
    want = oracle_sequences(exprs, flags, ids, blocks, mode)
    total, counts, digests = g.scan_digests()
    # the layout's scan order (hsbench.layout) -> block index: streams
    # grouped in order of first appearance
    first = {}
    for i, (_, sid, _) in enumerate(blocks):
        first.setdefault(sid, i)
    order = list(range(len(blocks))) if mode == hs.MODE_BLOCK else \
        sorted(range(len(blocks)), key=lambda i: (first[blocks[i][1]], i))
    bad = [(i, len(want[b]), int(counts[i])) for i, b in enumerate(order)
           if int(digests[i]) != hs.seq_digest(want[b]) or int(counts[i]) != len(want[b])]
    assert not bad, "chunks whose callback sequence differs (pos, want n, got n): %s" % bad[:8]
    assert total == sum(len(w) for w in want)
    # hsbench's pipelined repeat loop (pass k + 1 scanned while pass k
    # replays): every pass the same total, the last pass's sequences equal
    rc, tot, cnt2, dg2 = g.corpus.scan_repeats(3, True, 16, True)
    assert rc == hs.SUCCESS and [int(t) for t in tot] == [total] * 3
    assert np.array_equal(cnt2, counts) and np.array_equal(dg2, digests)
    return total


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [hs.MODE_BLOCK, hs.MODE_STREAM, hs.MODE_VECTORED])
def test_cfg5_mixed_literal_db(mode):
    """cfg-5-shaped database (10k mixed literals) on 64 MiB of 16 KiB chunks:
    every chunk's full callback sequence (id, from, to) out of the one-launch
    corpus scan + host report replay equals the oracle's (an order-dependent
    digest per chunk plus the count), in block, stream and vectored mode"""
    exprs, flags, ids, blocks = cfg5_case(64 << 20)
    g = hsbench.GpuCorpus(exprs, ids, flags, blocks, mode)
    try:
        total = _check_sequences(g, exprs, flags, ids, blocks, mode)
        assert total > 10000
        t2, _ = g.scan()
        assert t2 == total
    finally:
        g.close()


@pytest.mark.gpu
def test_cfg5_small_chunks_sequences():
    """the same set on 32 MiB of 2 KiB chunks (hsbench's small-block case),
    block mode: full callback sequences per chunk"""
    exprs, flags, ids, blocks = cfg5_case(32 << 20, chunk=2 << 10)
    g = hsbench.GpuCorpus(exprs, ids, flags, blocks, hs.MODE_BLOCK)
    try:
        assert _check_sequences(g, exprs, flags, ids, blocks, hs.MODE_BLOCK) > 2000
    finally:
        g.close()


@pytest.mark.gpu
def test_block_replay_ragged_parallel(monkeypatch):
    """The parallel block-mode replay (hs_lit.cpp corpus_replay_blocks: the
    records cut into per-thread ranges at block boundaries, each thread
    mapping and replaying its own) on ragged blocks -- lengths 0 to 64 KiB,
    gaps between some, a dense planted set so >= 8 threads get records, the
    cfg-5-shaped set with shared ids (dedupe and SOM-log paths): every
    block's count and callback-sequence digest equal the unit path's
    (VSA_REPLAY_UNITS=1, the round-5 replay) and, for every block, the
    oracle's (oracle.hs_lit over its own HWLM records of that block)."""
    import bench
    exprs, flags, ids = bench.make_mixed_set(10000)
    lits = [vsa.HwlmLiteral(e, False, i) for i, e in enumerate(exprs)]
    data = bench.make_corpus(12 << 20, lits, seed=13, plant_every=128)
    rng = random.Random(5)
    offs, lens, pos = [], [], 0
    while True:
        ln = rng.choice([0, 1, 9, 100, 2048, 16384, 40000, rng.randint(1, 65536)])
        if pos + ln > len(data):
            break
        offs.append(pos)
        lens.append(ln)
        pos += ln + rng.choice([0, 0, 0, 7, 1000])
    db = hs.compile_lit_multi(exprs, flags, ids, hs.MODE_BLOCK)
    scratch = hs.Scratch(db)
    ctx = vsa.Context(0)
    d = ctx.malloc(len(data))
    try:
        ctx.h2d(d, data)
        corpus = hs.Corpus(db, scratch, d, offs, lens, h_data=data)
        try:
            rc, tot, cnt, dg = corpus.scan(True, 16, digests=True)
            assert rc == hs.SUCCESS and tot > 8 * 2048
            monkeypatch.setenv("VSA_REPLAY_UNITS", "1")
            rc2, tot2, cnt2, dg2 = corpus.scan(True, 16, digests=True)
            monkeypatch.delenv("VSA_REPLAY_UNITS")
            assert rc2 == hs.SUCCESS and tot2 == tot
            assert np.array_equal(cnt, cnt2) and np.array_equal(dg, dg2)
            rc3, tot3, cnt3, dg3 = corpus.scan(True, 1, digests=True)
            assert tot3 == tot and np.array_equal(dg3, dg)
            odb = ohs.compile_lit_multi(exprs, flags, ids)
            oblob = vsa.hwlm_build([vsa.HwlmLiteral(t, nc, f, noruns=nr)
                                    for t, nc, f, nr in odb.hwlm_literals()])
            for b, (o, ln) in enumerate(zip(offs, lens)):
                seq = ohs.scan(odb, oblob.ptr, data[o:o + ln].copy()) if ln else []
                assert (int(cnt[b]), int(dg[b])) == (len(seq), hs.seq_digest(seq)), b
        finally:
            corpus.close()
    finally:
        ctx.free(d)
        ctx.close()
        scratch.close()
        db.close()


@pytest.mark.gpu
def test_block_replay_few_large_blocks():
    """Few large blocks (the end-to-end bench's shape: 4 blocks, 4-16
    threads): the replay's thread ranges snap to the nearer block boundary,
    so every thread count gives the one-thread counts and digests; and the
    pipelined repeats on a fresh corpus -- whose first pass outgrows the
    output and rescans inside its wait, so its record copy follows the
    rescan, not the mark queued with the first launch -- give every pass the
    same total and the same per-block sequences."""
    import bench
    exprs, flags, ids = bench.make_mixed_set(2000)
    lits = [vsa.HwlmLiteral(e, False, i) for i, e in enumerate(exprs)]
    data = bench.make_corpus(16 << 20, lits, seed=17, plant_every=96)
    bl = 4 << 20
    offs, lens = [i * bl for i in range(4)], [bl, bl, bl, bl - 3]
    db = hs.compile_lit_multi(exprs, flags, ids, hs.MODE_BLOCK)
    want = None
    for threads in (1, 2, 3, 4, 5, 8, 16):
        scratch = hs.Scratch(db)
        ctx = vsa.Context(0)
        d = ctx.malloc(len(data))
        try:
            ctx.h2d(d, data)
            corpus = hs.Corpus(db, scratch, d, offs, lens, h_data=data)
            try:
                if threads in (4, 16):
                    # a fresh corpus: pass 0 rescans (> 65,536 records)
                    rc, tot, cnt, dg = corpus.scan_repeats(3, True, threads, True)
                    assert rc == hs.SUCCESS and len(set(int(t) for t in tot)) == 1
                    tot = int(tot[-1])
                else:
                    rc, tot, cnt, dg = corpus.scan(True, threads, digests=True)
                    assert rc == hs.SUCCESS
                if want is None:
                    want = (tot, cnt.copy(), dg.copy())
                    assert tot > 65536
                assert tot == want[0], threads
                assert np.array_equal(cnt, want[1]) and np.array_equal(dg, want[2]), threads
            finally:
                corpus.close()
        finally:
            ctx.free(d)
            ctx.close()
            scratch.close()
    db.close()
