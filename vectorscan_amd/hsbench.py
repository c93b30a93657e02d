"""hsbench-compatible driver for pure-literal signature sets on the GPU.

    python -m vectorscan_amd.hsbench -e EXPRS [-s SIGFILE | -z ID] -c CORPUS.db
        [-N | -V] [-n REPEATS] --literal-on [--per-scan] [--echo-matches] [--json]

Mirrors the reference's tools/hsbench (main.cpp): expressions are lines
``ID:/literal/flags`` (util/expressions.cpp:59-94 processLine,
util/ExpressionParser.rl:130-190 readExpression: the text between the first
and the last '/', flags [iHL] -> CASELESS / SINGLEMATCH / SOM_LEFTMOST);
with --literal-on the text is taken literally with strlen() length
(engine_hyperscan.cpp:413-446, hs_compile_lit_multi).  The corpus is a
sqlite database in the CorpusBuilder.py schema — ``chunk(id integer primary
key, stream_id integer not null, data blob not null)`` read with ``SELECT
id, stream_id, data FROM chunk ORDER BY id`` (data_corpus.cpp:72-110).
Default mode is streaming (every stream's chunks in id order are its
writes); -N block mode (every chunk one hs_scan); -V vectored.

Difference by design: the corpus is uploaded to HBM and prepared once
(vsa_hs_corpus_prepare: launch plan on the device), and every repeat (the
block loop of main.cpp:487-511, or the stream loops) runs as ONE GPU launch
over all chunks (vsa_hs_corpus_scan), instead of one hs_scan call per chunk
on a CPU thread.  The timed region of a repeat is that call (launch, device
sort, count / record replay, synchronisation); the report
lines and calc_mbps (main.cpp:705-708: bytes / (seconds * 125000)) are the
reference's, with "per core" meaning per GPU.
"""
import argparse
import json
import os
import sqlite3
import sys
import time

import numpy as np

from . import Context
from . import hs

FLAG_CHARS = {"i": hs.FLAG_CASELESS, "s": hs.FLAG_DOTALL, "m": hs.FLAG_MULTILINE,
              "H": hs.FLAG_SINGLEMATCH, "V": hs.FLAG_ALLOWEMPTY, "W": hs.FLAG_UCP,
              "8": hs.FLAG_UTF8, "P": hs.FLAG_PREFILTER, "L": hs.FLAG_SOM_LEFTMOST,
              "C": hs.FLAG_COMBINATION, "Q": hs.FLAG_QUIET, "O": 0}


class ExpressionError(ValueError):
    pass


def read_expression(text):
    """readExpression (ExpressionParser.rl:130-190): (expr, flags); extended
    parameters ``{...}`` are refused (the literal API has none)."""
    if not text or text[0] != "/":
        raise ExpressionError("Error parsing PCRE: %s" % text)
    end = text.rfind("/")
    if end <= 0:
        raise ExpressionError("Error parsing PCRE: %s" % text)
    expr = text[1:end]
    flags = 0
    rest = text[end + 1:]
    for i, c in enumerate(rest):
        if c == "{":
            raise ExpressionError("Extended parameters are not supported for pure literal "
                                  "matching API.")
        if c not in FLAG_CHARS:
            raise ExpressionError("Error parsing PCRE: %s" % text)
        flags |= FLAG_CHARS[c]
    return expr, flags


def load_expressions(path):
    """loadExpressions (util/expressions.cpp:96-188): a file or a directory
    of files of ``ID:/expr/flags`` lines; '#' comments; duplicate ids are an
    error."""
    files = []
    if os.path.isdir(path):
        for name in sorted(os.listdir(path)):
            if name.startswith(".") or name.endswith("~"):
                continue
            p = os.path.join(path, name)
            if os.path.isfile(p):
                files.append(p)
    else:
        files.append(path)
    out = {}
    for fn in files:
        with open(fn, "rb") as f:
            for num, raw in enumerate(f, 1):
                line = raw.decode("latin-1").rstrip("\n")
                if not line or line[0] == "#":
                    continue
                line = line.strip()
                colon = line.find(":")
                if colon < 0:
                    raise ExpressionError("Parse error in file %s on line %d: Could not parse "
                                          "line." % (fn, num))
                try:
                    eid = int(line[:colon])
                    if eid < 0:
                        raise ValueError
                except ValueError:
                    raise ExpressionError("Parse error in file %s on line %d: Unable to parse "
                                          "ID." % (fn, num))
                if eid in out:
                    raise ExpressionError("Parse error in file %s on line %d: Duplicate ID "
                                          "found." % (fn, num))
                out[eid] = line[colon + 1:]
    return out


def load_signatures(path):
    """loadSignatureList (util/expressions.cpp:190-215): one id per line."""
    ids = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            ids.append(int(line))
    return ids


def read_corpus(path):
    """readCorpus (data_corpus.cpp:72-110): [(id, stream_id, bytes)]."""
    if not os.path.exists(path):
        raise IOError("Unable to open database '%s'" % path)
    con = sqlite3.connect("file:%s?mode=ro" % path, uri=True)
    try:
        rows = con.execute("SELECT id, stream_id, data FROM chunk ORDER BY id;").fetchall()
    finally:
        con.close()
    if not rows:
        raise IOError("Database contains no blocks.")
    out = []
    for cid, sid, data in rows:
        if not data:
            raise IOError("Invalid blob or bytes from sqlite3.")
        out.append((int(cid), int(sid), bytes(data)))
    return out


def write_corpus(path, chunks):
    """A corpus in the CorpusBuilder.py schema (tools/hsbench/scripts/
    CorpusBuilder.py): chunks = [(stream_id, bytes)], ids assigned in order."""
    if os.path.exists(path):
        os.unlink(path)
    con = sqlite3.connect(path)
    con.execute("PRAGMA page_size = 65536")
    con.execute("CREATE TABLE chunk (id integer primary key, stream_id integer not null, "
                "data blob not null)")
    con.executemany("insert into chunk (id, stream_id, data) values (?, ?, ?)",
                    [(i, s, sqlite3.Binary(d)) for i, (s, d) in enumerate(chunks)])
    con.execute("create index chunk_stream_id_idx on chunk(stream_id)")
    con.commit()
    con.close()


def calc_mbps(seconds, nbytes):
    """main.cpp:705-708"""
    return nbytes / (seconds * 125000.0)


def layout(blocks, mode):
    """Host image of the corpus as laid out in HBM: block mode in chunk id
    order; stream / vectored mode each stream's chunks back to back (id
    order), so each chunk's history precedes it.  Returns (image, offsets,
    lens, stream_ids) in scan order."""
    if mode == hs.MODE_BLOCK:
        order = list(range(len(blocks)))
    else:
        first = {}
        for i, (_, sid, _) in enumerate(blocks):
            first.setdefault(sid, i)
        order = sorted(range(len(blocks)), key=lambda i: (first[blocks[i][1]], i))
    lens = np.array([len(blocks[i][2]) for i in order], np.uint64)
    offs = np.zeros(len(order), np.uint64)
    if len(order) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    image = np.frombuffer(b"".join(blocks[i][2] for i in order), np.uint8)
    sids = np.array([blocks[i][1] for i in order], np.uint32)
    return image, offs, lens, sids


class GpuCorpus:
    """The corpus resident in HBM plus the compiled database and scratch."""

    def __init__(self, exprs, ids, flags, blocks, mode):
        self.mode = mode
        full_mode = mode | (hs.MODE_SOM_HORIZON_LARGE if mode == hs.MODE_STREAM else 0)
        t0 = time.perf_counter()
        self.db = hs.compile_lit_multi(exprs, flags, ids, full_mode)
        self.compile_secs = time.perf_counter() - t0
        self.scratch = hs.Scratch(self.db)
        self.image, self.offs, self.lens, self.sids = layout(blocks, mode)
        self.ctx = Context(int(os.environ.get("VSA_DEVICE", "0")))
        self.d_data = self.ctx.malloc(max(1, self.image.nbytes))
        self.ctx.h2d(self.d_data, self.image)
        self.long = any(len(e) > 8 for e in exprs)
        self.corpus = hs.Corpus(self.db, self.scratch, self.d_data, self.offs, self.lens,
                                self.sids if mode != hs.MODE_BLOCK else None,
                                self.image if self.long else None)

    def scan(self, counts=False, threads=16):
        rc, total, cnt = self.corpus.scan(counts, threads)
        if rc != hs.SUCCESS:
            raise hs.HsError(rc)
        return total, cnt

    def scan_digests(self, threads=16):
        """(total, per-block counts, per-block callback-sequence digests,
        hs.seq_digest) of one corpus scan"""
        rc, total, cnt, dg = self.corpus.scan(True, threads, digests=True)
        if rc != hs.SUCCESS:
            raise hs.HsError(rc)
        return total, cnt, dg

    def scan_repeats(self, repeats, threads=16):
        """per-pass totals of `repeats` pipelined passes (pass k + 1 on the
        GPU while pass k replays on the host)"""
        rc, tot, _, _ = self.corpus.scan_repeats(repeats, False, threads)
        if rc != hs.SUCCESS:
            raise hs.HsError(rc)
        return [int(t) for t in tot]

    def close(self):
        self.corpus.close()
        if self.d_data:
            self.ctx.free(self.d_data)
            self.d_data = None
        self.scratch.close()
        self.db.close()


def build_set(expr_map, sig_ids=None):
    """limitToSignatures + the literal compile inputs, in id order
    (ExpressionMap is an ordered map)."""
    items = sorted(expr_map.items())
    if sig_ids is not None:
        want = set(sig_ids)
        missing = want - set(expr_map)
        if missing:
            raise ExpressionError("Signature %d is not in the expression set" % min(missing))
        items = [kv for kv in items if kv[0] in want]
    exprs, ids, flags = [], [], []
    for eid, text in items:
        e, f = read_expression(text)
        exprs.append(e.encode("latin-1"))
        ids.append(eid)
        flags.append(f)
    return exprs, ids, flags


def main(argv=None):
    ap = argparse.ArgumentParser(prog="hsbench (vectorscan_amd)")
    ap.add_argument("-e", dest="exprs", required=True, help="expression file or directory")
    ap.add_argument("-s", dest="sigfile", help="signature id list")
    ap.add_argument("-z", dest="sigid", type=int, help="single signature id")
    ap.add_argument("-c", dest="corpus", required=True, help="corpus (sqlite)")
    ap.add_argument("-n", dest="repeats", type=int, default=20)
    ap.add_argument("-N", dest="block", action="store_true", help="block mode")
    ap.add_argument("-V", dest="vectored", action="store_true", help="vectored mode")
    ap.add_argument("-T", dest="threads", default=None,
                    help="accepted for compatibility; the GPU is the engine")
    ap.add_argument("--literal-on", action="store_true")
    ap.add_argument("--per-scan", action="store_true")
    ap.add_argument("--echo-matches", action="store_true")
    ap.add_argument("--json", action="store_true", help="also print a JSON summary line")
    ap.add_argument("--replay-threads", type=int, default=16)
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one pass at a time (per-pass times); the default overlaps "
                         "pass k + 1's GPU scan with pass k's host replay")
    a = ap.parse_args(argv)
    if not a.literal_on:
        print("Error: only pure literal signature sets are supported (--literal-on)")
        return 1
    if a.repeats <= 0:
        print("Error: Couldn't parse argument to -n flag, should be a positive integer.")
        return 1
    mode = hs.MODE_BLOCK if a.block else (hs.MODE_VECTORED if a.vectored else hs.MODE_STREAM)
    expr_map = load_expressions(a.exprs)
    sig_ids = None
    sig_name = "all"
    if a.sigfile:
        sig_ids, sig_name = load_signatures(a.sigfile), a.sigfile
    elif a.sigid is not None:
        sig_ids, sig_name = [a.sigid], "-z %d" % a.sigid
    exprs, ids, flags = build_set(expr_map, sig_ids)
    try:
        blocks = read_corpus(a.corpus)
    except IOError as e:
        print("Corpus data error: %s" % e)
        return 1
    try:
        g = GpuCorpus(exprs, ids, flags, blocks, mode)
    except hs.HsError as e:
        if e.expression >= 0:
            print("Compile error for signature #%d: %s" % (e.expression, e.message))
        else:
            print("Compile error: %s" % e.message)
        return 1
    _, blob_size, nfrag = g.db.hwlm()
    print("Signatures:        %s" % sig_name)
    print("Hyperscan info:    vectorscan_amd pure-literal GPU engine (%d fragments)" % nfrag)
    print("Expression count:  {:,}".format(len(exprs)))
    print("Bytecode size:     {:,} bytes".format(blob_size))
    print("Compile time:      %0.3f seconds" % g.compile_secs)
    print()
    if a.echo_matches:
        # the per-match echo runs the API path (one hs_scan / stream per unit)
        echo(g, blocks, mode)
    # warm-up: first-launch costs and the GPU clock ramp (tens of launches
    # after idle, profiles/r03_ramp.jsonl) outside the timed loop
    t_w = time.perf_counter()
    for i in range(200):
        g.scan()
        if i >= 7 and time.perf_counter() - t_w > 0.25:
            break
    secs, totals = [], []
    pipelined = not (a.no_pipeline or a.per_scan)
    t_all = time.perf_counter()
    if pipelined:
        # passes overlap, so a pass has no time of its own: each is the mean
        totals = g.scan_repeats(a.repeats, a.replay_threads)
        secs = [(time.perf_counter() - t_all) / a.repeats] * a.repeats
    else:
        for _ in range(a.repeats):
            t0 = time.perf_counter()
            total, _ = g.scan(threads=a.replay_threads)
            secs.append(time.perf_counter() - t0)
            totals.append(total)
    total_secs = time.perf_counter() - t_all
    nbytes = int(g.lens.sum())
    nstreams = len(set(b[1] for b in blocks))
    if len(set(totals)) != 1:
        print("\nWARNING: PER-SCAN MATCH COUNTS ARE INCONSISTENT!\n")
    print("Time spent scanning:       %0.3f seconds" % total_secs)
    kind = {hs.MODE_STREAM: "(%s blocks in %s streams)" % (format(len(blocks), ","),
                                                           format(nstreams, ",")),
            hs.MODE_VECTORED: "(%s blocks in %s vectors)" % (format(len(blocks), ","),
                                                             format(nstreams, ",")),
            hs.MODE_BLOCK: "(%s blocks)" % format(len(blocks), ",")}[mode]
    print("Corpus size:               {:,} bytes {}".format(nbytes, kind))
    rate = totals[0] * 1024.0 / nbytes
    print("Matches per iteration:     {:,} ({:0.3f} matches/kilobyte)".format(totals[0], rate))
    print("Overall block rate:        {:,.2f} blocks/sec".format(
        len(blocks) * a.repeats / total_secs))
    print("Mean throughput (overall): {:,.2f} Mbit/sec".format(
        calc_mbps(total_secs, nbytes * a.repeats)))
    print("Max throughput (per GPU):  {:,.2f} Mbit/sec".format(calc_mbps(min(secs), nbytes)))
    print()
    if a.per_scan:
        for j, s in enumerate(secs):
            print("T  0 Scan %2d: %0.2f Mbit/sec" % (j, calc_mbps(s, nbytes)))
    if a.json:
        print(json.dumps({"mode": {1: "block", 2: "streaming", 4: "vectored"}[mode],
                          "expressions": len(exprs), "corpus_bytes": nbytes,
                          "blocks": len(blocks), "streams": nstreams,
                          "matches": totals[0], "repeats": a.repeats,
                          "mean_mbps": calc_mbps(total_secs, nbytes * a.repeats),
                          "max_mbps": calc_mbps(min(secs), nbytes),
                          "best_ms": min(secs) * 1e3, "pipelined": pipelined}))
    g.close()
    return 0


def echo(g, blocks, mode):
    """--echo-matches (engine_hyperscan.cpp:103-115): every match through
    the callback API, per block (block mode) or per stream."""
    db, scratch = g.db, g.scratch
    if mode == hs.MODE_BLOCK:
        for cid, _, data in blocks:
            _, seq = hs.scan(db, data, scratch)
            for i, _, to in seq:
                print("Match @%u:%u for %u" % (cid, to, i))
        return
    streams = {}
    for cid, sid, data in blocks:
        streams.setdefault(sid, []).append((cid, data))
    for sid, parts in streams.items():
        datas = [d for _, d in parts]
        if mode == hs.MODE_VECTORED:
            _, seq = hs.scan_vector(db, datas, scratch)
            for i, _, to in seq:
                print("Match @%u:%u for %u" % (sid, to, i))
            continue
        st = hs.Stream(db)
        for cid, d in parts:  # streaming: "@stream:block:to"
            for i, _, to in st.scan(d, scratch)[1]:
                print("Match @%u:%u:%u for %u" % (sid, cid, to, i))
        st.close(scratch, lambda *x: 0)


if __name__ == "__main__":
    sys.exit(main())
