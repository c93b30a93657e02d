"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's pure-literal
database path (the checker for vectorscan_amd.hs).  Only tests/ may import
this module.

compile_lit_multi restates what the reference's build makes of pure
literals:
  src/compiler/compiler.cpp:391-433 addLitExpression (flag / length / empty
      checks), :121-150 ParsedLitExpression (SINGLEMATCH + SOM rejected,
      every position of a caseless literal nocase and upper-cased:
      util/ue2string.cpp:285-291 ue2_literal::push_back);
  src/util/report_manager.cpp:212-236 registerExtReport (SINGLEMATCH must
      agree per id);
  src/rose/rose_build_matchers.cpp:700-743 addFragmentLiteral (HWLM literal =
      the last ROSE_SHORT_LITERAL_LEN_MAX = 8 bytes; :511-557 isNoRunsLiteral:
      no-runs only for short, single-match literals).
The run restates src/runtime.c:204-230 pureLiteralBlockExec (hwlmExec from 0,
real end = end + lit_offset_adjust, lit_offset_adjust = offset + 1) and
:802-831 pureLiteralStreamExec (hwlmExecStreaming with hlen =
min(offset, history required), runtime.c:78), with the Rose report program
of a literal: CHECK_LONG_LIT on the bytes before the 8-byte tail, exhaustion
(isExhausted / markAsMatched) for single-match ids, dedupe of one external
id per offset, SOM from = to - len (ng.cpp:600-604 makeSomRelativeCallback);
SOM reports of an id with several patterns are held in the SOM dedupe log
and flushed (leftmost start per id, id order) when the offset moves on or
the write ends (flushStoredSomMatches).

The HWLM scan is oracle.hwlm_exec / hwlm_exec_stream (oracle.c), over the
HWLM blob built from `hwlm_literals()` by the product's builder (the same
bytes as the database's, checked by the tests).  Same-offset order: HWLM
confirm order of fragments, then patterns in compile order.
"""
import oracle

SHORT = 8
CASELESS, SINGLEMATCH, SOM_LEFTMOST = 1, 8, 256
SUPPORTED = CASELESS | SINGLEMATCH | SOM_LEFTMOST
FLAG_ALL = 0x7ff


class CompileError(Exception):
    def __init__(self, message, expression=-1):
        super().__init__(message)
        self.message = message
        self.expression = expression


def _upper(b):
    return bytes(c - 32 if 97 <= c <= 122 else c for c in b)


class LitDb:
    def __init__(self):
        self.pats = []   # dicts: id, s, caseless, single, som, ekey
        self.frags = []  # (tail, caseless, [pattern indices])
        self.dedupe = False
        self.n_ekeys = 0

    def hwlm_literals(self):
        """[(tail, nocase, fragment id, noruns)] in fragment order."""
        out = []
        for f, (tail, nc, pl) in enumerate(self.frags):
            noruns = all(self.pats[p]["single"] and len(self.pats[p]["s"]) <= SHORT
                         for p in pl)
            out.append((tail, nc, f, noruns))
        return out

    @property
    def min_width(self):
        if not hasattr(self, "_min_width"):
            self._min_width = min(len(p["s"]) for p in self.pats)
        return self._min_width

    @property
    def history_required(self):
        if not hasattr(self, "_hist_req"):
            self._hist_req = max(len(t) for t, _, _ in self.frags) - 1
        return self._hist_req


def compile_lit_multi(expressions, flags=None, ids=None):
    db = LitDb()
    ext = {}
    ekeys = {}
    frag_of = {}
    for i, e in enumerate(expressions):
        f = flags[i] if flags is not None else 0
        pid = ids[i] if ids is not None else 0
        e = bytes(e)
        if len(e) > 16000:
            raise CompileError("Pattern length exceeds limit.", i)
        if f & ~SUPPORTED & FLAG_ALL:
            raise CompileError("Only HS_FLAG_CASELESS, HS_FLAG_SINGLEMATCH and "
                               "HS_FLAG_SOM_LEFTMOST are supported in literal API.", i)
        if not e or e[0] == 0:  # strcmp(expression, "") sees a leading NUL
            raise CompileError("Pure literal API doesn't support empty string.", i)
        if f & ~FLAG_ALL:
            raise CompileError("Unrecognised flag.", i)
        single = bool(f & SINGLEMATCH)
        if single and f & SOM_LEFTMOST:
            raise CompileError("HS_FLAG_SINGLEMATCH is not supported in combination "
                               "with HS_FLAG_SOM_LEFTMOST.", i)
        if pid in ext:
            db.dedupe = True
            if ext[pid][0] != single:
                raise CompileError("SINGLEMATCH differs for match ID %d" % pid, i)
        else:
            ext[pid] = (single, i)
        caseless = bool(f & CASELESS)
        s = _upper(e) if caseless else e
        ekey = None
        if single:
            ekey = ekeys.setdefault(pid, len(ekeys))
        p = dict(id=pid, s=s, caseless=caseless, single=single, som=bool(f & SOM_LEFTMOST),
                 ekey=ekey)
        tail = s[-SHORT:]
        key = (tail, caseless)
        if key not in frag_of:
            frag_of[key] = len(db.frags)
            db.frags.append((tail, caseless, []))
        db.frags[frag_of[key]][2].append(len(db.pats))
        db.pats.append(p)
    db.n_ekeys = len(ekeys)
    return db


class _Run:
    """Rose report program state of one scan / stream."""

    def __init__(self, db):
        self.db = db
        self.exhausted = [False] * db.n_ekeys
        # the stream's bytes as far back as any check reaches: buf holds the
        # kept tail of earlier writes plus the current write, buf_off is the
        # stream offset of buf[0], length the bytes written so far
        self.buf = b""
        self.buf_off = 0
        self.length = 0
        self.terminated = False
        self.som_log = {}  # id -> leftmost from at the current offset
        self.som_to = None
        if not hasattr(db, "_run_consts"):  # per-database, computed once
            counts = {}
            for p in db.pats:
                counts[p["id"]] = counts.get(p["id"], 0) + 1
            db._run_consts = (max(db.history_required, max(len(p["s"]) for p in db.pats)),
                              [p["som"] and counts[p["id"]] > 1 for p in db.pats])
        self.keep, self.som_dedupe = db._run_consts

    def flush(self, out, stop_after):
        """flushStoredSomMatches: leftmost start per id, in id order."""
        for i in sorted(self.som_log):
            if self.terminated:
                break
            out.append((i, self.som_log[i], self.som_to))
            if stop_after is not None and len(out) >= stop_after:
                self.terminated = True
        self.som_log = {}
        return not self.terminated

    def deliver(self, frag, to, out, at_to, stop_after):
        for pi in self.db.frags[frag][2]:
            p = self.db.pats[pi]
            s = p["s"]
            if len(s) > SHORT:
                if to < len(s):
                    continue
                seg = self.buf[to - len(s) - self.buf_off:to - SHORT - self.buf_off]
                if p["caseless"]:
                    seg = _upper(seg)
                if seg != s[:-SHORT]:
                    continue
            if p["ekey"] is not None and self.exhausted[p["ekey"]]:
                continue
            if self.som_dedupe[pi]:
                f = to - len(s)
                self.som_log[p["id"]] = min(self.som_log.get(p["id"], f), f)
                self.som_to = to
                continue
            if self.db.dedupe:
                if p["id"] in at_to:
                    continue
                at_to.add(p["id"])
            if p["ekey"] is not None:
                self.exhausted[p["ekey"]] = True
            out.append((p["id"], to - len(s) if p["som"] else 0, to))
            if stop_after is not None and len(out) >= stop_after:
                self.terminated = True
                return False
        return True

    def write(self, blob_ptr, data, out, stop_after=None, recs=None):
        """One write (pureLiteralStreamExec; offset 0 = block mode).  recs:
        the write's HWLM records [(end, fragment)] in callback order when the
        caller has them already (oracle.records_mt over a large block)."""
        off = self.length
        tail = self.buf[max(0, len(self.buf) - self.keep):]
        self.buf_off = off - len(tail)
        if recs is not None and self.keep <= SHORT:
            # given records and no pattern past the 8-byte tail: the report
            # program reads no bytes, so a large block is not copied
            n = len(data)
            self.buf = b""
            self.buf_off = off + n
        else:
            data_b = bytes(data) if not hasattr(data, "tobytes") else data.tobytes()
            n = len(data_b)
            self.buf = tail + data_b
        self.length += n
        if not n:
            return
        if recs is None and off == 0:
            _, recs = oracle.hwlm_exec(blob_ptr, data, cap=4096)
        elif recs is None:
            hl = min(off, self.db.history_required)
            hist = tail[len(tail) - hl:]
            _, recs = oracle.hwlm_exec_stream(blob_ptr, hist, data, cap=4096)
        last_to, at_to = None, set()
        for end, frag in recs:
            to = off + end + 1
            if to != last_to:
                if self.som_log and not self.flush(out, stop_after):
                    return
                last_to, at_to = to, set()
            if not self.deliver(frag, to, out, at_to, stop_after):
                return
        self.flush(out, stop_after)


def scan(db, blob_ptr, data, stop_after=None):
    """hs_scan: [(id, from, to)] in delivery order; stop_after = the
    callback returns nonzero on that many-th match."""
    out = []
    if db.min_width > len(data):
        return out
    _Run(db).write(blob_ptr, data, out, stop_after)
    return out


def scan_records(db, data, recs):
    """hs_scan of one block whose HWLM records (end, fragment) the caller
    computed (oracle.records_mt): the report program over them."""
    out = []
    if db.min_width > len(data):
        return out
    _Run(db).write(None, data, out, None, recs)
    return out


def scan_writes(db, blob_ptr, writes, stop_after=None):
    """hs_scan_vector / a stream's hs_scan_stream calls."""
    r = _Run(db)
    out = []
    for w in writes:
        if r.terminated:
            break
        r.write(blob_ptr, w, out, stop_after)
    return out


def brute_force(db, data):
    """Every occurrence of every pattern, sorted by (to, pattern order), with
    single-match patterns kept to their first `to` and one report per id per
    offset — the match set without any engine."""
    data = bytes(data)
    up = _upper(data)
    hits = []
    for pi, p in enumerate(db.pats):
        s = p["s"]
        hay = up if p["caseless"] else data
        start = hay.find(s)
        while start >= 0:
            hits.append((start + len(s), pi))
            start = hay.find(s, start + 1)
    hits.sort()
    out, seen_at, last, exhausted = {}, set(), None, set()
    for to, pi in hits:
        p = db.pats[pi]
        if to != last:
            last, seen_at = to, set()
        if p["single"] and p["id"] in exhausted:
            continue
        frm = to - len(p["s"]) if p["som"] else 0
        key = (p["id"], to)
        if key in out:  # one report per id per offset, the leftmost start
            out[key] = min(out[key], frm)
            continue
        if p["single"]:
            exhausted.add(p["id"])
        out[key] = frm
    return [(i, f, t) for (i, t), f in out.items()]
