"""Pure-literal database API (include/vectorscan_amd_hs.h) — the Python
mirror of the reference's hs_compile_lit_multi / hs_scan / hs_scan_vector /
stream calls (src/hs_compile.h:608-697, src/hs_runtime.h:148-609) for
databases of pure literals, over the GPU literal matcher.

Callbacks take ``(id, from, to, flags)`` and return a truthy value to stop
matching (match_event_handler, hs_runtime.h:125-128).  Every scan runs on
the GPU; there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import lib, _sig, _as_buf

SUCCESS = 0
INVALID = -1
NOMEM = -2
SCAN_TERMINATED = -3
COMPILER_ERROR = -4
DB_VERSION_ERROR = -5
DB_PLATFORM_ERROR = -6
DB_MODE_ERROR = -7
SCRATCH_IN_USE = -10
UNKNOWN_ERROR = -13

FLAG_CASELESS = 1
FLAG_DOTALL = 2
FLAG_MULTILINE = 4
FLAG_SINGLEMATCH = 8
FLAG_ALLOWEMPTY = 16
FLAG_UTF8 = 32
FLAG_UCP = 64
FLAG_PREFILTER = 128
FLAG_SOM_LEFTMOST = 256
FLAG_COMBINATION = 512
FLAG_QUIET = 1024
MODE_BLOCK = 1
MODE_STREAM = 2
MODE_VECTORED = 4
MODE_SOM_HORIZON_LARGE = 1 << 24
MODE_SOM_HORIZON_MEDIUM = 1 << 25
MODE_SOM_HORIZON_SMALL = 1 << 26


class _CompileError(ctypes.Structure):
    _fields_ = [("message", ctypes.c_char_p), ("expression", ctypes.c_int)]


EventHandler = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint, ctypes.c_ulonglong,
                                ctypes.c_ulonglong, ctypes.c_uint, ctypes.c_void_p)

_vp = ctypes.c_void_p
_sig("vsa_hs_compile_lit_multi", ctypes.c_int, _vp, _vp, _vp, _vp, ctypes.c_uint,
     ctypes.c_uint, _vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.POINTER(_CompileError)))
_sig("vsa_hs_free_compile_error", ctypes.c_int, ctypes.POINTER(_CompileError))
_sig("vsa_hs_free_database", ctypes.c_int, _vp)
_sig("vsa_hs_database_hwlm", ctypes.c_int, _vp, ctypes.POINTER(_vp),
     ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint))
_sig("vsa_hs_alloc_scratch", ctypes.c_int, _vp, ctypes.POINTER(_vp))
_sig("vsa_hs_free_scratch", ctypes.c_int, _vp)
_sig("vsa_hs_scan", ctypes.c_int, _vp, _vp, ctypes.c_uint, ctypes.c_uint, _vp, EventHandler,
     _vp)
_sig("vsa_hs_scan_vector", ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint, ctypes.c_uint, _vp,
     EventHandler, _vp)
_sig("vsa_hs_open_stream", ctypes.c_int, _vp, ctypes.c_uint, ctypes.POINTER(_vp))
_sig("vsa_hs_scan_stream", ctypes.c_int, _vp, _vp, ctypes.c_uint, ctypes.c_uint, _vp,
     EventHandler, _vp)
_sig("vsa_hs_close_stream", ctypes.c_int, _vp, _vp, EventHandler, _vp)
_sig("vsa_hs_reset_stream", ctypes.c_int, _vp, ctypes.c_uint, _vp, EventHandler, _vp)
_sig("vsa_hs_copy_stream", ctypes.c_int, ctypes.POINTER(_vp), _vp)
_sig("vsa_hs_reset_and_copy_stream", ctypes.c_int, _vp, _vp, _vp, EventHandler, _vp)
_sig("vsa_hs_stream_size", ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_size_t))
_sig("vsa_hs_clone_scratch", ctypes.c_int, _vp, ctypes.POINTER(_vp))
_sig("vsa_hs_scratch_size", ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_size_t))
_sig("vsa_hs_valid_platform", ctypes.c_int)
_sig("vsa_hs_version", ctypes.c_char_p)
_sig("vsa_hs_serialize_database", ctypes.c_int, _vp, ctypes.POINTER(_vp),
     ctypes.POINTER(ctypes.c_size_t))
_sig("vsa_hs_deserialize_database", ctypes.c_int, _vp, ctypes.c_size_t, ctypes.POINTER(_vp))
_sig("vsa_hs_serialized_database_size", ctypes.c_int, _vp, ctypes.c_size_t,
     ctypes.POINTER(ctypes.c_size_t))
_sig("vsa_hs_database_size", ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_size_t))
_sig("vsa_hs_serialized_database_info", ctypes.c_int, _vp, ctypes.c_size_t, ctypes.POINTER(_vp))
_sig("vsa_hs_database_info", ctypes.c_int, _vp, ctypes.POINTER(_vp))

_libc = ctypes.CDLL(None)
_libc.free.argtypes = [_vp]
_libc.free.restype = None


def _take_string(p):
    """a malloc'ed C string from the library, freed"""
    try:
        return ctypes.string_at(p.value).decode()
    finally:
        _libc.free(p)


class HsError(RuntimeError):
    def __init__(self, code, message="", expression=-1):
        super().__init__("hs error %d%s" % (code, (": " + message) if message else ""))
        self.code = code
        self.message = message
        self.expression = expression


class Database:
    """hs_database_t of pure literals (hs_compile_lit_multi)."""

    def __init__(self, handle, mode):
        self.handle = handle
        self.mode = mode

    def hwlm(self):
        """(address, size, fragments) of the database's HWLM blob."""
        p, n, f = _vp(), ctypes.c_size_t(), ctypes.c_uint()
        rc = lib.vsa_hs_database_hwlm(self.handle, ctypes.byref(p), ctypes.byref(n),
                                      ctypes.byref(f))
        if rc:
            raise HsError(rc)
        return p.value, n.value, f.value

    def hwlm_bytes(self):
        p, n, _ = self.hwlm()
        return ctypes.string_at(p, n)

    def serialize(self):
        """hs_serialize_database (hs_common.h:104): the reference's envelope
        around this engine's bytecode."""
        p, n = _vp(), ctypes.c_size_t()
        rc = lib.vsa_hs_serialize_database(self.handle, ctypes.byref(p), ctypes.byref(n))
        if rc:
            raise HsError(rc)
        try:
            return ctypes.string_at(p.value, n.value)
        finally:
            _libc.free(p)

    def size(self):
        """hs_database_size (hs_common.h:199)"""
        n = ctypes.c_size_t()
        rc = lib.vsa_hs_database_size(self.handle, ctypes.byref(n))
        if rc:
            raise HsError(rc)
        return n.value

    def info(self):
        """hs_database_info (hs_common.h:245): "Version: ... Mode: ..." """
        p = _vp()
        rc = lib.vsa_hs_database_info(self.handle, ctypes.byref(p))
        if rc:
            raise HsError(rc)
        return _take_string(p)

    def stream_size(self):
        """hs_stream_size (hs_common.h:183)"""
        n = ctypes.c_size_t()
        rc = lib.vsa_hs_stream_size(self.handle, ctypes.byref(n))
        if rc:
            raise HsError(rc)
        return n.value

    def close(self):
        if self.handle:
            lib.vsa_hs_free_database(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def compile_lit_multi(expressions, flags=None, ids=None, mode=MODE_BLOCK):
    """hs_compile_lit_multi (hs_compile.h:690).  Raises HsError(code,
    message, expression) as the reference reports a compile error."""
    n = len(expressions)
    bufs = [ctypes.create_string_buffer(bytes(e), max(1, len(e))) for e in expressions]
    exprs = (ctypes.c_void_p * max(1, n))(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[len(e) for e in expressions])
    fl = (ctypes.c_uint * max(1, n))(*flags) if flags is not None else None
    idv = (ctypes.c_uint * max(1, n))(*ids) if ids is not None else None
    db = _vp()
    err = ctypes.POINTER(_CompileError)()
    rc = lib.vsa_hs_compile_lit_multi(exprs, fl, idv, lens, n, mode, None, ctypes.byref(db),
                                      ctypes.byref(err))
    if rc != SUCCESS:
        msg, idx = "", -1
        if err:
            msg = err.contents.message.decode()
            idx = err.contents.expression
            lib.vsa_hs_free_compile_error(err)
        raise HsError(rc, msg, idx)
    return Database(db.value, mode)


def deserialize(data):
    """hs_deserialize_database (hs_common.h:133).  Raises HsError with the
    reference's codes (INVALID, DB_VERSION_ERROR, DB_PLATFORM_ERROR)."""
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    h = _vp()
    rc = lib.vsa_hs_deserialize_database(buf, len(data), ctypes.byref(h))
    if rc:
        raise HsError(rc)
    mode = int.from_bytes(bytes(data[32 + 12:32 + 16]), "little")
    return Database(h.value, mode)


def serialized_size(data):
    """hs_serialized_database_size (hs_common.h:226)"""
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    n = ctypes.c_size_t()
    rc = lib.vsa_hs_serialized_database_size(buf, len(data), ctypes.byref(n))
    if rc:
        raise HsError(rc)
    return n.value


def serialized_info(data):
    """hs_serialized_database_info (hs_common.h:267)"""
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    p = _vp()
    rc = lib.vsa_hs_serialized_database_info(buf, len(data), ctypes.byref(p))
    if rc:
        raise HsError(rc)
    return _take_string(p)


def valid_platform():
    """hs_valid_platform (hs_common.h:463)"""
    return lib.vsa_hs_valid_platform()


def version():
    """hs_version (hs_common.h:446)"""
    return lib.vsa_hs_version().decode()


def compile_lit(expression, flags=0, mode=MODE_BLOCK):
    """hs_compile_lit (hs_compile.h:608): id 0."""
    return compile_lit_multi([expression], [flags], [0], mode)


class Scratch:
    """hs_scratch_t: one per thread; grows to serve every database passed."""

    def __init__(self, db):
        self.handle = None
        self.grow(db)

    def grow(self, db):
        h = _vp(self.handle)
        rc = lib.vsa_hs_alloc_scratch(db.handle, ctypes.byref(h))
        if rc:
            raise HsError(rc)
        self.handle = h.value

    def clone(self):
        """hs_clone_scratch (hs_runtime.h:576): a scratch with its own GPU
        context serving the same databases"""
        h = _vp()
        rc = lib.vsa_hs_clone_scratch(self.handle, ctypes.byref(h))
        if rc:
            raise HsError(rc)
        s = Scratch.__new__(Scratch)
        s.handle = h.value
        return s

    def size(self):
        """hs_scratch_size (hs_runtime.h:593)"""
        n = ctypes.c_size_t()
        rc = lib.vsa_hs_scratch_size(self.handle, ctypes.byref(n))
        if rc:
            raise HsError(rc)
        return n.value

    def close(self):
        if self.handle:
            lib.vsa_hs_free_scratch(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _handler(on_event, out):
    def cb(id_, frm, to, flags, ctx):
        if on_event is None:
            out.append((id_, frm, to))
            return 0
        return 1 if on_event(id_, frm, to, flags) else 0
    return EventHandler(cb)


def scan(db, data, scratch, on_event=None, flags=0):
    """hs_scan (hs_runtime.h:479).  Returns (rc, [(id, from, to)]) — the list
    collects the matches when no on_event is given."""
    keep, ptr, n = _as_buf(data)
    out = []
    rc = lib.vsa_hs_scan(db.handle, ptr, n, flags, scratch.handle if scratch else None,
                         _handler(on_event, out), None)
    return rc, out


def scan_vector(db, pieces, scratch, on_event=None, flags=0):
    """hs_scan_vector (hs_runtime.h:522).  A piece of None is a NULL data
    pointer (the call returns HS_INVALID after the pieces before it)."""
    keeps, ptrs, lens = [], [], []
    for p in pieces:
        if p is None:
            ptrs.append(None)
            lens.append(0)
            continue
        k, ptr, n = _as_buf(p)
        keeps.append(k)
        ptrs.append(ptr)
        lens.append(n)
    cnt = len(pieces)
    pv = (ctypes.c_void_p * max(1, cnt))(*ptrs)
    lv = (ctypes.c_uint * max(1, cnt))(*lens)
    out = []
    rc = lib.vsa_hs_scan_vector(db.handle, pv, lv, cnt, flags,
                                scratch.handle if scratch else None, _handler(on_event, out),
                                None)
    return rc, out


class Stream:
    """hs_stream_t (hs_open_stream / hs_scan_stream / hs_close_stream /
    hs_reset_stream)."""

    def __init__(self, db, flags=0):
        h = _vp()
        rc = lib.vsa_hs_open_stream(db.handle, flags, ctypes.byref(h))
        if rc:
            raise HsError(rc)
        self.handle = h.value
        self._keep = []

    def scan(self, data, scratch, on_event=None, flags=0):
        keep, ptr, n = _as_buf(data)
        out = []
        rc = lib.vsa_hs_scan_stream(self.handle, ptr, n, flags,
                                    scratch.handle if scratch else None,
                                    _handler(on_event, out), None)
        return rc, out

    def copy(self):
        """hs_copy_stream (hs_runtime.h:291)"""
        h = _vp()
        rc = lib.vsa_hs_copy_stream(ctypes.byref(h), self.handle)
        if rc:
            raise HsError(rc)
        s = Stream.__new__(Stream)
        s.handle = h.value
        s._keep = []
        return s

    def reset_and_copy(self, src, scratch=None, on_event=None):
        """hs_reset_and_copy_stream (hs_runtime.h:324): this stream becomes a
        copy of src (both open on the same database)"""
        out = []
        h = _handler(on_event, out) if on_event else EventHandler()
        return lib.vsa_hs_reset_and_copy_stream(self.handle, src.handle,
                                                scratch.handle if scratch else None, h, None)

    def reset(self, scratch=None, on_event=None, flags=0):
        out = []
        h = _handler(on_event, out) if on_event else EventHandler()
        return lib.vsa_hs_reset_stream(self.handle, flags, scratch.handle if scratch else None,
                                       h, None)

    def close(self, scratch=None, on_event=None):
        if not self.handle:
            return SUCCESS
        out = []
        h = _handler(on_event, out) if on_event else EventHandler()
        rc = lib.vsa_hs_close_stream(self.handle, scratch.handle if scratch else None, h, None)
        if rc == SUCCESS:
            self.handle = None
        return rc


_u64p = ctypes.POINTER(ctypes.c_uint64)
_sig("vsa_hs_scan_corpus", ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32,
     _vp, _u64p, ctypes.c_uint)


def scan_corpus(db, scratch, d_data, offsets, lens, stream_ids=None, h_data=None,
                counts=False, threads=16):
    """vsa_hs_scan_corpus: hsbench's corpus loop as one launch over
    device-resident blocks.  Returns (rc, total, per-block counts or None)."""
    offs = np.ascontiguousarray(offsets, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint64)
    n = len(offs)
    sid = np.ascontiguousarray(stream_ids, np.uint32) if stream_ids is not None else None
    cnt = np.zeros(n, np.uint64) if counts else None
    hk = None
    hp = None
    if h_data is not None:
        hk, hp, _ = _as_buf(h_data)
    total = ctypes.c_uint64()
    rc = lib.vsa_hs_scan_corpus(db.handle, scratch.handle, d_data, hp, offs.ctypes.data,
                                ln.ctypes.data, sid.ctypes.data if sid is not None else None,
                                n, cnt.ctypes.data if cnt is not None else None,
                                ctypes.byref(total), threads)
    return rc, total.value, cnt


_sig("vsa_hs_corpus_prepare", ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32,
     ctypes.POINTER(_vp))
_sig("vsa_hs_corpus_scan", ctypes.c_int, _vp, _vp, _u64p, ctypes.c_uint)
_sig("vsa_hs_corpus_scan_ex", ctypes.c_int, _vp, _vp, _vp, _u64p, ctypes.c_uint)
_sig("vsa_hs_corpus_scan_repeats", ctypes.c_int, _vp, ctypes.c_uint32, _vp, _vp, _vp,
     ctypes.c_uint)
_sig("vsa_hs_corpus_free", ctypes.c_int, _vp)

_M64 = (1 << 64) - 1


def seq_digest(matches, h=0):
    """vsa_hs_seq_digest_step (vectorscan_amd_hs.h) folded over a callback
    sequence [(id, from, to)] in delivery order."""
    for i, f, t in matches:
        x = h ^ ((i * 0x9E3779B97F4A7C15) & _M64) ^ ((f * 0xC2B2AE3D27D4EB4F) & _M64) ^ \
            ((t * 0x165667B19E3779F9) & _M64)
        x ^= x >> 30
        x = (x * 0xBF58476D1CE4E5B9) & _M64
        x ^= x >> 27
        x = (x * 0x94D049BB133111EB) & _M64
        h = x ^ (x >> 31)
    return h


class Corpus:
    """vsa_hs_corpus_t: device-resident blocks prepared once (launch plan,
    stream grouping) for repeated vsa_hs_corpus_scan calls."""

    def __init__(self, db, scratch, d_data, offsets, lens, stream_ids=None, h_data=None):
        self._offs = np.ascontiguousarray(offsets, np.uint64)
        self._lens = np.ascontiguousarray(lens, np.uint64)
        self._sid = (np.ascontiguousarray(stream_ids, np.uint32)
                     if stream_ids is not None else None)
        self._hk, hp = None, None
        if h_data is not None:
            self._hk, hp, _ = _as_buf(h_data)
        self.n = len(self._offs)
        h = _vp()
        rc = lib.vsa_hs_corpus_prepare(db.handle, scratch.handle, d_data, hp,
                                       self._offs.ctypes.data, self._lens.ctypes.data,
                                       self._sid.ctypes.data if self._sid is not None else None,
                                       self.n, ctypes.byref(h))
        if rc:
            raise HsError(rc)
        self.handle = h.value
        self._db, self._scratch = db, scratch  # keep alive

    def scan(self, counts=False, threads=16, digests=False):
        """(rc, total, per-block counts or None[, per-block sequence digests
        (seq_digest of each block's callback sequence) when digests])"""
        cnt = np.zeros(self.n, np.uint64) if counts else None
        dg = np.zeros(self.n, np.uint64) if digests else None
        total = ctypes.c_uint64()
        rc = lib.vsa_hs_corpus_scan_ex(self.handle, cnt.ctypes.data if cnt is not None else None,
                                       dg.ctypes.data if dg is not None else None,
                                       ctypes.byref(total), threads)
        if digests:
            return rc, total.value, cnt, dg
        return rc, total.value, cnt

    def scan_repeats(self, repeats, counts=False, threads=16, digests=False):
        """vsa_hs_corpus_scan_repeats: `repeats` passes, pass k + 1 scanned
        while pass k replays.  (rc, per-pass totals, last pass counts or
        None, last pass digests or None)"""
        tot = np.zeros(repeats, np.uint64)
        cnt = np.zeros(self.n, np.uint64) if counts else None
        dg = np.zeros(self.n, np.uint64) if digests else None
        rc = lib.vsa_hs_corpus_scan_repeats(self.handle, repeats, tot.ctypes.data,
                                            cnt.ctypes.data if cnt is not None else None,
                                            dg.ctypes.data if dg is not None else None, threads)
        return rc, tot, cnt, dg

    def close(self):
        if self.handle:
            lib.vsa_hs_corpus_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
