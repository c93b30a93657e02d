"""TEST INFRASTRUCTURE ONLY — the CPU oracle (checker) for vectorscan_amd.

ctypes bindings for oracle/oracle.c, a scalar C restatement of the
reference runtime (see that file's header for the file:line it restates),
plus a brute-force literal matcher in numpy that depends on nothing but the
literal definitions.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package; the product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")


def build():
    os.makedirs(os.path.join(HERE, "_build"), exist_ok=True)
    subprocess.check_call(["gcc", "-O2", "-march=x86-64-v3", "-std=gnu11", "-fPIC", "-shared",
                           "-Wall", "-pthread",
                           os.path.join(HERE, "oracle.c"), "-o", LIB])


if not os.path.exists(LIB):
    build()
_lib = ctypes.CDLL(LIB)


class _Match(ctypes.Structure):
    _fields_ = [("end", ctypes.c_uint64), ("id", ctypes.c_uint32)]


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_vp, _sz, _u64, _i64, _int = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                              ctypes.c_long, ctypes.c_int)
_sig("orc_hwlm_exec", _i64, _vp, _vp, _sz, _sz, _u64, _vp, _sz, _i64, _u64,
     ctypes.POINTER(_int))
_sig("orc_fdr_exec", _i64, _vp, _vp, _sz, _sz, _u64, _vp, _sz, _i64, _u64,
     ctypes.POINTER(_int))
_sig("orc_nood_exec", _i64, _vp, _vp, _sz, _sz, _vp, _sz, _i64, ctypes.POINTER(_int))
_sig("orc_shufti", _i64, _vp, _vp, _vp, _sz)
_sig("orc_rshufti", _i64, _vp, _vp, _vp, _sz)
_sig("orc_truffle", _i64, _vp, _vp, _vp, _sz)
_sig("orc_shufti_double", _i64, _vp, _vp, _vp, _vp, _vp, _sz, _i64, _i64)
_sig("orc_rtruffle", _i64, _vp, _vp, _vp, _sz)
_sig("orc_verm", _i64, ctypes.c_uint8, _int, _int, _int, _vp, _sz)
_sig("orc_dverm", _i64, ctypes.c_uint8, ctypes.c_uint8, _int, _vp, _sz)
_sig("orc_rdverm", _i64, ctypes.c_uint8, ctypes.c_uint8, _int, _vp, _sz)
_sig("orc_dverm_masked", _i64, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8,
     ctypes.c_uint8, _vp, _sz)
_sig("orc_fdr_candidates", _u64, _vp, _vp, _sz)
_sig("orc_hwlm_exec_stream", _i64, _vp, _vp, _sz, _vp, _sz, _sz, _u64, _vp, _sz, _i64, _u64,
     ctypes.POINTER(_int))
_sig("orc_fdr_exec_stream", _i64, _vp, _vp, _sz, _vp, _sz, _sz, _u64, _vp, _sz, _i64, _u64,
     ctypes.POINTER(_int))
_sig("orc_nood_exec_stream", _i64, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _i64,
     ctypes.POINTER(_int))

ALL = (1 << 64) - 1

_sig("orc_set_vector_size", None, ctypes.c_long)


def set_vector_size(v):
    """Teddy build whose loop shape the flood restatement follows (16 SSE,
    32 AVX2, 64 AVX-512 VBMI; default 64) — vsa.set_accel_vector_size on the
    engine side."""
    _lib.orc_set_vector_size(int(v))


def _buf(data):
    if isinstance(data, np.ndarray):
        data = np.ascontiguousarray(data, np.uint8)
        return data, data.ctypes.data, data.nbytes
    data = bytes(data)
    b = ctypes.create_string_buffer(data, max(1, len(data)))
    return b, ctypes.addressof(b), len(data)


def _run(fn, ptr, data, start, extra, term_after, cap, cb_ret=ALL):
    keep, p, n = _buf(data)
    while True:
        out = (_Match * max(1, cap))()
        st = _int()
        cnt = fn(ptr, p, n, start, *extra, out, cap, term_after, *(
            [cb_ret] if fn is not _lib.orc_nood_exec else []), ctypes.byref(st))
        if cnt <= cap:
            return st.value, [(out[i].end, out[i].id) for i in range(cnt)]
        cap = cnt


def hwlm_exec(blob_ptr, data, start=0, groups=ALL, term_after=-1, cap=4096, cb_ret=ALL):
    """Reference hwlmExec callback sequence [(end, id)]: the emulated
    callback returns `cb_ret` (the new group mask), or TERMINATE once
    `term_after` matches have been reported."""
    return _run(_lib.orc_hwlm_exec, blob_ptr, data, start, [groups], term_after, cap, cb_ret)


def fdr_exec(engine_ptr, data, start=0, groups=ALL, term_after=-1, cap=4096, cb_ret=ALL):
    return _run(_lib.orc_fdr_exec, engine_ptr, data, start, [groups], term_after, cap, cb_ret)


def fdr_exec_simd(engine_ptr, data, start=0, groups=ALL, cap=1 << 16):
    """fdrExec through the SSE2 main loop (the CPU baseline engine)"""
    keep, p, n = _buf(data)
    while True:
        out = (_Match * max(1, cap))()
        st = _int()
        cnt = _lib.orc_fdr_exec_simd(engine_ptr, p, n, start, groups, out, cap, ctypes.byref(st))
        if cnt <= cap:
            return st.value, [(out[i].end, out[i].id) for i in range(cnt)]
        cap = cnt


# the 16 bytes before the end of a short history, as the reference's
# unit/internal/fdr.cpp safeExecStreaming provides them
HIST_FILLER = b"0123456789abcdef"


def history_buffer(hist, filler=HIST_FILLER):
    """(keepalive, hend address, hlen): `hist` preceded by filler so the 16
    bytes before hend are readable, as streaming callers guarantee."""
    hist = bytes(hist)
    raw = (bytes(filler) + hist) if len(hist) < 16 else hist
    b = ctypes.create_string_buffer(raw, max(1, len(raw)))
    return b, ctypes.addressof(b) + len(raw), len(hist)


def _run_stream(fn, ptr, hist, data, start, groups, term_after, cap, cb_ret, filler):
    hk, hend, hlen = history_buffer(hist, filler)
    keep, p, n = _buf(data)
    while True:
        out = (_Match * max(1, cap))()
        st = _int()
        if fn is _lib.orc_nood_exec_stream:
            cnt = fn(ptr, hend, hlen, p, n, out, cap, term_after, ctypes.byref(st))
        else:
            cnt = fn(ptr, hend, hlen, p, n, start, groups, out, cap, term_after, cb_ret,
                     ctypes.byref(st))
        if cnt <= cap:
            return st.value, [(out[i].end, out[i].id) for i in range(cnt)]
        cap = cnt


def hwlm_exec_stream(blob_ptr, hist, data, start=0, groups=ALL, term_after=-1, cap=4096,
                     cb_ret=ALL, filler=HIST_FILLER):
    """hwlmExecStreaming (hwlm.c:207) over history `hist` + `data`."""
    return _run_stream(_lib.orc_hwlm_exec_stream, blob_ptr, hist, data, start, groups,
                       term_after, cap, cb_ret, filler)


def fdr_exec_stream(engine_ptr, hist, data, start=0, groups=ALL, term_after=-1, cap=4096,
                    cb_ret=ALL, filler=HIST_FILLER):
    """fdrExecStreaming (fdr.c:827)."""
    return _run_stream(_lib.orc_fdr_exec_stream, engine_ptr, hist, data, start, groups,
                       term_after, cap, cb_ret, filler)


def nood_exec_stream(engine_ptr, hist, data, term_after=-1, cap=4096, filler=HIST_FILLER):
    """noodExecStreaming (noodle_engine.cpp:136)."""
    return _run_stream(_lib.orc_nood_exec_stream, engine_ptr, hist, data, 0, 0, term_after,
                       cap, 0, filler)


_sig("orc_fdr_exec_squash", _i64, _vp, _vp, _sz, _sz, _u64, _vp, _sz, _vp, _sz,
     ctypes.POINTER(_int))


def fdr_exec_squash(engine_ptr, data, squash, start=0, groups=ALL, cap=1 << 16):
    """fdrExec whose callback, on reporting literal id, runs a Rose
    INCLUDED_JUMP with squash mask squash[id] (program_runtime.c:2985-2997:
    *scratch->fdr_conf &= ~squash << (fdr_conf_offset & ~7)).  `squash` is a
    dict id -> u8 mask."""
    n = max(squash) + 1 if squash else 0
    tab = np.zeros(max(n, 1), np.uint8)
    for k, v in squash.items():
        tab[k] = v
    keep, p, ln = _buf(data)
    while True:
        out = (_Match * max(1, cap))()
        st = _int()
        cnt = _lib.orc_fdr_exec_squash(engine_ptr, p, ln, start, groups, out, cap,
                                       tab.ctypes.data, n, ctypes.byref(st))
        if cnt <= cap:
            return st.value, [(out[i].end, out[i].id) for i in range(cnt)]
        cap = cnt


def nood_exec(engine_ptr, data, start=0, term_after=-1, cap=4096):
    return _run(_lib.orc_nood_exec, engine_ptr, data, start, [], term_after, cap)


def shufti(lo, hi, data, reverse=False):
    keep, p, n = _buf(data)
    f = _lib.orc_rshufti if reverse else _lib.orc_shufti
    return f(bytes(lo), bytes(hi), p, n)


def shufti_double(lo1, hi1, lo2, hi2, data, vector_size=64, mis=0):
    """shuftiDoubleExec with VECTORSIZE `vector_size` on a buffer whose
    address is `mis` mod vector_size; returns the first match index or len."""
    keep, p, n = _buf(data)
    return _lib.orc_shufti_double(bytes(lo1), bytes(hi1), bytes(lo2), bytes(hi2), p, n,
                                  vector_size, mis)


def truffle(m1, m2, data, reverse=False):
    keep, p, n = _buf(data)
    f = _lib.orc_rtruffle if reverse else _lib.orc_truffle
    return f(bytes(m1), bytes(m2), p, n)


def verm(c, nocase, data, negate=False, reverse=False):
    keep, p, n = _buf(data)
    return _lib.orc_verm(c, int(nocase), int(negate), int(reverse), p, n)


def dverm(c1, c2, nocase, data):
    keep, p, n = _buf(data)
    return _lib.orc_dverm(c1, c2, int(nocase), p, n)


def rdverm(c1, c2, nocase, data):
    keep, p, n = _buf(data)
    return _lib.orc_rdverm(c1, c2, int(nocase), p, n)


def dverm_masked(c1, c2, m1, m2, data):
    keep, p, n = _buf(data)
    return _lib.orc_dverm_masked(c1, c2, m1, m2, p, n)


def fdr_candidates(engine_ptr, data):
    keep, p, n = _buf(data)
    return _lib.orc_fdr_candidates(engine_ptr, p, n)


# ------------------------------------------------------------ brute force

def _upper(b):
    return bytes(c - 0x20 if 0x61 <= c <= 0x7A else c for c in b)


def brute_force(lits, data, start=0):
    """All (end, id) occurrences of each literal fully inside `data`, ending
    at >= start: the match set any correct HWLM engine confirms (callers
    apply NOREPEAT/groups separately).  Literals: objects with s, nocase,
    id, msk, cmp (hwlm_literal.h semantics)."""
    arr = np.frombuffer(bytes(data), np.uint8)
    n = len(arr)
    out = set()
    for lit in lits:
        s = np.frombuffer(_upper(lit.s) if lit.nocase else bytes(lit.s), np.uint8)
        L = len(s)
        W = max(L, len(lit.msk))
        if n < W:
            continue
        ok = np.ones(n - W + 1, bool)  # window start positions
        for k in range(L):
            col = arr[W - L + k: n - L + k + 1]
            c = s[k]
            if lit.nocase and (0x41 <= c <= 0x5A):
                ok &= (col & 0xDF) == c
            else:
                ok &= col == c
        for k in range(len(lit.msk)):
            m, v = lit.msk[k], lit.cmp[k]
            col = arr[W - len(lit.msk) + k: n - len(lit.msk) + k + 1]
            ok &= (col & m) == (v & m)
        for w in np.nonzero(ok)[0]:
            end = int(w) + W - 1
            if end >= start:
                out.add((end, lit.id))
    return out


_sig("orc_fdr_count_mt", ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.c_int)


_sig("orc_digest_mt", ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p)

M64 = (1 << 64) - 1


_sig("orc_digest_mt2", ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p)
_sig("orc_fdr_exec_simd", _i64, _vp, _vp, _sz, _sz, _u64, _vp, _sz, ctypes.POINTER(_int))


def digest_mt(engine_ptr, data, nthreads, nood=False, simd=False):
    """(count, sum, xor) of the block scan's (end, id) match set (oracle.c
    orc_digest_mt: the restatement over `nthreads` stripes with a 7-byte
    halo; simd: the FDR main zone through the SSE2 get_conf_stride_1 port,
    the CPU baseline).  Compare with :func:`digest_of`."""
    buf = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.zeros(2, np.uint64)
    n = _lib.orc_digest_mt2(engine_ptr, int(nood), int(simd), buf.ctypes.data, len(buf),
                            int(nthreads), out.ctypes.data)
    if n < 0:
        raise RuntimeError("orc_digest_mt failed")
    return int(n), int(out[0]), int(out[1])


_sig("orc_shufti_bitmap", ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_void_p)
_sig("orc_truffle_bitmap", ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_void_p)


def class_bitmap_of_masks(kind, a, b, data):
    """(bitmap as uint64 words, member count) of every position's shufti
    (kind "shufti": lo, hi) or truffle ("truffle": m1, m2) verdict, from the
    masks (oracle.c orc_shufti_bitmap / orc_truffle_bitmap)."""
    buf = np.ascontiguousarray(data, dtype=np.uint8)
    bits = np.zeros((len(buf) + 63) // 64, np.uint64)
    ma = ctypes.create_string_buffer(bytes(a), 16)
    mb = ctypes.create_string_buffer(bytes(b), 16)
    fn = _lib.orc_shufti_bitmap if kind == "shufti" else _lib.orc_truffle_bitmap
    n = fn(ma, mb, buf.ctypes.data, len(buf), bits.ctypes.data)
    return bits, int(n)


_sig("orc_set_pin", None, ctypes.c_void_p, ctypes.c_int)


def set_pin(cpus):
    """pin the multi-threaded harness's thread t to cpus[t % len(cpus)]
    (empty: no pinning)"""
    arr = (ctypes.c_int * max(1, len(cpus)))(*cpus)
    _lib.orc_set_pin(arr, len(cpus))


_sig("orc_records_mt", ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


def records_mt(engine_ptr, data, nthreads, nood=False, cap=1 << 24):
    """(ends, ids) of the block scan in the reference's callback order
    (oracle.c orc_records_mt: `nthreads` stripes with a 7-byte halo,
    concatenated in stripe order).  Raises if more than `cap` records."""
    buf = np.ascontiguousarray(data, dtype=np.uint8)
    for _ in range(2):
        ends = np.zeros(cap, np.uint64)
        ids = np.zeros(cap, np.uint32)
        n = _lib.orc_records_mt(engine_ptr, int(nood), buf.ctypes.data, len(buf), int(nthreads),
                                ends.ctypes.data, ids.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("orc_records_mt failed")
        if n <= cap:
            return ends[:n], ids[:n]
        cap = n
    raise RuntimeError("orc_records_mt: record count changed between runs")


_sig("orc_records_blocks", ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_size_t)


def records_blocks(engine_ptr, data, block_len, nthreads, nood=False, cap=1 << 22):
    """(ends, ids, blocks) of every `block_len`-byte block of `data` scanned
    as its own call (oracle.c orc_records_blocks: hsbench's fixed-size
    chunks), in block order, each block's records in callback order, ends
    relative to their block."""
    buf = np.ascontiguousarray(data, dtype=np.uint8)
    for _ in range(2):
        ends = np.zeros(cap, np.uint64)
        ids = np.zeros(cap, np.uint32)
        blks = np.zeros(cap, np.uint32)
        n = _lib.orc_records_blocks(engine_ptr, int(nood), buf.ctypes.data, len(buf),
                                    int(block_len), int(nthreads), ends.ctypes.data,
                                    ids.ctypes.data, blks.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("orc_records_blocks failed")
        if n <= cap:
            return ends[:n], ids[:n], blks[:n]
        cap = n
    raise RuntimeError("orc_records_blocks: record count changed between runs")


def mix64(x):
    """splitmix64 finalizer over a uint64 numpy array (oracle.c orc_mix64)."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, np.uint64) + np.uint64(0x9e3779b97f4a7c15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        return z ^ (z >> np.uint64(31))


def digest_of(ends, ids):
    """(count, sum, xor) digest of an (end, id) match set, as orc_digest_mt."""
    e = np.asarray(ends, np.uint64)
    i = np.asarray(ids, np.uint64)
    m = mix64((e << np.uint64(32)) ^ i)
    with np.errstate(over="ignore"):
        s = int(np.sum(m, dtype=np.uint64)) & M64
    x = int(np.bitwise_xor.reduce(m)) if len(m) else 0
    return int(len(m)), s, x


def fdr_count_mt(engine_ptr, data, nthreads):
    """match count of the scalar fdrExec restatement over `nthreads` stripes
    (timing harness for bench.py's cpu_baseline; see oracle.c)"""
    buf = np.ascontiguousarray(data, dtype=np.uint8)
    n = _lib.orc_fdr_count_mt(engine_ptr, buf.ctypes.data, len(buf), int(nthreads))
    if n < 0:
        raise RuntimeError("orc_fdr_count_mt failed")
    return n
