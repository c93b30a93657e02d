"""vectorscan_amd — MI355X engine for Vectorscan's literal / char-class
prefilter hot path.

Python mirror of the reference interface for this path, over the C ABI of
``libvectorscan_amd.so`` (include/vectorscan_amd.h):

* :class:`HwlmLiteral` / :func:`hwlm_build`  — hwlmLiteral + hwlmBuild
  (src/hwlm/hwlm_literal.h:51, src/hwlm/hwlm_build.cpp:120-214)
* :func:`hwlm_exec`, :func:`fdr_exec`, :func:`nood_exec` — hwlmExec /
  fdrExec / noodExec with a Python callback ``cb(end, id) -> groups``
  (src/hwlm/hwlm.h:116, src/fdr/fdr.h:58, src/hwlm/noodle_engine.h:47)
* :func:`shufti_exec` … :func:`vermicelli_double_exec` — the accel
  find-first/last entry points (src/nfa/shufti.h, truffle.h, vermicelli.hpp)
* :class:`Context` / :class:`Database` — the device batch API (many blocks
  per launch, device-resident corpora, sorted match records).

There is no CPU fallback: every scan runs on the GPU through the HIP
library, and importing this package fails loudly if the library is absent.
"""
import ctypes
import os

import numpy as np

__all__ = [
    "HWLM_SUCCESS", "HWLM_TERMINATED", "HWLM_ERROR_UNKNOWN",
    "HWLM_ALL_GROUPS", "HWLM_CONTINUE_MATCHING", "HWLM_TERMINATE_MATCHING",
    "HwlmLiteral", "hwlm_build", "hwlm_exec", "fdr_exec", "nood_exec",
    "engine_blob", "shufti_exec", "rshufti_exec", "truffle_exec",
    "rtruffle_exec", "vermicelli_exec", "nvermicelli_exec",
    "rvermicelli_exec", "rnvermicelli_exec", "vermicelli_double_exec",
    "vermicelli_double_masked_exec", "shufti_build_masks",
    "truffle_build_masks", "Context", "Database", "lib", "LIB_PATH",
]

HWLM_SUCCESS = 0
HWLM_TERMINATED = 1
HWLM_ERROR_UNKNOWN = 2
HWLM_ALL_GROUPS = (1 << 64) - 1
HWLM_CONTINUE_MATCHING = HWLM_ALL_GROUPS
HWLM_TERMINATE_MATCHING = 0

ENGINE_NOOD = 16
HWLM_HEADER = 192  # ROUNDUP_CL(sizeof(struct HWLM))

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        os.environ.get("VSA_LIB_VARIANT", "libvectorscan_amd.so"))
if not os.path.exists(LIB_PATH):
    raise ImportError(
        "vectorscan_amd: %s is missing — build it with `make` (or "
        "__graft_entry__.build()); there is no CPU fallback" % LIB_PATH)
lib = ctypes.CDLL(LIB_PATH)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
HWLMCallback = ctypes.CFUNCTYPE(ctypes.c_uint64, ctypes.c_size_t,
                                ctypes.c_uint32, ctypes.c_void_p)


class _Literal(ctypes.Structure):
    _fields_ = [("s", ctypes.c_void_p), ("len", ctypes.c_uint32),
                ("id", ctypes.c_uint32), ("nocase", ctypes.c_uint8),
                ("noruns", ctypes.c_uint8), ("msk_len", ctypes.c_uint8),
                ("pad", ctypes.c_uint8), ("groups", ctypes.c_uint64),
                ("msk", ctypes.c_void_p), ("cmp", ctypes.c_void_p)]


class _BuildOpts(ctypes.Structure):
    _fields_ = [("engine_hint", ctypes.c_int32), ("allow_noodle", ctypes.c_uint8),
                ("allow_teddy", ctypes.c_uint8),
                ("allow_fat_teddy", ctypes.c_uint8),
                ("allow_flood", ctypes.c_uint8)]


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("vsa_hwlm_build", ctypes.c_int, ctypes.POINTER(_Literal), ctypes.c_size_t,
     ctypes.POINTER(_BuildOpts), ctypes.POINTER(ctypes.c_void_p),
     ctypes.POINTER(ctypes.c_size_t))
_sig("vsa_blob_free", None, ctypes.c_void_p)
_sig("vsa_hwlm_set_accel", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_uint64)
_sig("hwlmExec", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.c_size_t, HWLMCallback, ctypes.c_void_p, ctypes.c_uint64)
_sig("fdrExec", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.c_size_t, HWLMCallback, ctypes.c_void_p, ctypes.c_uint64)
_sig("noodExec", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.c_size_t, HWLMCallback, ctypes.c_void_p)
_sig("hwlmExecStreaming", ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
     HWLMCallback, ctypes.c_void_p, ctypes.c_uint64)
_sig("fdrExecStreaming", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, HWLMCallback, ctypes.c_void_p,
     ctypes.c_uint64)
_sig("noodExecStreaming", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.c_void_p, ctypes.c_size_t, HWLMCallback, ctypes.c_void_p)
_sig("vsa_get_scratch_core_info", None, ctypes.POINTER(ctypes.c_long),
     ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long))
_sig("vsa_shufti_find", ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)
_sig("vsa_shufti_double_find", ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_sig("vsa_set_accel_vector_size", None, ctypes.c_uint32)
_sig("vsa_shufti_build_double_masks", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)
_sig("vsa_truffle_find", ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)
_sig("vsa_verm_find", ctypes.c_int64, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint8,
     ctypes.c_uint8, ctypes.c_uint8, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t)
_sig("vsa_shufti_build_masks", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p)
_sig("vsa_truffle_build_masks", None, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p)
_sig("vsa_device_count", ctypes.c_int)
_sig("vsa_ctx_create", ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_ctx_destroy", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_ctx_create_shared", ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_ctx_stream", ctypes.c_void_p, ctypes.c_void_p)
_sig("vsa_db_load", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_db_free", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_db_engine", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_malloc", ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
     ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_free", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
_sig("vsa_memcpy_h2d", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_size_t)
_sig("vsa_memcpy_d2h", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_size_t)
_sig("vsa_sync", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_scan_blocks", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, _u64p, _u64p, ctypes.c_void_p, ctypes.c_uint32,
     ctypes.c_uint32, _u64p)
_sig("vsa_scan_blocks_ex", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, _u64p, _u64p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
     ctypes.c_uint32, _u64p)
_sig("vsa_scan_blocks_stream", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, _u64p, _u64p, ctypes.c_void_p, _u64p, ctypes.c_uint32,
     ctypes.c_uint32, _u64p)
_sig("vsa_plan_create", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
     ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_plan_free", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_plan_rebuilds", ctypes.c_uint32, ctypes.c_void_p)
_sig("vsa_scan_plan", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_uint32, _u64p)
_sig("vsa_scan_wait", ctypes.c_int, ctypes.c_void_p, _u64p)
_sig("vsa_scan_pack", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
_sig("vsa_scan_plan_pack", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_uint64)
_sig("vsa_scan_results", ctypes.c_int, ctypes.c_void_p,
     ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_scan_copy", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_uint64, _u64p)
_sig("vsa_scan_copy_device", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_uint64, _u64p)
_sig("vsa_scan_candidates", ctypes.c_uint64, ctypes.c_void_p)
_sig("vsa_scan_debug_counters", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
_sig("vsa_derive_first_stage", ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
     ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32))
_sig("vsa_scan_kernel_ms", ctypes.c_double, ctypes.c_void_p)
_sig("vsa_scan_launches", ctypes.c_uint64, ctypes.c_void_p)
_sig("vsa_scan_last_fused", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_scan_last_dyn", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_ctx_set_dyn_shares", ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64)
_sig("vsa_ctx_set_fused_finish", ctypes.c_int, ctypes.c_void_p, ctypes.c_int)
_sig("vsa_ctx_set_timing", ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32)
_sig("vsa_ctx_set_reserved_cus", ctypes.c_int, ctypes.c_void_p, ctypes.c_int)
_sig("vsa_read_ceiling", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
     ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), _u64p)
_sig("vsa_class_scan", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, _u64p,
     _u64p, _u64p, ctypes.c_uint32)
_sig("vsa_class_scan_masks", ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, _u64p, _u64p, _u64p)
_sig("vsa_version", ctypes.c_char_p)
_sig("vsa_set_scratch_layout", None, ctypes.c_long, ctypes.c_long)
_sig("vsa_get_scratch_layout", None, ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long))
_sig("vsa_last_error", ctypes.c_int)


class HwlmLiteral:
    """hwlmLiteral (src/hwlm/hwlm_literal.h:51-130).

    ``msk``/``cmp`` are bytes in memory order, aligned to the end of ``s``.
    Normalisation (upper-casing nocase literals, zapping an all-zero msk)
    happens in the C builder exactly as hwlm_literal.cpp:85-117.
    """

    def __init__(self, s, nocase=False, id=0, noruns=False,
                 groups=HWLM_ALL_GROUPS, msk=b"", cmp=b""):
        if isinstance(s, str):
            s = s.encode("latin-1")
        self.s = bytes(s)
        self.nocase = bool(nocase)
        self.id = int(id)
        self.noruns = bool(noruns)
        self.groups = int(groups)
        self.msk = bytes(msk)
        self.cmp = bytes(cmp)

    def __repr__(self):
        return "HwlmLiteral(%r, nocase=%s, id=%d)" % (self.s, self.nocase, self.id)


class Blob:
    """An HWLM bytecode blob (reference layout) owned by the C library."""

    def __init__(self, ptr, size, owned=True):
        self.ptr = ptr
        self.size = size
        self.owned = owned  # False: a view of memory the caller owns

    def tobytes(self):
        return ctypes.string_at(self.ptr, self.size)

    @property
    def type(self):
        return ctypes.string_at(self.ptr, 1)[0]

    @property
    def is_noodle(self):
        return self.type == ENGINE_NOOD

    @property
    def engine_id(self):
        """FDR/Teddy engine id (fdr.c:776-796); None for a noodle table."""
        if self.is_noodle:
            return None
        return int(np.frombuffer(ctypes.string_at(self.ptr + HWLM_HEADER, 4), np.uint32)[0])

    def set_accel(self, accel0=None, accel1=None, accel1_groups=0):
        """Set HWLM.accel0/accel1 (80-byte AccelAux images, accel.h:72)."""
        a0 = ctypes.create_string_buffer(bytes(accel0), 80) if accel0 else None
        a1 = ctypes.create_string_buffer(bytes(accel1), 80) if accel1 else None
        _check(lib.vsa_hwlm_set_accel(self.ptr, a0, a1, accel1_groups))

    def __del__(self):
        # lib is None once the interpreter is tearing the module down
        if getattr(self, "ptr", None) and getattr(self, "owned", True) and lib is not None:
            lib.vsa_blob_free(self.ptr)
        self.ptr = None


class BuildError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise BuildError("vectorscan_amd call failed with %d" % rc)


def hwlm_build(lits, engine_hint=-1, allow_noodle=True, allow_teddy=True,
               allow_fat_teddy=True, allow_flood=True):
    """hwlmBuildProto + hwlmBuild (hwlm_build.cpp:120-214).

    ``engine_hint`` mirrors fdrBuildProtoHinted (fdr_compile.cpp:899-910):
    0 forces FDR (domain 9, stride 1), 3..18 a Teddy engine id.
    ``allow_flood`` is Grey::fdrAllowFlood (default on, grey.cpp:68): off,
    every flood record carries idCount = FDR_FLOOD_MAX_IDS and never fires
    (flood_compile.cpp:191-195).
    Returns a :class:`Blob`; raises :class:`BuildError` when the literal set
    cannot be built with the requested engine.
    """
    arr = (_Literal * len(lits))()
    keep = []
    for i, l in enumerate(lits):
        sb = ctypes.create_string_buffer(l.s, len(l.s))
        mb = ctypes.create_string_buffer(l.msk, max(1, len(l.msk)))
        cb = ctypes.create_string_buffer(l.cmp, max(1, len(l.cmp)))
        keep += [sb, mb, cb]
        arr[i].s = ctypes.cast(sb, ctypes.c_void_p)
        arr[i].len = len(l.s)
        arr[i].id = l.id
        arr[i].nocase = int(l.nocase)
        arr[i].noruns = int(l.noruns)
        arr[i].msk_len = len(l.msk)
        arr[i].groups = l.groups
        arr[i].msk = ctypes.cast(mb, ctypes.c_void_p)
        arr[i].cmp = ctypes.cast(cb, ctypes.c_void_p)
    opts = _BuildOpts(engine_hint, int(allow_noodle), int(allow_teddy),
                      int(allow_fat_teddy), int(allow_flood))
    out = ctypes.c_void_p()
    size = ctypes.c_size_t()
    rc = lib.vsa_hwlm_build(arr, len(lits), ctypes.byref(opts), ctypes.byref(out),
                            ctypes.byref(size))
    if rc != 0:
        raise BuildError("hwlm_build failed (%d)" % rc)
    return Blob(out.value, size.value)


def derive_first_stage(blob):
    """(table u64 array, key_bits, field_bits) the engine derives from an FDR
    or Teddy blob's confirm records (host only; see vsa_derive_first_stage)"""
    cap = 1 << 14
    out = np.zeros(cap, np.uint64)
    kb, fb = ctypes.c_uint32(0), ctypes.c_uint32(0)
    n = lib.vsa_derive_first_stage(blob.ptr, blob.size, out.ctypes.data, cap, ctypes.byref(kb),
                                   ctypes.byref(fb))
    if n < 0:
        raise BuildError("vsa_derive_first_stage failed with %d" % n)
    return out[:n], kb.value, fb.value


_sig("vsa_derive_fdr4_table", ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
     ctypes.c_void_p, ctypes.c_uint32)


def derive_fdr4_table(blob, bits=15):
    """the 4-field FDR first stage (u32 array of 2^bits entries) the engine
    scans with (host only; see vsa_derive_fdr4_table)"""
    cap = 1 << bits
    out = np.zeros(cap, np.uint32)
    n = lib.vsa_derive_fdr4_table(blob.ptr, blob.size, bits, out.ctypes.data, cap)
    if n < 0:
        raise BuildError("vsa_derive_fdr4_table failed with %d" % n)
    return out[:n]


_sig("vsa_derive_fdr4_pass", ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
     ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double))
_sig("vsa_db_split", ctypes.c_int, ctypes.c_void_p)


def derive_fdr4_pass(blob, par=-1):
    """(table, estimated text candidate rate) of one split pass (par 0 / 1)
    or of the one-pass table (par -1), 15-bit keys (host only; see
    vsa_derive_fdr4_pass)"""
    cap = 1 << 15
    out = np.zeros(cap, np.uint32)
    rate = ctypes.c_double()
    n = lib.vsa_derive_fdr4_pass(blob.ptr, blob.size, par, out.ctypes.data, cap,
                                 ctypes.byref(rate))
    if n < 0:
        raise BuildError("vsa_derive_fdr4_pass failed with %d" % n)
    return out[:n], rate.value


def engine_blob(blob):
    """Pointer to the engine inside an HWLM blob (HWLM_C_DATA, hwlm_internal.h:56)."""
    return blob.ptr + HWLM_HEADER


def _as_buf(data):
    if isinstance(data, np.ndarray):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        return data, data.ctypes.data, data.nbytes
    data = bytes(data)
    b = ctypes.create_string_buffer(data, max(1, len(data)))
    return b, ctypes.addressof(b), len(data)


def _runner(fn, cb, *head):
    matches = []

    def c_cb(end, id_, scratch):
        if cb is None:
            matches.append((end, id_))
            return HWLM_CONTINUE_MATCHING
        r = cb(end, id_)
        return HWLM_CONTINUE_MATCHING if r is None else int(r) & HWLM_ALL_GROUPS

    ccb = HWLMCallback(c_cb)
    return ccb, matches


def hwlm_exec(blob, data, start=0, cb=None, groups=HWLM_ALL_GROUPS, scratch=None):
    """hwlmExec (hwlm.h:116).  ``cb(end, id)`` returns the new group mask
    (None = continue).  Without ``cb`` returns ``(status, [(end, id), ...])``."""
    keep, ptr, n = _as_buf(data)
    ccb, matches = _runner(None, cb)
    rc = lib.hwlmExec(blob.ptr, ptr, n, start, ccb, scratch, groups)
    return rc if cb is not None else (rc, matches)


_sig("vsa_hwlm_register", ctypes.c_int, ctypes.c_void_p, ctypes.c_int)
_sig("vsa_hwlm_unregister", ctypes.c_int, ctypes.c_void_p)


def hwlm_register(blob, bare_type=-1):
    """vsa_hwlm_register: the drop-ins serve this (immutable) blob without
    comparing it with their cached device copy on every call"""
    _check(lib.vsa_hwlm_register(blob.ptr, bare_type))


def hwlm_unregister(blob):
    _check(lib.vsa_hwlm_unregister(blob.ptr))


_sig("vsa_batcher_create", ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
     ctypes.POINTER(ctypes.c_void_p))
_sig("vsa_batcher_destroy", ctypes.c_int, ctypes.c_void_p)
_sig("vsa_batcher_stats", ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
     ctypes.POINTER(ctypes.c_uint64))
_sig("vsa_batcher_hwlmExec", ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_size_t, ctypes.c_size_t, HWLMCallback, ctypes.c_void_p, ctypes.c_uint64)


class Batcher:
    """vsa_batcher: concurrent hwlmExec calls from many threads share
    launches (a worker with its own GPU context scans the calls queued
    within ``window_us`` as one batch; each caller's callback runs on its
    own thread)."""

    def __init__(self, device=0, max_batch=256, window_us=20):
        self.ptr = ctypes.c_void_p()
        _check(lib.vsa_batcher_create(device, max_batch, window_us, ctypes.byref(self.ptr)))

    def hwlm_exec(self, blob, data, start=0, cb=None, groups=HWLM_ALL_GROUPS, scratch=None):
        """as hwlm_exec, through the batcher"""
        keep, ptr, n = _as_buf(data)
        ccb, matches = _runner(None, cb)
        rc = lib.vsa_batcher_hwlmExec(self.ptr, blob.ptr, ptr, n, start, ccb, scratch, groups)
        return rc if cb is not None else (rc, matches)

    def stats(self):
        """(launches, calls served)"""
        b, c = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.vsa_batcher_stats(self.ptr, ctypes.byref(b), ctypes.byref(c)))
        return b.value, c.value

    def close(self):
        if self.ptr:
            lib.vsa_batcher_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fdr_exec(blob, data, start=0, cb=None, groups=HWLM_ALL_GROUPS, scratch=None):
    """fdrExec (fdr.h:58) on the FDR/Teddy engine inside an HWLM blob."""
    keep, ptr, n = _as_buf(data)
    ccb, matches = _runner(None, cb)
    rc = lib.fdrExec(engine_blob(blob), ptr, n, start, ccb, scratch, groups)
    return rc if cb is not None else (rc, matches)


def nood_exec(blob, data, start=0, cb=None, scratch=None):
    """noodExec (noodle_engine.h:47) on the noodle table inside an HWLM blob."""
    keep, ptr, n = _as_buf(data)
    ccb, matches = _runner(None, cb)
    rc = lib.noodExec(engine_blob(blob), ptr, n, start, ccb, scratch)
    return rc if cb is not None else (rc, matches)


ACCEL_TYPES = {"none": 0, "verm": 1, "verm_nocase": 2, "dverm": 3, "dverm_nocase": 4,
               "shufti": 13, "truffle": 15}


def accel_aux(kind, offset=0, c=0, c2=0, masks=None):
    """An 80-byte union AccelAux image (accel.h:72-124) of the kinds an HWLM
    header carries (hwlm.c:48-80): verm / dverm take chars c (, c2); shufti
    and truffle take their two 16-byte masks."""
    b = bytearray(80)
    b[0] = ACCEL_TYPES[kind]
    b[1] = offset
    if kind.startswith("verm"):
        b[2] = c
    elif kind.startswith("dverm"):
        b[2], b[3] = c, c2
    elif kind in ("shufti", "truffle"):
        m1, m2 = masks
        b[16:32] = bytes(m1)
        b[32:48] = bytes(m2)
    return bytes(b)


def _history(hist, filler):
    """(keepalive, start address, hlen) of a history buffer with at least 16
    readable bytes before its end (fdr.c:835-841): short histories are
    preceded by `filler`."""
    hist = bytes(hist)
    pad = bytes(filler)[:16].rjust(16, b"\0") if len(hist) < 16 else b""
    raw = pad + hist
    b = ctypes.create_string_buffer(raw, max(1, len(raw)))
    return b, ctypes.addressof(b) + len(pad), len(hist)


def fdr_exec_stream(blob, hist, data, start=0, cb=None, groups=HWLM_ALL_GROUPS,
                    scratch=None, filler=b""):
    """fdrExecStreaming (fdr.h:75): matches of `data` whose literal may begin
    inside `hist`; ends are relative to `data`."""
    hk, hptr, hlen = _history(hist, filler)
    keep, ptr, n = _as_buf(data)
    ccb, matches = _runner(None, cb)
    rc = lib.fdrExecStreaming(engine_blob(blob), hptr if hlen else None, hlen, ptr, n, start,
                              ccb, scratch, groups)
    return rc if cb is not None else (rc, matches)


def nood_exec_stream(blob, hist, data, cb=None, scratch=None, filler=b""):
    """noodExecStreaming (noodle_engine.h:52)."""
    hk, hptr, hlen = _history(hist, filler)
    keep, ptr, n = _as_buf(data)
    ccb, matches = _runner(None, cb)
    rc = lib.noodExecStreaming(engine_blob(blob), hptr if hlen else None, hlen, ptr, n, ccb,
                               scratch)
    return rc if cb is not None else (rc, matches)


def hwlm_exec_stream(blob, hist, data, start=0, cb=None, groups=HWLM_ALL_GROUPS,
                     filler=b""):
    """hwlmExecStreaming (hwlm.h:137).  The reference reads buf / hbuf / hlen
    from scratch->core_info; this builds a scratch image carrying them at the
    offsets the library uses (vsa_get_scratch_core_info)."""
    hk, hptr, hlen = _history(hist, filler)
    keep, ptr, n = _as_buf(data)
    offs = [ctypes.c_long() for _ in range(3)]
    lib.vsa_get_scratch_core_info(*[ctypes.byref(o) for o in offs])
    scratch = ctypes.create_string_buffer(max(o.value for o in offs) + 4096)
    base = ctypes.addressof(scratch)
    ctypes.c_void_p.from_address(base + offs[0].value).value = ptr
    ctypes.c_void_p.from_address(base + offs[1].value).value = hptr if hlen else None
    ctypes.c_size_t.from_address(base + offs[2].value).value = hlen
    ccb, matches = _runner(None, cb)
    rc = lib.hwlmExecStreaming(blob.ptr, n, start, ccb, base, groups)
    return rc if cb is not None else (rc, matches)


def _m16(x):
    x = bytes(x)
    assert len(x) == 16
    return ctypes.create_string_buffer(x, 16)


def shufti_exec(lo, hi, data):
    """shuftiExec: index of the first byte in the class, or len(data)."""
    keep, ptr, n = _as_buf(data)
    return lib.vsa_shufti_find(_m16(lo), _m16(hi), ptr, n, 0)


def shufti_double_find(lo1, hi1, lo2, hi2, ptr, n):
    """shuftiDoubleExec on host memory at address `ptr` (its alignment
    matters, as in the reference): first match index or n."""
    return lib.vsa_shufti_double_find(_m16(lo1), _m16(hi1), _m16(lo2), _m16(hi2), ptr, n)


def set_accel_vector_size(vsize):
    """VECTORSIZE of the reference build emulated by shuftiDoubleExec."""
    lib.vsa_set_accel_vector_size(vsize)


def shufti_build_double_masks(pairs, onechar=b""):
    """shuftiBuildDoubleMasks (shufticompile.cpp:135): (lo1, hi1, lo2, hi2)
    or None when more than 8 buckets are needed."""
    cls = class_bitmap(onechar)
    pr = np.array([b for p in pairs for b in p], np.uint8)
    out = [np.zeros(16, np.uint8) for _ in range(4)]
    r = lib.vsa_shufti_build_double_masks(cls.ctypes.data, pr.ctypes.data if len(pr) else None,
                                          len(pairs), *[o.ctypes.data for o in out])
    if r < 0:
        return None
    return tuple(o.tobytes() for o in out)


def rshufti_exec(lo, hi, data):
    """rshuftiExec: index of the last byte in the class, or -1."""
    keep, ptr, n = _as_buf(data)
    return lib.vsa_shufti_find(_m16(lo), _m16(hi), ptr, n, 1)


def truffle_exec(m1, m2, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_truffle_find(_m16(m1), _m16(m2), ptr, n, 0)


def rtruffle_exec(m1, m2, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_truffle_find(_m16(m1), _m16(m2), ptr, n, 1)


def _ch(c):
    return c[0] if isinstance(c, (bytes, bytearray)) else (ord(c) if isinstance(c, str) else int(c))


def vermicelli_exec(c, nocase, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(0, _ch(c), 0, 0, 0, int(nocase), ptr, n)


def nvermicelli_exec(c, nocase, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(1, _ch(c), 0, 0, 0, int(nocase), ptr, n)


def rvermicelli_exec(c, nocase, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(2, _ch(c), 0, 0, 0, int(nocase), ptr, n)


def rnvermicelli_exec(c, nocase, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(3, _ch(c), 0, 0, 0, int(nocase), ptr, n)


def vermicelli_double_exec(c1, c2, nocase, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(4, _ch(c1), _ch(c2), 0, 0, int(nocase), ptr, n)


def rvermicelli_double_exec(c1, c2, nocase, data):
    """rvermicelliDoubleExec: index of c2 of the last (c1, c2) pair, or -1."""
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(6, _ch(c1), _ch(c2), 0, 0, int(nocase), ptr, n)


def vermicelli_double_masked_exec(c1, c2, m1, m2, data):
    keep, ptr, n = _as_buf(data)
    return lib.vsa_verm_find(5, _ch(c1), _ch(c2), _ch(m1), _ch(m2), 0, ptr, n)


def class_bitmap(chars):
    """256-bit class image (bit c of byte c>>3) from an iterable of bytes."""
    cls = np.zeros(32, np.uint8)
    for c in chars:
        cls[c >> 3] |= 1 << (c & 7)
    return cls


def shufti_build_masks(chars):
    """shuftiBuildMasks (shufticompile.cpp:54): (lo, hi) or None."""
    cls = class_bitmap(chars)
    lo = np.zeros(16, np.uint8)
    hi = np.zeros(16, np.uint8)
    r = lib.vsa_shufti_build_masks(cls.ctypes.data, lo.ctypes.data, hi.ctypes.data)
    if r < 0:
        return None
    return lo.tobytes(), hi.tobytes()


def truffle_build_masks(chars):
    """truffleBuildMasks (trufflecompile.cpp:60)."""
    cls = class_bitmap(chars)
    m1 = np.zeros(16, np.uint8)
    m2 = np.zeros(16, np.uint8)
    lib.vsa_truffle_build_masks(cls.ctypes.data, m1.ctypes.data, m2.ctypes.data)
    return m1.tobytes(), m2.tobytes()


# ---------------------------------------------------------------- batch API

class Context:
    """vsa_ctx: a HIP stream + device workspace on one GPU."""

    def __init__(self, device=0, share_stream_with=None):
        """share_stream_with: another Context whose stream this one queues
        on (vsa_ctx_create_shared): a second workspace for pipelined scans
        that still run one at a time"""
        self.ptr = ctypes.c_void_p()
        if share_stream_with is not None:
            device = share_stream_with.device
            rc = lib.vsa_ctx_create_shared(share_stream_with.ptr, ctypes.byref(self.ptr))
        else:
            rc = lib.vsa_ctx_create(device, ctypes.byref(self.ptr))
        if rc != 0:
            raise RuntimeError("vsa_ctx_create(%d) failed (%d)" % (device, rc))
        self.device = device

    @property
    def stream(self):
        return lib.vsa_ctx_stream(self.ptr)

    def malloc(self, nbytes):
        p = ctypes.c_void_p()
        _check(lib.vsa_malloc(self.ptr, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, p):
        _check(lib.vsa_free(self.ptr, p))

    def h2d(self, dptr, host):
        host = np.ascontiguousarray(host)
        _check(lib.vsa_memcpy_h2d(self.ptr, dptr, host.ctypes.data, host.nbytes))

    def d2h(self, host, dptr):
        _check(lib.vsa_memcpy_d2h(self.ptr, host.ctypes.data, dptr, host.nbytes))

    def sync(self):
        _check(lib.vsa_sync(self.ptr))

    def scan_blocks(self, db, d_data, offsets, lens, starts=None, sort=True,
                    asynchronous=False):
        off = np.ascontiguousarray(offsets, np.uint64)
        ln = np.ascontiguousarray(lens, np.uint64)
        st = None if starts is None else np.ascontiguousarray(starts, np.uint64)
        n = ctypes.c_uint64()
        flags = (0 if sort else 1) | (2 if asynchronous else 0)
        rc = lib.vsa_scan_blocks(
            self.ptr, db.ptr, d_data, off.ctypes.data_as(_u64p),
            ln.ctypes.data_as(_u64p), None if st is None else st.ctypes.data,
            len(off), flags, ctypes.byref(n))
        if rc != 0:
            raise RuntimeError("vsa_scan_blocks failed (%d)" % rc)
        return n.value

    def scan_blocks_ex(self, db, d_data, offsets, lens, starts=None, report_lo=None,
                       sort=True, asynchronous=False):
        """vsa_scan_blocks_ex: as scan_blocks, ends below report_lo[i] of
        block i are not reported (the FDR start state stays at starts[i])."""
        off = np.ascontiguousarray(offsets, np.uint64)
        ln = np.ascontiguousarray(lens, np.uint64)
        st = None if starts is None else np.ascontiguousarray(starts, np.uint64)
        rl = None if report_lo is None else np.ascontiguousarray(report_lo, np.uint64)
        n = ctypes.c_uint64()
        flags = (0 if sort else 1) | (2 if asynchronous else 0)
        rc = lib.vsa_scan_blocks_ex(
            self.ptr, db.ptr, d_data, off.ctypes.data_as(_u64p), ln.ctypes.data_as(_u64p),
            None if st is None else st.ctypes.data, None if rl is None else rl.ctypes.data,
            len(off), flags, ctypes.byref(n))
        if rc != 0:
            raise RuntimeError("vsa_scan_blocks_ex failed (%d)" % rc)
        return n.value

    def scan_blocks_stream(self, db, d_data, offsets, lens, hlens, starts=None, sort=True,
                           asynchronous=False):
        """vsa_scan_blocks_stream: block i is a streaming call whose hlens[i]
        history bytes sit just before offsets[i] in the same device buffer."""
        off = np.ascontiguousarray(offsets, np.uint64)
        ln = np.ascontiguousarray(lens, np.uint64)
        hl = np.ascontiguousarray(hlens, np.uint64)
        st = None if starts is None else np.ascontiguousarray(starts, np.uint64)
        n = ctypes.c_uint64()
        flags = (0 if sort else 1) | (2 if asynchronous else 0)
        rc = lib.vsa_scan_blocks_stream(
            self.ptr, db.ptr, d_data, off.ctypes.data_as(_u64p), ln.ctypes.data_as(_u64p),
            None if st is None else st.ctypes.data, hl.ctypes.data_as(_u64p), len(off), flags,
            ctypes.byref(n))
        if rc != 0:
            raise RuntimeError("vsa_scan_blocks_stream failed (%d)" % rc)
        return n.value

    def plan(self, d_data, offsets, lens, starts=None, hlens=None, report_lo=None):
        """vsa_plan_create: the batch's launch tables built once (Plan.scan
        reuses them)."""
        arrs = [None if a is None else np.ascontiguousarray(a, np.uint64)
                for a in (offsets, lens, starts, hlens, report_lo)]
        h = ctypes.c_void_p()
        rc = lib.vsa_plan_create(self.ptr, d_data, *[None if a is None else a.ctypes.data
                                                      for a in arrs], len(arrs[0]),
                                 ctypes.byref(h))
        if rc != 0:
            raise RuntimeError("vsa_plan_create failed (%d)" % rc)
        return Plan(self, h.value)

    def scan_plan(self, db, plan, sort=True, asynchronous=False):
        n = ctypes.c_uint64()
        flags = (0 if sort else 1) | (2 if asynchronous else 0)
        rc = lib.vsa_scan_plan(self.ptr, db.ptr, plan.ptr, flags, ctypes.byref(n))
        if rc != 0:
            raise RuntimeError("vsa_scan_plan failed (%d)" % rc)
        return n.value

    def scan_wait(self):
        n = ctypes.c_uint64()
        _check(lib.vsa_scan_wait(self.ptr, ctypes.byref(n)))
        return n.value

    def scan_pack(self, d_dst, cap):
        """vsa_scan_pack: the last scan's sorted records packed into device
        memory d_dst as [header | keys (cap) | ids (cap x u32)] for a
        collective (queued behind an asynchronous binned scan, no wait)."""
        _check(lib.vsa_scan_pack(self.ptr, d_dst, cap))

    def scan_plan_pack(self, db, plan, d_dst, cap):
        """vsa_scan_plan_pack: an asynchronous plan scan whose binned sort
        also writes the records into d_dst in scan_pack's layout (no pack
        launch); vsa_scan_pack still repacks after a rescan."""
        _check(lib.vsa_scan_plan_pack(self.ptr, db.ptr, plan.ptr, d_dst, cap))

    def results(self, n):
        """Copy the last scan's sorted (key, id) records to the host."""
        out = np.zeros(n, dtype=[("key", np.uint64), ("id", np.uint32), ("pad", np.uint32)])
        got = ctypes.c_uint64()
        _check(lib.vsa_scan_copy(self.ptr, out.ctypes.data, n, ctypes.byref(got)))
        return out[: got.value]

    def results_to_device(self, d_keys, d_ids, cap):
        """Copy up to cap results of the last scan into caller device buffers
        (stream-ordered on this context's stream); returns the count."""
        got = ctypes.c_uint64()
        _check(lib.vsa_scan_copy_device(self.ptr, d_keys, d_ids, cap, ctypes.byref(got)))
        return got.value

    def candidates(self):
        return lib.vsa_scan_candidates(self.ptr)

    def debug_counters(self):
        """device counters 0..15 of the last scan (see vsa_scan_debug_counters)"""
        out = (ctypes.c_uint64 * 16)()
        _check(lib.vsa_scan_debug_counters(self.ptr, out))
        return list(out)

    def kernel_ms(self):
        """Device time of the last scan kernel (hipEvents on the scan stream)."""
        return lib.vsa_scan_kernel_ms(self.ptr)

    def reserve_cus(self, n):
        """vsa_ctx_set_reserved_cus: plans built afterwards leave n CUs free
        of the scan's persistent grid (for a concurrent collective)."""
        _check(lib.vsa_ctx_set_reserved_cus(self.ptr, n))

    def launches(self):
        """Literal-scan launches queued on this context (reruns included)."""
        return lib.vsa_scan_launches(self.ptr)

    def timing(self, every=1):
        """Time every `every`-th literal-scan launch (vsa_ctx_set_timing;
        kernel_ms() is -1 after an untimed one)."""
        _check(lib.vsa_ctx_set_timing(self.ptr, every))

    def fused_finish(self, on=True):
        """Sort inside the scan kernel when the plan allows it
        (vsa_ctx_set_fused_finish; results are identical either way)."""
        _check(lib.vsa_ctx_set_fused_finish(self.ptr, 1 if on else 0))

    def last_fused(self):
        """True when the last literal-scan launch sorted its records inside
        the scan (the fused finish, no vsa_bin_finish launch)."""
        return lib.vsa_scan_last_fused(self.ptr) == 1

    def last_dyn(self):
        """True when the last literal-scan launch set its workgroups' shares
        itself (dynamic shares, kernels.hip dyn_bounds)."""
        return lib.vsa_scan_last_dyn(self.ptr) == 1

    def dyn_shares(self, on=True, min_mib=2048):
        """Dynamic shares for the FDR launches of >= min_mib MiB over eligible
        plans (vsa_ctx_set_dyn_shares)."""
        _check(lib.vsa_ctx_set_dyn_shares(self.ptr, 1 if on else 0, int(min_mib) << 20))

    def read_ceiling(self, d_data, length, runs=5):
        """(GB/s, ms, bytes): this device's streaming-read ceiling over the
        device buffer at d_data (vsa_read_ceiling), best of `runs`."""
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        _check(lib.vsa_read_ceiling(self.ptr, d_data, length, runs, ctypes.byref(ms),
                                    ctypes.byref(n)))
        return n.value / (ms.value * 1e-3) / 1e9, ms.value, n.value

    def class_scan(self, cls, d_data, length, d_bitmap=None, cls2=None):
        cls = np.ascontiguousarray(cls, np.uint8)
        c2 = None if cls2 is None else np.ascontiguousarray(cls2, np.uint8)
        f, l, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.vsa_class_scan(self.ptr, cls.ctypes.data,
                                  None if c2 is None else c2.ctypes.data, d_data,
                                  length, d_bitmap, ctypes.byref(f), ctypes.byref(l),
                                  ctypes.byref(c), 0))
        return f.value, l.value, c.value

    def class_scan_masks(self, kind, a, b, d_data, length, d_bitmap=None):
        """vsa_class_scan_masks: the shufti (kind "shufti": lo, hi) or truffle
        ("truffle": m1, m2) masks over a device buffer -> (first, last, count)"""
        ma = ctypes.create_string_buffer(bytes(a), 16)
        mb = ctypes.create_string_buffer(bytes(b), 16)
        f, l, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.vsa_class_scan_masks(self.ptr, 0 if kind == "shufti" else 1, ma, mb, d_data,
                                        length, d_bitmap, ctypes.byref(f), ctypes.byref(l),
                                        ctypes.byref(c)))
        return f.value, l.value, c.value

    def close(self):
        if self.ptr:
            lib.vsa_ctx_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    """vsa_plan_t: a batch's block table and segment map on the device."""

    def __init__(self, ctx, ptr):
        self.ctx = ctx
        self.ptr = ptr

    def rebuilds(self):
        """how many times the plan's segment map was rebuilt for new XCD
        feedback weights (vsa_plan_rebuilds)"""
        return lib.vsa_plan_rebuilds(self.ptr)

    def close(self):
        if self.ptr:
            lib.vsa_plan_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Database:
    """vsa_db: device-resident copy of an HWLM blob."""

    def __init__(self, ctx, blob):
        self.ctx = ctx
        self.blob = blob
        self.ptr = ctypes.c_void_p()
        rc = lib.vsa_db_load(ctx.ptr, blob.ptr, blob.size, ctypes.byref(self.ptr))
        if rc != 0:
            raise RuntimeError("vsa_db_load failed (%d)" % rc)

    @property
    def engine(self):
        return lib.vsa_db_engine(self.ptr)

    @property
    def split(self):
        """True when the database scans in split passes (large FDR sets)"""
        return lib.vsa_db_split(self.ptr) == 1

    def close(self):
        if self.ptr:
            lib.vsa_db_free(self.ptr)
            self.ptr = None


def version():
    return lib.vsa_version().decode()
