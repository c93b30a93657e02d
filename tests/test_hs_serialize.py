"""Serialized databases and the rest of the hs_common / hs_runtime surface
(include/vectorscan_amd_hs.h): the reference's envelope (database.c:61-455),
restated from unit/hyperscan/serialize.cpp's checks with pure-literal
databases (the reference's own regex patterns need its regex compiler, which
is out of scope).  The CPU tests need no GPU: compiling and serializing are
host work.  Byte identity with a reference-serialized database stays
unpinned (nothing reference-built is available here); the envelope, CRC and
error codes are checked against the reference's rules."""
import ctypes
import random
import struct

import pytest

import vectorscan_amd as vsa
from vectorscan_amd import hs


def crc32c(b):
    """CRC-32C as Crc32c_ComputeBuf(0, ...) (crc32.c: reflected 0x82F63B78,
    no inversion), bit by bit"""
    c = 0
    for x in b:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c


MODES = [hs.MODE_BLOCK, hs.MODE_STREAM | hs.MODE_SOM_HORIZON_LARGE, hs.MODE_VECTORED]
PATTERNS = [
    ([b"hatstand", b"teakettle", b"badgerbrush"], [hs.FLAG_CASELESS, 0, hs.FLAG_SINGLEMATCH],
     [1000, 1001, 1002]),
    ([b"foobar", b"xyzzy"], [hs.FLAG_SOM_LEFTMOST, 0], [1004, 1005]),
    ([b".exe", b".pdf", b"\x01\xff\x00"], [0, hs.FLAG_CASELESS, 0], [1008, 1008, 7]),
]


def mode_string(mode):
    return "STREAM" if mode & hs.MODE_STREAM else "BLOCK" if mode & hs.MODE_BLOCK else "VECTORED"


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("pat", range(len(PATTERNS)))
def test_serialize_deserialize_any_alignment(mode, pat):
    """serialize.cpp:85-150 DeserializeFromAnyAlignment: info starts with
    "Version:" and names the mode; serialized info, deserialized info and the
    original agree at every alignment of the bytes; the round trip keeps the
    bytecode (same HWLM blob, same serialized bytes)."""
    if (mode & hs.MODE_STREAM) == 0 and any(f & hs.FLAG_SOM_LEFTMOST
                                            for f in PATTERNS[pat][1]):
        pass  # SOM is accepted in any mode for literals
    db = hs.compile_lit_multi(*PATTERNS[pat], mode=mode)
    info = db.info()
    assert info.startswith("Version:") and mode_string(mode) in info
    data = db.serialize()
    assert len(data) > 0
    for i in range(16):
        buf = ctypes.create_string_buffer(len(data) + 16)
        ctypes.memmove(ctypes.addressof(buf) + i, data, len(data))
        p = ctypes.c_void_p(ctypes.addressof(buf) + i)
        sinfo = ctypes.c_void_p()
        assert vsa.lib.vsa_hs_serialized_database_info(p, len(data), ctypes.byref(sinfo)) == 0
        assert hs._take_string(sinfo) == info
        h = ctypes.c_void_p()
        assert vsa.lib.vsa_hs_deserialize_database(p, len(data), ctypes.byref(h)) == 0
        d2 = hs.Database(h.value, mode & 7)
        assert d2.info() == info
        assert d2.serialize() == data
        assert d2.hwlm_bytes() == db.hwlm_bytes()
        d2.close()
    db.close()


def test_serialized_layout():
    """database.c:61-110: 32 header bytes (magic, HS_VERSION_32BIT of the
    reference's 5.4.11, bytecode length, platform at byte 12, CRC-32C of the
    bytecode, reserved words 0), the bytecode, zero padding to
    sizeof(struct hs_database) = 104 plus the length; the bytecode's first
    bytes are RoseEngine's pureLiteral / runtimeImpl / mode fields
    (rose_internal.h:330-345)."""
    db = hs.compile_lit_multi([b"abc", b"defgh"], [0, 0], [1, 2], hs.MODE_STREAM)
    data = db.serialize()
    magic, version, length = struct.unpack_from("<III", data, 0)
    platform, = struct.unpack_from("<Q", data, 12)
    crc, r0, r1 = struct.unpack_from("<III", data, 20)
    assert magic == 0xdbdbdbdb
    assert version == (5 << 24) | (4 << 16) | (11 << 8)
    assert len(data) == 104 + length
    code = data[32:32 + length]
    assert crc == crc32c(code)
    assert (r0, r1) == (0, 0)
    assert data[32 + length:] == bytes(72)
    assert platform == (4 << 13) | (8 << 13) | (0x10 << 13)
    assert code[0] == 1 and code[4] == 1  # pureLiteral, ROSE_RUNTIME_PURE_LITERAL
    assert struct.unpack_from("<I", code, 12)[0] == hs.MODE_STREAM
    # CrossCompileSom (serialize.cpp:244-277): database size == serialized size
    assert db.size() == hs.serialized_size(data) == len(data)


def test_serialized_errors():
    """db_decode_header (database.c:122-170) and db_check_crc: bad magic /
    length / CRC -> HS_INVALID, another version -> HS_DB_VERSION_ERROR; a
    bytecode that is not this engine's (a reference RoseEngine) ->
    HS_DB_PLATFORM_ERROR, while hs_serialized_database_info still reads its
    mode."""
    db = hs.compile_lit_multi([b"needle"], [0], [3], hs.MODE_BLOCK)
    data = bytearray(db.serialize())

    def code_of(b):
        try:
            hs.deserialize(bytes(b))
        except hs.HsError as e:
            return e.code
        return 0

    assert code_of(data) == 0
    bad = bytearray(data); bad[0] ^= 1
    assert code_of(bad) == hs.INVALID
    bad = bytearray(data); bad[5] ^= 1
    assert code_of(bad) == hs.DB_VERSION_ERROR
    assert code_of(data[:-1]) == hs.INVALID
    assert code_of(data + b"\0") == hs.INVALID
    bad = bytearray(data); bad[32 + 70] ^= 0x40
    assert code_of(bad) == hs.INVALID  # CRC
    # a foreign bytecode with a valid envelope (RoseEngine prefix, mode
    # VECTORED, no engine tag)
    code = bytearray(256)
    code[0] = 1
    code[12:16] = struct.pack("<I", hs.MODE_VECTORED)
    foreign = bytearray(104 + len(code))
    struct.pack_into("<IIIQIII", foreign, 0, 0xdbdbdbdb, (5 << 24) | (4 << 16) | (11 << 8),
                     len(code), 0, crc32c(code), 0, 0)
    foreign[32:32 + len(code)] = code
    assert code_of(foreign) == hs.DB_PLATFORM_ERROR
    info = hs.serialized_info(bytes(foreign))
    assert info == "Version: 5.4.11 Features: AVX512VBMI Mode: VECTORED"
    assert hs.serialized_size(bytes(foreign)) == len(foreign)


def test_version_and_platform():
    """hs_version / hs_valid_platform (hs_common.h:446 / :463)"""
    assert hs.version().startswith("5.4.11")
    assert hs.valid_platform() == hs.SUCCESS


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [hs.MODE_BLOCK, hs.MODE_STREAM, hs.MODE_VECTORED])
def test_gpu_deserialized_scans(mode):
    """A deserialized database scans exactly like the original (callback
    sequences), through a cloned scratch too; streams: hs_copy_stream /
    hs_reset_and_copy_stream continue from the copied state."""
    rng = random.Random(31 + mode)
    alpha = b"abcdefgh"
    lits = sorted({bytes(rng.choice(alpha) for _ in range(rng.randint(2, 9)))
                   for _ in range(60)})
    flags = [rng.choice([0, 0, hs.FLAG_CASELESS, hs.FLAG_SINGLEMATCH, hs.FLAG_SOM_LEFTMOST])
             for _ in lits]
    ids = [rng.randrange(40) for _ in lits]
    # one flag per id for SINGLEMATCH (compile rule)
    single = {}
    for k, i in enumerate(ids):
        single.setdefault(i, flags[k] == hs.FLAG_SINGLEMATCH)
        if single[i] != (flags[k] == hs.FLAG_SINGLEMATCH):
            flags[k] = hs.FLAG_SINGLEMATCH if single[i] else 0
    db = hs.compile_lit_multi(lits, flags, ids, mode)
    db2 = hs.deserialize(db.serialize())
    s1 = hs.Scratch(db)
    s1.grow(db2)
    s2 = s1.clone()
    assert s2.size() >= s1.size() > 0
    data = bytes(rng.choice(alpha + b"ABC") for _ in range(50000))
    pieces = [data[:7000], data[7000:7001], data[7001:30000], data[30000:]]
    try:
        if mode == hs.MODE_BLOCK:
            rc1, m1 = hs.scan(db, data, s1)
            rc2, m2 = hs.scan(db2, data, s2)
        elif mode == hs.MODE_VECTORED:
            rc1, m1 = hs.scan_vector(db, pieces, s1)
            rc2, m2 = hs.scan_vector(db2, pieces, s2)
        else:
            st1, st2 = hs.Stream(db), hs.Stream(db2)
            m1, m2 = [], []
            for k, p in enumerate(pieces):
                m1 += st1.scan(p, s1)[1]
                m2 += st2.scan(p, s2)[1]
                if k == 1:
                    # continue a copy from here: it must deliver what the
                    # original delivers from here on
                    cp = st1.copy()
                    other = hs.Stream(db)
                    assert other.reset_and_copy(st1, s1) == hs.SUCCESS
            rest = [p for p in pieces[2:]]
            mc, mo = [], []
            for p in rest:
                mc += cp.scan(p, s1)[1]
                mo += other.scan(p, s1)[1]
            tail = [m for m in m1 if m[2] > 7001]
            assert mc == tail and mo == tail
            for st in (st1, st2, cp, other):
                assert st.close(s1) == hs.SUCCESS
            rc1 = rc2 = 0
            assert db.stream_size() > 0
        assert rc1 == rc2 == 0
        assert m1 == m2 and len(m1) > 0
    finally:
        s2.close()
        s1.close()
        db2.close()
        db.close()
