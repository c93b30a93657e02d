"""Generate tests/golden/*.json — the known answers of the reference's own
unit tests for this path, restated as data (inputs + expected outputs).

Each case cites the reference test it restates.  The expected values are
the reference tests' assertions (literal positions / the test's own
std::string::compare brute force), not outputs of our oracle or engine.

    python tests/golden/make_golden.py      # rewrites the JSON files
"""
import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def hx(b):
    return bytes(b).hex()


# --------------------------------------------------------------- noodle
def noodle_cases():
    """unit/internal/noodle.cpp:81-262 (noodleMatch calls noodExec from 0)."""
    cases = []

    def add(src, data, lit, nocase, expected):
        cases.append({"src": src, "data": hx(data), "lit": hx(lit), "nocase": nocase,
                      "expected": expected})

    a1024 = b"a" * 1024
    # nood1 :81-121
    add("noodle.cpp:87", a1024, b"a", 0, list(range(1024)))
    add("noodle.cpp:93", a1024, b"A", 0, [])
    add("noodle.cpp:97", a1024, b"A", 1, list(range(1024)))
    for j in range(16):
        add("noodle.cpp:105", a1024[j:], b"A", 1, list(range(1024 - j)))
        add("noodle.cpp:112", a1024[:1024 - j], b"A", 1, list(range(1024 - j)))
    # nood2 :123-177
    add("noodle.cpp:130", a1024, b"aa", 0, [i + 1 for i in range(1023)])
    add("noodle.cpp:137", a1024, b"aA", 0, [])
    add("noodle.cpp:141", a1024, b"AA", 0, [])
    add("noodle.cpp:145", a1024, b"aa", 1, [i + 1 for i in range(1023)])
    add("noodle.cpp:152", a1024, b"Aa", 1, [i + 1 for i in range(1023)])
    add("noodle.cpp:159", a1024, b"AA", 1, [i + 1 for i in range(1023)])
    for j in range(16):
        add("noodle.cpp:167", a1024[j:], b"Aa", 1, [i + 1 for i in range(1023 - j)])
        add("noodle.cpp:174", a1024[:1024 - j], b"aA", 1, [i + 1 for i in range(1023 - j)])
    # noodLong :179-221
    add("noodle.cpp:186", a1024, b"aaaa", 0, [i + 3 for i in range(1021)])
    add("noodle.cpp:192", a1024, b"aaAA", 0, [])
    add("noodle.cpp:196", a1024, b"aaAA", 1, [i + 3 for i in range(1021)])
    for j in range(16):
        add("noodle.cpp:204", a1024[j:], b"AAaa", 1, [i + 3 for i in range(1021 - j)])
        add("noodle.cpp:211", a1024[j:], b"aaaA", 1, [i + 3 for i in range(1021 - j)])
    # noodCutoverSingle / Double :223-262 (alignment sweep -> lengths)
    for ln in range(128):
        add("noodle.cpp:233", b"a" * ln, b"a", 0, list(range(ln)))
        add("noodle.cpp:253", b"a" * ln, b"aa", 0, [i + 1 for i in range(max(0, ln - 1))])
    return cases


# ------------------------------------------------------------------ FDR
def fdr_cases():
    """unit/internal/fdr.cpp:167-744, run for every engine hint by the
    tests (FDRp is parameterised over getValidFdrEngines, :113-137)."""
    cases = []

    def lit(s, nocase=0, id=0, noruns=0):
        return {"s": hx(s), "nocase": nocase, "id": id, "noruns": noruns}

    def add(src, lits, data, expected, start=0, term_after=-1, exact_order=True,
            expected_len=None):
        c = {"src": src, "lits": lits, "data": hx(data), "start": start,
             "term_after": term_after, "expected": expected,
             "exact_order": exact_order}
        if expected_len is not None:
            c["expected_len"] = expected_len
        cases.append(c)

    d = b"mnopqrabcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ12345678901234567890mnopqr\0"
    add("fdr.cpp:167 Simple", [lit(b"mnopqr", 0, 0)], d, [[5, 0], [23, 0], [83, 0]])
    d2 = b"mnopqrabcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ12345678901234567890m0m"
    add("fdr.cpp:191 SimpleSingle", [lit(b"m", 0, 0)], d2,
        [[0, 0], [18, 0], [78, 0], [80, 0]])
    for i in range(128 - 3):
        buf = bytearray(128)
        buf[i:i + 3] = b"abc"
        add("fdr.cpp:216 MultiLocation", [lit(b"abc", 0, 1)], bytes(buf), [[i + 2, 1]])
    add("fdr.cpp:246 NoRepeat1", [lit(b"m", 0, 0, 1)], d2, [[0, 0]])
    # NoRepeat2 asserts only matches[0], matches[2] and the count (:290-293)
    add("fdr.cpp:270 NoRepeat2", [lit(b"m", 0, 0, 1), lit(b"A", 0, 42)], d2,
        [[0, 0], [32, 42], [78, 0]])
    add("fdr.cpp:297 NoRepeat3", [lit(b"90m", 0, 0, 1), lit(b"zA", 0, 0, 1)], d2,
        [[32, 0]])
    d3 = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ12345678901234567890"
    add("fdr.cpp:405 moveByteStream", [lit(b"mnopqr", 0, 0)], d3, [[17, 0]])
    # FDRTermB :721-744: first callback terminates
    add("fdr.cpp:721 FDRTermB", [lit(b"f", 0, 0), lit(b"ff", 0, 1)], b"f" * 17, None,
        term_after=1, expected_len=1)
    # AlignAndTooEarly :496-567: matches at both ends only when j == 0
    for pat, alien in ((b"abaabaaa", b"x"), (b"zzzyyzyz", b"\x99"), (b"abcdef l", b"\0")):
        for ll in range(1, len(pat) + 1):
            for i in range(0, 32, 5):
                buf = bytearray(alien * 160)
                buf[i:i + ll] = pat[:ll]
                buf[i + 128 - ll:i + 128] = pat[:ll]
                for j in range(0, ll + 1):
                    data = bytes(buf[i + j:i + j + 128 - 2 * j])
                    exp = [[ll - 1, 0], [127, 0]] if j == 0 else []
                    add("fdr.cpp:496 AlignAndTooEarly", [lit(pat[:ll], 0, 0)], data, exp)
    return cases


def short_writings_spec():
    """fdr.cpp:594-692 ShortWritings: buffers and literal groups; the test's
    expected set is its own std::string::compare brute force."""
    out = []
    for alphabet in ([0x61, 0x62, 0x78], [0x78, 0x79, 0x7A], [0x00, 0x41, 0x20],
                     [0x61, 0x20, 0x99]):
        bufs = []
        for ln in range(1, 7):
            for j in range(3 ** ln):
                bufs.append(bytes(alphabet[(j // (3 ** k)) % 3] for k in range(ln)))
        nb = len(bufs)

        def fib(n):
            f0 = f1 = f2 = 1
            for _ in range(n):
                f2 = f1 + f0
                f0 = f1
                f1 = f2
            return f2

        for ln in range(7, 64):
            for i in range(10):
                s = b""
                j = 0
                while len(s) < ln:
                    s += bufs[fib(i * 5 + j + (ln - 6) * 10) % nb]
                    j += 1
                bufs.append(s)
        pats = []
        for ln in range(1, 9):
            for j in range(2 ** ln):
                pats.append(bytes(alphabet[(j >> k) & 1] for k in range(ln)))
        out.append({"alphabet": alphabet, "bufs": [hx(b) for b in bufs],
                    "pats": [hx(p) for p in pats]})
    return out


# ---------------------------------------------------------------- accel
def accel_cases():
    """shufti.cpp / truffle.cpp / vermicelli.cpp / rvermicelli.cpp known
    answers.  kind: shufti|rshufti|truffle|rtruffle (class = chars),
    verm|nverm|rverm|rnverm (c, nocase), dverm|rdverm (c1, c2, nocase)."""
    cases = []

    def add(src, kind, data, expected, **kw):
        c = {"src": src, "kind": kind, "data": hx(data), "expected": expected}
        c.update(kw)
        cases.append(c)

    t = b"bbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(32):
        add("shufti.cpp:166 ExecMatch1", "shufti", t[i:], 33 - i, chars=[0x61])
    t = b"bbbbbbbbbbbbbbbbbaaaaaaaaaaaaaaaabbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        add("shufti.cpp:185 ExecMatch2", "shufti", t[i:], 17 - i, chars=[0x61])
        add("truffle.cpp:249 ExecMatch2", "truffle", t[i:], 17 - i, chars=[0x61])
    t = b"bbbbbbbbbbbbbbbbbBaaaaaaaaaaaaaaabbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        add("shufti.cpp:204 ExecMatch3", "shufti", t[i:], 17 - i, chars=[0x61, 0x42])
    for ch in b"ACca":
        t = b"bbbbbbbbbbbbbbbbb" + bytes([ch]) + b"aaaaaaaaaaaaaaabbbbbbbbbbbbbbbabbbbbbbbbbbb"
        for i in range(16):
            add("shufti.cpp:224 ExecMatch4", "shufti", t[i:], 17 - i,
                chars=[0x61, 0x43, 0x41, 0x63])
    t = bytearray(b"b" * 76)
    for i in range(31):
        t[48 - i] = 0x61
        add("shufti.cpp:261 ExecMatch5", "shufti", bytes(t), 48 - i, chars=[0x61])
    t = b"b" * 61
    for i in range(32):
        add("shufti.cpp:111 ExecNoMatch1", "shufti", t[i:], len(t) - i, chars=[0x61])
    t = b"bbbbbbabbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbbb"
    for i in range(16):
        add("shufti.cpp:964 ReverseExecMatch1", "rshufti", t[:len(t) - i], 17, chars=[0x61])
    t = bytearray(b"b" * 76)
    for i in range(76):
        t[i] = 0x61
        add("shufti.cpp:1076 ReverseExecMatch5", "rshufti", bytes(t), i, chars=[0x61])
    t = bytearray(b"b" * 256)
    for i in range(256):
        t[i] = 0x61
        add("shufti.cpp:1096 ReverseExecMatch6", "rshufti", bytes(t), i, chars=[0x61])
    # truffle
    t = b"b" * 61 + b"\xff"
    for i in range(16):
        add("truffle.cpp:94 ExecNoMatch1", "truffle", t[i:], len(t) - i, chars=[0x61])
    add("truffle.cpp:151 ExecMiniMatch0", "truffle", b"a", 0, chars=[0x61])
    add("truffle.cpp:166 ExecMiniMatch1", "truffle", b"bbbbbbbabbb", 7, chars=[0x61])
    add("truffle.cpp:181 ExecMiniMatch2", "truffle", b"bbbbbbb\0bbb", 7, chars=[0])
    add("truffle.cpp:196 ExecMiniMatch3", "truffle", b"\0\0\0\0\0\0\0a\0\0\0", 7, chars=[0x61])
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        add("truffle.cpp:230 ExecMatch1", "truffle", t[i:], 17 - i, chars=[0x61])
    t = b"eeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeeee"
    for i in range(16):
        add("truffle.cpp:133 ExecNoMatch3", "truffle", t[i:], len(t) - i, chars=[0x56])
    t = bytearray(b"b" * 76)
    for i in range(76):
        t[i] = 0x61
        add("truffle.cpp:602 ReverseExecMatch5", "rtruffle", bytes(t), i, chars=[0x61])
    # vermicelli
    t = b"b" * 61
    for i in range(16):
        for j in range(16):
            s = t[i:len(t) - j]
            add("vermicelli.cpp:35 ExecNoMatch1", "verm", s, len(s), c=0x61, nocase=0)
            add("vermicelli.cpp:35 ExecNoMatch1", "verm", s, len(s), c=0x41, nocase=1)
            add("vermicelli.cpp:122 DV ExecNoMatch1", "dverm", s, len(s), c1=0x61, c2=0x62,
                nocase=0)
            add("vermicelli.cpp:140 DV partial", "dverm", s, len(s) - 1, c1=0x62, c2=0x42,
                nocase=0)
            add("vermicelli.cpp:145 DV partial", "dverm", s, len(s) - 1, c1=0x42, c2=0x41,
                nocase=1)
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        add("vermicelli.cpp:58 Exec1", "verm", t[i:], 17 - i, c=0x61, nocase=0)
        add("vermicelli.cpp:58 Exec1", "verm", t[i:], 17 - i, c=0x41, nocase=1)
    t = b"bbbbbbbbbbbbbbbbbAaaaaaaaaaaaaaaaaaaaaaabbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        add("vermicelli.cpp:90 Exec3", "verm", t[i:], 18 - i, c=0x61, nocase=0)
        add("vermicelli.cpp:90 Exec3", "verm", t[i:], 17 - i, c=0x41, nocase=1)
    t = b"bbbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbb"
    for i in range(16):
        add("vermicelli.cpp:157 DV Exec1", "dverm", t[i:], 18 - i, c1=0x61, c2=0x62, nocase=0)
        add("vermicelli.cpp:157 DV Exec1", "dverm", t[i:], 18 - i, c1=0x41, c2=0x42, nocase=1)
        add("vermicelli.cpp:157 DV Exec1", "dverm", t[i:], 17 - i, c1=0x62, c2=0x61, nocase=0)
    t = b"bbbbbbbbbbbbbbbbbaAaaAAaaaaaaaaaaaaaaaaaabbbbbbbaaaaabbbbbbbb"
    for i in range(16):
        add("vermicelli.cpp:199 DV Exec3", "dverm", t[i:], 18 - i, c1=0x41, c2=0x61, nocase=0)
        add("vermicelli.cpp:199 DV Exec3", "dverm", t[i:], 17 - i, c1=0x41, c2=0x41, nocase=1)
        add("vermicelli.cpp:199 DV Exec3", "dverm", t[i:], 21 - i, c1=0x41, c2=0x41, nocase=0)
        add("vermicelli.cpp:199 DV Exec3", "dverm", t[i:], 17 - i, c1=0x61, c2=0x41, nocase=0)
    la = b"abcdefghijklmnopqrstuvwxyz"
    add("vermicelli.cpp:244 noodEarlyExit", "verm", la, 26, c=0x30, nocase=0)
    add("vermicelli.cpp:244 noodEarlyExit", "verm", la, 26, c=0x41, nocase=0)
    for i, ch in enumerate(la):
        add("vermicelli.cpp:253 noodEarlyExit", "verm", la, i, c=ch, nocase=0)
        add("vermicelli.cpp:253 noodEarlyExit", "verm", la, i, c=ch - 0x20, nocase=1)
    t = b"b" * 61
    for i in range(16):
        for j in range(16):
            s_ = t[i:len(t) - j]
            add("vermicelli.cpp:262 NVerm ExecNoMatch1", "nverm", s_, len(s_), c=0x62, nocase=0)
            add("vermicelli.cpp:262 NVerm ExecNoMatch1", "nverm", s_, len(s_), c=0x42, nocase=1)
            add("rvermicelli.cpp:37 ExecNoMatch1", "rverm", s_, -1, c=0x61, nocase=0)
            add("rvermicelli.cpp:37 ExecNoMatch1", "rverm", s_, -1, c=0x42, nocase=0)
            add("rvermicelli.cpp:37 ExecNoMatch1", "rverm", s_, -1, c=0x41, nocase=1)
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        add("vermicelli.cpp:282 NVerm Exec1", "nverm", t[i:], 17 - i, c=0x62, nocase=0)
        add("vermicelli.cpp:282 NVerm Exec1", "nverm", t[i:], 17 - i, c=0x42, nocase=1)
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbb"
    for i in range(16):
        add("rvermicelli.cpp:57 Exec1", "rverm", t[:len(t) - i], 48, c=0x61, nocase=0)
        add("rvermicelli.cpp:57 Exec1", "rverm", t[i:], 48 - i, c=0x41, nocase=1)
    # rvermicelli.cpp:117-200 (RNVermicelli); expected index relative to the
    # scanned slice, -1 = none (buf - 1)
    t = b"b" * 61
    for i in range(16):
        for j in range(16):
            s_ = t[i:len(t) - j]
            add("rvermicelli.cpp:117 RNV ExecNoMatch1", "rnverm", s_, -1, c=0x62, nocase=0)
            add("rvermicelli.cpp:117 RNV ExecNoMatch1", "rnverm", s_, -1, c=0x42, nocase=1)
    for src, t in (("rvermicelli.cpp:137 RNV Exec1",
                    b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbb"),
                   ("rvermicelli.cpp:153 RNV Exec2",
                    b"bbbbbbbbbbbbbbbbbabbbbbbbbaaaaaaaaaaaaaaaaaaaaaaabbbbbbbbbbbbbbbbbbbbb")):
        for i in range(16):
            add(src, "rnverm", t[:len(t) - i], 48, c=0x62, nocase=0)
            add(src, "rnverm", t[i:len(t) - i], 48 - i, c=0x42, nocase=1)
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbaaaaaaaaaaaaaaaaaaaaaaAbbbbbbbbbbbbbbbbbbbbbb"
    for i in range(16):
        add("rvermicelli.cpp:169 RNV Exec3", "rnverm", t[i:], 48 - i, c=0x62, nocase=0)
        add("rvermicelli.cpp:169 RNV Exec3", "rnverm", t[i:], 48 - i, c=0x42, nocase=1)
    t = bytearray(b"b" * 73)
    for i in range(31):
        t[16 + i] = 0x61
        add("rvermicelli.cpp:185 RNV Exec4", "rnverm", bytes(t), 16 + i, c=0x62, nocase=0)
        add("rvermicelli.cpp:185 RNV Exec4", "rnverm", bytes(t), 16 + i, c=0x42, nocase=1)
    # rvermicelli.cpp:203-311 (RDoubleVermicelli): position of c2 of the last
    # pair (a c2 at buf[0] counts), -1 = none
    t = b"bbbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbb"
    for i in range(16):
        add("rvermicelli.cpp:203 RDV Exec1", "rdverm", t[:len(t) - i], 50, c1=0x61, c2=0x62,
            nocase=0)
        add("rvermicelli.cpp:203 RDV Exec1", "rdverm", t[i:], 50 - i, c1=0x41, c2=0x42, nocase=1)
        add("rvermicelli.cpp:203 RDV Exec1", "rdverm", t[i:], 49 - i, c1=0x62, c2=0x61, nocase=0)
        add("rvermicelli.cpp:203 RDV Exec1", "rdverm", t[i:], 49 - i, c1=0x42, c2=0x41, nocase=1)
    t = b"bbbbbbbbbbbbbbbbbaaaaaaaaaaaaaaaaaaaaaaaabbbbbbbaaaaabbbbbbbbbbbbbbbbbb"
    for i in range(16):
        add("rvermicelli.cpp:229 RDV Exec2", "rdverm", t[:len(t) - i], 52, c1=0x61, c2=0x61,
            nocase=0)
        add("rvermicelli.cpp:229 RDV Exec2", "rdverm", t[:len(t) - i], 52, c1=0x41, c2=0x41,
            nocase=1)
    t = b"bbbbbbbbbbbbbbbbbaAaaAAaaaaaaaaaaaaaaaaaabbbbbbbaaaaabbbbbbbbbbbbbbbbbb"
    for i in range(16):
        sl = t[:len(t) - i]
        add("rvermicelli.cpp:245 RDV Exec3", "rdverm", sl, 23, c1=0x41, c2=0x61, nocase=0)
        add("rvermicelli.cpp:245 RDV Exec3", "rdverm", sl, 52, c1=0x41, c2=0x41, nocase=1)
        add("rvermicelli.cpp:245 RDV Exec3", "rdverm", sl, 22, c1=0x41, c2=0x41, nocase=0)
        add("rvermicelli.cpp:245 RDV Exec3", "rdverm", sl, 21, c1=0x61, c2=0x41, nocase=0)
    t = bytearray(b"b" * 93)
    for i in range(31):
        t[32 + i] = 0x61
        t[32 + i - 1] = 0x61
        add("rvermicelli.cpp:272 RDV Exec4", "rdverm", bytes(t), 32 + i, c1=0x61, c2=0x61,
            nocase=0)
        add("rvermicelli.cpp:272 RDV Exec4", "rdverm", bytes(t), 32 + i, c1=0x41, c2=0x41,
            nocase=1)
    t = bytearray(b"b" * 61)
    L = len(t)
    for i in range(16):
        for j in range(1, 17):
            t[L - i - j] = 0x61
            add("rvermicelli.cpp:288 RDV Exec5", "rdverm", bytes(t[:L - i]), L - i - j,
                c1=0x62, c2=0x61, nocase=0)
            add("rvermicelli.cpp:288 RDV Exec5", "rdverm", bytes(t[:L - i]), L - i - j,
                c1=0x42, c2=0x41, nocase=1)
            t[L - i - j] = 0x62
    return cases


def dshufti_cases():
    """shufti.cpp:280-890 (DoubleShufti): mask-builder checks and
    shuftiDoubleExec known answers.  Positions are relative to the test's
    char array t; the scan covers t[start:end].  expect kinds:
      eq       rv == t + value
      ge       rv >= t + value
      ge_end16 rv >= (addr(t) + end) & ~15   (depends on t's alignment)
    """
    build, ex = [], []
    o = ord

    def b(src, pairs, onechar=(), ok=True, checks=(), exact=None):
        build.append({"src": src, "pairs": [[o(x), o(y)] for x, y in pairs],
                      "onechar": [o(c) for c in onechar], "ok": ok,
                      "checks": [[o(a), o(c), rel] for a, c, rel in checks],
                      "exact": exact})

    # BuildMask1 :280-320 (exact masks)
    ex1 = {"lo1": [254 if i == o("a") % 16 else 255 for i in range(16)],
           "hi1": [254 if i == o("a") >> 4 else 255 for i in range(16)],
           "lo2": [254 if i == o("B") % 16 else 255 for i in range(16)],
           "hi2": [254 if i == o("B") >> 4 else 255 for i in range(16)]}
    b("shufti.cpp:280 BuildMask1", [("a", "B")], exact=ex1)
    b("shufti.cpp:322 BuildMask2", [("a", "z"), ("B", "z")],
      checks=[("a", "z", "ne"), ("B", "z", "ne")])
    b("shufti.cpp:348 BuildMask4", [("a", "z"), ("B", "z"), ("A", "z"), ("b", "z")],
      checks=[(c, "z", "ne") for c in "aAbB"])
    b("shufti.cpp:376 BuildMask5", [("a", "z")], onechar="X",
      checks=[("a", "z", "ne")] + [(c, "X", "eq") for c in "aAbB"])
    six = [(c, d) for d in "zyx" for c in "aBAb"]
    b("shufti.cpp:407 BuildMask6", six, checks=[(c, d, "ne") for c, d in six])
    b("shufti.cpp:459 BuildMask7", [(chr(x), chr(x + 1)) for x in range(o("a"), o("x"), 2)],
      ok=False)

    def e(src, pairs, data, start, end, kind, value, onechar=()):
        ex.append({"src": src, "pairs": [[o(x), o(y)] for x, y in pairs],
                   "onechar": [o(c) for c in onechar], "data": hx(data), "start": start,
                   "end": end, "kind": kind, "value": value})

    allb = b"b" * 61
    alle = b"e" * 61
    for i in range(16):
        e("shufti.cpp:482 ExecNoMatch1", [("a", "b")], allb, i, 61, "ge_end16", 0)
        e("shufti.cpp:503 ExecNoMatch1b", [("b", "a")], allb, i, 61, "ge", i + 15)
        e("shufti.cpp:524 ExecNoMatch2", [("a", "b"), ("B", "b")], allb, i, 61, "ge_end16", 0)
        e("shufti.cpp:546 ExecNoMatch2b", [("b", "a"), ("b", "B")], allb, i, 61, "ge", i + 15)
        e("shufti.cpp:568 ExecNoMatch3", [("V", "e")], alle, i, 61, "ge_end16", 0)
        e("shufti.cpp:589 ExecNoMatch3b", [("e", "V")], alle, i, 61, "ge", i + 15)
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbb"
    for i in range(16):
        e("shufti.cpp:610 ExecMatchShort1", [("a", "b")], t, i, len(t), "eq", 17)
    t = b"bbbbbbbbbbbbbbbbbabbbbbbbbbbbbbbbbbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        e("shufti.cpp:632 ExecMatch1", [("a", "b")], t, i, len(t), "eq", 17)
    t = b"bbbbbbbbbbbbbbbbbaaaaaaaaaaaaaaaabbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        e("shufti.cpp:654 ExecMatch2", [("a", "a")], t, i, len(t), "eq", 17)
    t = b"bbbbbbbbbbbbbbbbbBaaaaaaaaaaaaaaaabbbbbbbbbbbbbbbabbbbbbbbbbbb"
    for i in range(16):
        e("shufti.cpp:676 ExecMatch3", [("B", "a"), ("a", "a")], t, i, len(t), "eq", 17)
    p4 = [("A", "a"), ("a", "a"), ("C", "a"), ("c", "a")]
    p4b = [("a", "A"), ("a", "a"), ("a", "C"), ("a", "c")]
    for c in "ACca":
        t = b"b" * 17 + c.encode() + b"a" * 15 + b"b" * 15 + b"a" + b"b" * 11
        tb = b"b" * 17 + b"a" + c.encode() + b"a" * 14 + b"b" * 15 + b"a" + b"b" * 11
        for i in range(16):
            e("shufti.cpp:699 ExecMatch4", p4, t, i, len(t), "eq", 17)
            e("shufti.cpp:742 ExecMatch4b", p4b, tb, i, len(tb), "eq", 17)
    t = bytearray(b"b" * 76)
    for i in range(31):
        t[48 - i] = o("a")
        t[48 - i + 1] = o("A")
        e("shufti.cpp:785 ExecMatch5", [("a", "A")], bytes(t), 0, 76, "eq", 48 - i)
    t = bytearray(b"b" * 76)
    for i in range(31):
        t[48 - i] = o("a")
        e("shufti.cpp:808 ExecMatchMixed1", [], bytes(t), 0, 76, "eq", 48 - i, onechar="a")
    t = bytearray(b"b" * 76)
    for i in range(31):
        t[48 - i] = o("a")
        e("shufti.cpp:832 ExecMatchMixed2", [("x", "y")], bytes(t), 0, 76, "eq", 48 - i,
          onechar="a")
    t2 = bytearray(b"b" * 76)
    for i in range(31):
        t2[48 - i] = o("x")
        t2[48 - i + 1] = o("y")
        e("shufti.cpp:832 ExecMatchMixed2", [("x", "y")], bytes(t2), 0, 76, "eq", 48 - i,
          onechar="a")
    # Mixed3 :867-890 (len 420; t[len - i] written inside / just past the buffer)
    L = 420
    t = bytearray(b"b" * (L + 1))
    for i in range(1, 400):
        t[L - i] = o("a")
        e("shufti.cpp:867 ExecMatchMixed3", [("x", "y")], bytes(t[:L]), 0, L, "eq", L - i,
          onechar="a")
    t = bytearray(b"b" * (L + 2))
    for i in range(0, 400):
        t[L - i] = o("x")
        t[L - i + 1] = o("y")
        e("shufti.cpp:867 ExecMatchMixed3", [("x", "y")], bytes(t[:L]), 0, L, "eq", L - i,
          onechar="a")
    return {"build": build, "exec": ex}


def fdr_stream_cases():
    """unit/internal/fdr.cpp streaming known answers (safeExecStreaming
    :323-337 places a short history after '0123456789abcdef' filler so that
    16 bytes before its end are readable).  Ends are relative to buf."""
    cases = []

    def lit(s, nocase=0, id=0, noruns=0):
        return {"s": hx(s), "nocase": nocase, "id": id, "noruns": noruns}

    def add(src, lits, hist, data, expected, start=0, term_after=-1, hinted=True,
            status=0, expected_len=None):
        c = {"src": src, "lits": lits, "hist": hx(hist), "data": hx(data), "start": start,
             "term_after": term_after, "expected": expected, "hinted": hinted,
             "status": status}
        if expected_len is not None:
            c["expected_len"] = expected_len
        cases.append(c)

    l1 = [lit(b"a", 1, 1), lit(b"aardvark", 0, 10)]
    add("fdr.cpp:339 SmallStreaming", l1, b"", b"aaar", [[0, 1], [1, 1], [2, 1]])
    add("fdr.cpp:367 SmallStreaming", l1, b"aaar", b"dvark", [[2, 1], [4, 10]])
    l2 = [lit(b"a", 1, 1), lit(b"kk", 1, 2), lit(b"aardvark", 0, 10)]
    add("fdr.cpp:377 SmallStreaming2", l2, b"foobar", b"aardvarkkk",
        [[0, 1], [1, 1], [5, 1], [7, 10], [8, 2], [9, 2]])
    add("fdr.cpp:454 Stream1", [lit(b"f", 0, 0), lit(b"literal", 0, 1)],
        b"fffffffffffffffff", b"ffffuuuuuuuuuuuuu", [[0, 0], [1, 0], [2, 0], [3, 0]])
    # FDRTermS :697-717: default engine, callback terminates at the first match
    add("fdr.cpp:697 FDRTermS", [lit(b"f", 0, 0), lit(b"ff", 0, 1)], b"fffffffffffffffff",
        b"ffffuuuuuuuuuuuuu", None, term_after=1, hinted=False, status=1, expected_len=1)
    return cases


def _isalpha(c):
    return 0x41 <= c <= 0x5A or 0x61 <= c <= 0x7A


def fdr_flood_cases():
    """unit/internal/fdr_flood.cpp:148-560 (FDRFloodp, every char c, the
    engine built with the default Grey, i.e. flood detection on): literal
    sets generated from c and the per-id match counts the tests assert over
    a 1024-byte buffer filled with c (and with cAlt = c ^ bit).  Ids a test
    does not assert are absent from `expected`.  Literal = [s, nocase, id,
    msk, cmp] (hex strings)."""
    N = 1024
    out = []
    for c in range(256):
        bit = 1 << (c & 7)
        cAlt = c ^ bit
        cb = bit == 0x20 and _isalpha(c)  # bit == CASE_BIT && isalpha(c)

        # NoMask :148-233
        lits = []
        for i in range(4):
            L = 1 << i
            s = bytearray([c] * L)
            lits.append([hx(s), 0, i * 8 + 0, "", ""])
            s[0] = cAlt
            lits.append([hx(s), 0, i * 8 + 1, "", ""])
            lits.append([hx(s), 1, i * 8 + 2, "", ""])
            s[0] = c
            s[-1] = cAlt
            lits.append([hx(s), 0, i * 8 + 3, "", ""])
            lits.append([hx(s), 1, i * 8 + 4, "", ""])
            sa = bytearray([cAlt] * L)
            lits.append([hx(sa), 1, i * 8 + 5, "", ""])
            sa[0] = c
            lits.append([hx(sa), 1, i * 8 + 6, "", ""])
            lits.append([hx(sa), 0, i * 8 + 7, "", ""])
        exp_c, exp_alt = {}, {}
        for i in range(4):
            cnt = N - (1 << i) + 1
            one = cnt if i == 0 else 0
            exp_c.update({i * 8 + 0: cnt, i * 8 + 1: 0, i * 8 + 3: 0, i * 8 + 7: one})
            if cb:
                exp_c.update({i * 8 + k: cnt for k in (2, 4, 5, 6)})
            else:
                exp_c.update({i * 8 + 2: 0, i * 8 + 4: 0, i * 8 + 5: 0, i * 8 + 6: one})
            exp_alt.update({i * 8 + 0: 0, i * 8 + 1: one, i * 8 + 3: one, i * 8 + 5: cnt,
                            i * 8 + 7: 0})
            if cb:
                exp_alt.update({i * 8 + k: cnt for k in (2, 4, 6)})
            else:
                exp_alt.update({i * 8 + 2: one, i * 8 + 4: one, i * 8 + 6: 0})
        out.append({"src": "fdr_flood.cpp:148 NoMask", "c": c, "lits": lits,
                    "runs": [{"fill": c, "expected": exp_c}, {"fill": cAlt, "expected": exp_alt}]})

        # WithMask :235-402 (StreamingMask :404-558 builds the same set)
        lits = []
        s4, s4a = bytes([c] * 4), bytes([cAlt] * 4)
        for i in range(4):
            ml = 1 << i
            msk, cmp = bytearray(ml), bytearray(ml)
            cmp[0], msk[0] = cAlt, 0xFF

            def add(st, nc, k):
                lits.append([hx(st), nc, i * 12 + k, hx(msk), hx(cmp)])
            if ml > len(s4):
                add(s4, 0, 0)
                add(s4, 1, 1)
            if cb:
                add(s4, 1, 2)
            if (cAlt & bit) == 0:
                msk[0] = (~bit) & 0xFF
                add(s4, 0, 3)
                add(s4, 1, 4)
            cmp[0], msk[0] = c, 0xFF
            add(s4, 0, 5)
            add(s4, 1, 6)
            if ml > len(s4a):
                add(s4a, 0, 7)
                add(s4a, 1, 8)
            if cb:
                add(s4a, 1, 9)
                cmp[ml - 1], msk[ml - 1] = cAlt, 0xFF
                add(s4, 1, 10)
                cmp[0] = cAlt
                add(s4, 1, 11)
        cnt4 = N - 4 + 1
        exp_c, exp_alt = {}, {}
        for i in range(4):
            ml = 1 << i
            cm = min(cnt4, N - ml + 1)
            exp_c.update({i * 12 + 0: 0, i * 12 + 1: 0, i * 12 + 2: 0})
            if (cAlt & bit) == 0:
                exp_c.update({i * 12 + 3: cm, i * 12 + 4: cm})
            if ml > 4:
                exp_c.update({i * 12 + 5: cm, i * 12 + 6: cm, i * 12 + 7: 0,
                              i * 12 + 8: cm if cb else 0})
            else:
                exp_c.update({i * 12 + 5: cnt4, i * 12 + 6: cnt4})
            if cb:
                exp_c.update({i * 12 + 9: cm, i * 12 + 10: 0, i * 12 + 11: 0})
            exp_alt.update({i * 12 + k: 0 for k in (0, 3, 5, 6, 7, 8, 9)})
            if cb:
                exp_alt.update({i * 12 + 1: cm if ml > 4 else 0, i * 12 + 2: cm,
                                i * 12 + 4: cm if 0x61 <= c <= 0x7A else 0,
                                i * 12 + 10: cnt4 if ml == 1 else 0, i * 12 + 11: cm})
            else:
                exp_alt.update({i * 12 + k: 0 for k in (1, 2, 4, 10, 11)})
        out.append({"src": "fdr_flood.cpp:235 WithMask / :404 StreamingMask", "c": c,
                    "lits": lits, "stream": True,
                    "runs": [{"fill": c, "expected": exp_c}, {"fill": cAlt, "expected": exp_alt}]})
    return out


# ------------------------------------------------------- hs behaviour
def hs_behaviour_cases():
    """unit/hyperscan/behaviour.cpp, the rows whose pattern is a pure
    literal (no regex syntax, so hs_compile builds the same database as
    hs_compile_lit_multi of the literal with the same flags).  Inputs are
    the tests' construction rules (a zero-filled block with a pre-block and
    a post-block, runs of 'a', the corpus strings) with every size spelled
    out; expected values are the tests' own assertions.  Rows with regex
    syntax (foobar\\z, hatstand.*teakettle, ...) are out of scope: the
    pure-literal API refuses them."""
    HS_SCAN_TERMINATED = -3
    CASELESS = 1
    gig = [  # behaviour.cpp:301-303 (the pure-literal rows of gigTests)
        {"pattern": "foobar", "flags": 0, "pre": "flibble", "post": "foobar"},
        {"pattern": "longliteralislongerthanlong", "flags": 0, "pre": "precursor",
         "post": "longliteralislongerthanlong"},
    ]
    kib = [1, 4, 8, 16, 32, 64, 128, 256, 512, 1024]  # :261-265
    block = []
    for g in gig:
        # allocAndScanBlock :211-235: calloc(len), pre at 0, post at
        # len - strlen(post), hs_scan -> HS_SUCCESS and lastMatchTo == len;
        # three lengths per size :284-292
        lens = []
        for k in kib:
            b = k * 1024
            lens += [b, b + 4, b + len(g["post"])]
        block.append(dict(g, src="behaviour.cpp:241-299 (allocAndScanBlock :211-235)",
                          lens=lens, expected_status=0, expected_last_to=lens))
    # BIG_BLOCKS sizes (:266-273): 4, 32, 128, 512 MiB, 1, 2, 3 GiB, each
    # below UINT_MAX with the post-block (:280-282)
    big = [4 << 20, 32 << 20, 128 << 20, 512 << 20, 1 << 30, 2 << 30, 3 << 30]
    big_block = [dict(g, src="behaviour.cpp:266-273 (BIG_BLOCKS), :284-292", lens=big,
                      expected_status=0, expected_last_to=big) for g in gig]
    # StreamingMatch :137-208: pre-block, gb * 1024 writes of 1 MiB of 'X',
    # post-block, close; lastMatchTo stays 0 until the post-block; after the
    # close it equals pre + gb GiB + post.  gb = 1, 2 (debug build; 1..8
    # under NDEBUG)
    stream = []
    for g in gig:
        for gb in (1, 2):
            total = len(g["pre"]) + gb * 1024 * (1 << 20) + len(g["post"])
            stream.append(dict(g, src="behaviour.cpp:137-208", fill="X", chunk=1 << 20,
                               chunks=gb * 1024, expected_status=0,
                               expected_last_to_before_post=0,
                               expected_last_to_after_close=total))
    # LiteralLength FloatingBlock :404-440, sizes :481-483: pattern 'a' * L,
    # data 'a' * (L + 4): 5 matches; data[5:]: 0 matches
    lens = [1, 2, 3, 4, 8, 16, 17, 32, 100, 200, 400, 1000, 4096, 8192, 15000, 15999]
    floating = [{"src": "behaviour.cpp:404-440, 481-483", "literal_len": L, "data_len": L + 4,
                 "fill": "a", "expected_count": 5, "expected_count_from5": 0} for L in lens]
    # CallbackReturnStop Block / Streaming / Vectored :494-594, rows :596-599:
    # exactly one match and HS_SCAN_TERMINATED (the stream's close: HS_SUCCESS)
    stop = [{"src": "behaviour.cpp:494-599", "pattern": p, "flags": f, "corpus": c,
             "expected_count": 1, "expected_status": HS_SCAN_TERMINATED,
             "expected_close_status": 0}
            for p, f, c in [("foobar", 0, "xxxfoobarxxxfoobarxxxfoobar"),
                            ("a", 0, "xxxaaaaaaaaaaaaaaaaaaa"),
                            ("a", CASELESS, "xxxAaAaAaAa")]]
    # SerializedDogfood1 :613-662: serialize, free, deserialize; same
    # database size; hs_scan of "delicious puppy treats!" -> lastMatchTo = len
    dog = [{"src": "behaviour.cpp:613-662", "pattern": "puppy treats!", "flags": 0,
            "data": "delicious puppy treats!", "expected_size_equal": True,
            "expected_last_to": len("delicious puppy treats!")}]
    return {"block_gigabytes": block, "big_block": big_block, "stream_gigabytes": stream,
            "literal_length_floating": floating, "callback_stop": stop,
            "serialized_dogfood": dog}


def main():
    with open(os.path.join(HERE, "hs_behaviour.json"), "w") as f:
        json.dump(hs_behaviour_cases(), f, indent=1)
    with open(os.path.join(HERE, "noodle.json"), "w") as f:
        json.dump(noodle_cases(), f)
    with open(os.path.join(HERE, "fdr.json"), "w") as f:
        json.dump(fdr_cases(), f)
    with open(os.path.join(HERE, "fdr_shortwritings.json"), "w") as f:
        json.dump(short_writings_spec(), f)
    with open(os.path.join(HERE, "accel.json"), "w") as f:
        json.dump(accel_cases(), f)
    with open(os.path.join(HERE, "dshufti.json"), "w") as f:
        json.dump(dshufti_cases(), f)
    with open(os.path.join(HERE, "fdr_stream.json"), "w") as f:
        json.dump(fdr_stream_cases(), f)
    with open(os.path.join(HERE, "fdr_flood.json"), "w") as f:
        json.dump(fdr_flood_cases(), f, separators=(",", ":"))


if __name__ == "__main__":
    main()
