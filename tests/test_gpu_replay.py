"""Host replay semantics of the drop-in hwlmExec / fdrExec that only a Rose
callback exercises: the INCLUDED_JUMP squash of later buckets at the same
end through scratch->fdr_conf (program_runtime.c:2985-2997,
fdr_confirm_runtime.h:62-64, :101), against the oracle's restatement."""
import ctypes
import random

import numpy as np
import pytest

import oracle
import vectorscan_amd as vsa
from test_cpu_oracle import rand_data, rand_lits

M64 = (1 << 64) - 1


def squash_case(seed, nlits):
    rng = random.Random(seed)
    # short literals over a small alphabet: many ends carry several buckets
    lits = rand_lits(rng, nlits, minlen=1, maxlen=6, alphabet=b"abcd", msk_frac=0.0)
    for l in lits:
        l.noruns = rng.random() < 0.2
    squash = {l.id: rng.choice([0, 0, 0xff, rng.randrange(256)]) for l in lits}
    data = rand_data(rng, 20000, alphabet=b"abcdab")
    return lits, squash, data


def test_oracle_squash_is_per_end_prefix():
    """CPU: squashing only ever drops later candidates at the same end, so
    each end's report list is a prefix of the unsquashed one, and squashing
    everything leaves one bucket per end."""
    lits, _, data = squash_case(1, 40)
    for l in lits:
        l.noruns = False  # NOREPEAT state would differ once reports are squashed
    blob = vsa.hwlm_build(lits, engine_hint=0)
    eng = vsa.engine_blob(blob)
    _, full = oracle.fdr_exec(eng, data, cap=1 << 20)
    _, sq = oracle.fdr_exec_squash(eng, data, {l.id: 0xff for l in lits}, cap=1 << 20)
    by = {}
    for e, i in full:
        by.setdefault(e, []).append(i)
    got = {}
    for e, i in sq:
        got.setdefault(e, []).append(i)
    assert set(got) <= set(by)
    shorter = 0
    for e, ids in got.items():
        assert by[e][:len(ids)] == ids
        shorter += len(ids) < len(by[e])
    assert shorter > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,nlits", [(1, 40), (2, 12), (3, 200), (4, 1000)])
def test_gpu_included_jump_squash(seed, nlits):
    lits, squash, data = squash_case(seed, nlits)
    blob = vsa.hwlm_build(lits, engine_hint=0)
    eng = vsa.engine_blob(blob)
    _, want = oracle.fdr_exec_squash(eng, data, squash, cap=1 << 20)
    _, plain = oracle.fdr_exec(eng, data, cap=1 << 20)
    assert want != plain  # the squash changes the stream

    # a scratch image with fdr_conf at +8 and fdr_conf_offset at +16
    old = (ctypes.c_long(), ctypes.c_long())
    vsa.lib.vsa_get_scratch_layout(ctypes.byref(old[0]), ctypes.byref(old[1]))
    vsa.lib.vsa_set_scratch_layout(8, 16)
    scratch = ctypes.create_string_buffer(64)
    base = ctypes.addressof(scratch)
    seq = []

    def cb(end, id_, scr):
        seq.append((end, id_))
        sq = squash.get(id_, 0)
        conf_p = ctypes.c_uint64.from_address(base + 8).value
        if sq and conf_p:
            off = ctypes.c_uint8.from_address(base + 16).value
            w = ctypes.c_uint64.from_address(conf_p)
            w.value &= ((~sq) << (off & ~7)) & M64
        return vsa.HWLM_ALL_GROUPS

    ccb = vsa.HWLMCallback(cb)
    try:
        keep = ctypes.create_string_buffer(bytes(data), len(data))
        rc = vsa.lib.fdrExec(eng, keep, len(data), 0, ccb, base, vsa.HWLM_ALL_GROUPS)
    finally:
        vsa.lib.vsa_set_scratch_layout(old[0].value, old[1].value)
    assert rc == 0
    assert ctypes.c_uint64.from_address(base + 8).value == 0  # cleared after each callback
    assert seq == want
