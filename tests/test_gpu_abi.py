"""The drop-ins called from plain C through their real reference
signatures (__m128i masks in XMM registers): tests/c/abi_harness.c links
libvectorscan_amd.so and the test-only oracle and compares every call
(shufti / rshufti / truffle / rtruffle / the vermicelli family incl.
vermicelliDoubleMaskedExec / shuftiDoubleExec / run_accel over every
AccelAux scheme, accel.c:36-183) on random buffers at random alignments."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "c", "abi_harness")


def test_harness_built():
    assert os.path.exists(HARNESS), "build with make (tests/c/abi_harness)"


@pytest.mark.gpu
def test_gpu_c_abi_harness():
    r = subprocess.run([HARNESS, "300"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout, r.stdout


def test_hwlm_registration_host_side():
    """vsa_hwlm_register / unregister (host bookkeeping, no GPU): register
    accepts an HWLM (-1) or a bare FDR / noodle engine type, unregister of a
    blob that is not registered is an error"""
    import bench
    import vectorscan_amd as vsa
    b = vsa.hwlm_build(bench.make_literals(50, seed=1))
    vsa.hwlm_register(b)
    vsa.hwlm_unregister(b)
    with pytest.raises(Exception):
        vsa.hwlm_unregister(b)
    with pytest.raises(Exception):
        vsa.hwlm_register(b, 7)  # not an engine type


HS_NAMES = os.path.join(ROOT, "tests", "c", "hs_names_demo")


def test_hs_names_header_compiles_strict():
    """include/vectorscan_amd_hs_names.h: a program written against the
    reference's hs names (tests/c/hs_names_demo.c) compiles with every
    warning as an error, C and C++, and the built demo exists (make all)."""
    src = os.path.join(ROOT, "tests", "c", "hs_names_demo.c")
    for cc, std in (("gcc", "-std=gnu11"), ("g++", "-std=c++17")):
        lang = ["-x", "c++"] if cc == "g++" else []
        r = subprocess.run([cc, std, *lang, "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                            "-I" + os.path.join(ROOT, "include"), src],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
    assert os.path.exists(HS_NAMES), "build with make (tests/c/hs_names_demo)"


@pytest.mark.gpu
def test_gpu_hs_names_demo():
    """The hs-names program run on the GPU: block scan, a deserialized copy,
    a stream of 1,000-byte writes and a vectored scan each give exactly the
    brute-force match set of its 4 MiB buffer."""
    r = subprocess.run([HS_NAMES, str(4 << 20)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK"), r.stdout
