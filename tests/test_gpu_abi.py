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
