"""LD_PRELOAD interposition (`-m gpu`).

build/preload/prog is a liquid-dsp program already linked against a
libliquid.so (a stand-in exporting the symbols it calls and marking each call
on stderr: tests/preload/liquid_stub.c -- the reference library itself is not
built in this image).  Run with LD_PRELOAD=libliquid_mi355x.so, every one of
those calls must be served by this library instead (no stub marks) and give
the convolution and dot product the program asks for.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROG = os.path.join(ROOT, "build", "preload", "prog")
LIB = os.path.join(ROOT, "liquid-dsp_amd", "lib", "libliquid_mi355x.so")


def _expected():
    h = np.array([0.1 * (i + 1) for i in range(9)], np.float32)
    x = np.array([(i % 7) - 3.0 + 1j * (i % 5) for i in range(32)], np.complex64)
    y = np.convolve(x.astype(np.complex128), h.astype(np.float64))[:32]
    d = np.sum(h * x[:9])
    return y, d


@pytest.mark.skipif(not os.path.exists(PROG), reason="build/preload not built (tools/build_preload_test.sh)")
def test_preload_takes_over_an_already_linked_program():
    stub = subprocess.run([PROG], capture_output=True, text=True, timeout=60)
    assert stub.returncode == 0 and "STUB firfilt_crcf_create" in stub.stderr
    # appended to whatever the environment already preloads (left in place)
    pre = os.environ.get("LD_PRELOAD", "")
    env = dict(os.environ, LD_PRELOAD=(pre + " " + LIB).strip())
    out = subprocess.run([PROG], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr
    assert "STUB" not in out.stderr
    vals = np.array([[float(v) for v in ln.split()] for ln in out.stdout.split("\n") if ln.strip()])
    got = vals[:, 0] + 1j * vals[:, 1]
    y, d = _expected()
    assert np.max(np.abs(got[:32] - y)) < 1e-4
    assert abs(got[32] - d) < 1e-4
