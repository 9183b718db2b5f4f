"""The drop-in boundary, checked without a GPU.

* the C-ABI library builds for gfx950 and loads;
* it exports every function include/liquid_mi355x.h declares;
* the header compiles as C99 and as C++ (std::complex), like liquid.h;
* a C program written against liquid.h's API compiles and links against it
  unchanged (examples/ is the drop-in smoke test).
No compute call is made here (no GPU in the build container).
"""
import ctypes as C
import os
import subprocess
import sys

import pytest

import liquidmi as LQ

ROOT = LQ.ROOT


def test_library_builds_and_loads():
    LQ.build()
    assert os.path.exists(LQ.LIB_PATH)
    assert LQ.lib().liquid_libversion_number() == 1002000


def test_exports_every_declared_symbol():
    names = LQ.header_functions()
    assert len(names) > 100
    L = C.CDLL(LQ.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_liquid_h_hot_path_symbols_present():
    # the liquid.h symbols SURVEY 8(b) lists for the implemented objects
    expected = []
    for t in ("rrrf", "crcf", "cccf"):
        expected += ["dotprod_%s_%s" % (t, s) for s in
                     ("run", "run4", "create", "recreate", "destroy", "print", "execute")]
        expected += ["firfilt_%s_%s" % (t, s) for s in
                     ("create", "create_kaiser", "create_rect", "recreate", "destroy", "reset", "print",
                      "set_scale", "push", "execute", "execute_block", "get_length")]
    expected += ["firdecim_crcf_%s" % s for s in
                 ("create", "create_kaiser", "destroy", "print", "clear", "execute", "execute_block")]
    expected += ["firinterp_crcf_%s" % s for s in
                 ("create", "create_kaiser", "destroy", "print", "reset", "execute", "execute_block")]
    expected += ["fftfilt_crcf_%s" % s for s in
                 ("create", "destroy", "reset", "print", "set_scale", "execute", "get_length")]
    expected += ["firpfbch_crcf_%s" % s for s in
                 ("create", "create_kaiser", "destroy", "reset", "print", "synthesizer_execute",
                  "analyzer_execute")]
    expected += ["firpfbch2_crcf_%s" % s for s in
                 ("create", "create_kaiser", "destroy", "reset", "print", "execute")]
    expected += ["liquid_firdes_kaiser", "kaiser_beta_As", "liquid_libversion", "liquid_libversion_number",
                 "liquid_msb_index"]
    L = C.CDLL(LQ.LIB_PATH)
    missing = [n for n in expected if not hasattr(L, n)]
    assert not missing, missing


def test_header_compiles_as_c_and_cxx(tmp_path):
    inc = os.path.join(ROOT, "include")
    c = tmp_path / "t.c"
    c.write_text('#include "liquid_mi355x.h"\nint main(void){return 0;}\n')
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-I", inc, str(c)])
    cc = tmp_path / "t.cc"
    cc.write_text('#include <complex>\n#include "liquid_mi355x.h"\nint main(){return 0;}\n')
    subprocess.check_call(["g++", "-std=c++11", "-Wall", "-fsyntax-only", "-I", inc, str(cc)])


@pytest.mark.parametrize("src", sorted(f for f in os.listdir(os.path.join(ROOT, "examples")) if f.endswith(".c")))
def test_examples_compile_and_link(src, tmp_path):
    inc = os.path.join(ROOT, "include")
    libdir = os.path.dirname(LQ.LIB_PATH)
    out = tmp_path / "a.out"
    subprocess.check_call(["gcc", "-std=gnu99", "-O2", "-Wall", "-I", inc, os.path.join(ROOT, "examples", src),
                           "-L", libdir, "-lliquid_mi355x", "-Wl,-rpath," + libdir, "-lm", "-o", str(out)])
    assert out.exists()


@pytest.mark.skipif(not os.path.isdir("/root/reference/examples"), reason="reference sources not present")
def test_reference_examples_compile_unchanged():
    """liquid-dsp's own examples for this path compile and link, unchanged,
    against include/liquid.h + libliquid_mi355x (tools/build_ref_examples.sh)."""
    subprocess.check_call(["bash", os.path.join(ROOT, "tools", "build_ref_examples.sh")])
    built = os.listdir(os.path.join(ROOT, "build", "ref_examples"))
    assert len(built) == 25


def test_liquid_msb_index_known_answers():
    """src/utility/tests/count_bits_autotest.c:140-177: msb_index(0) = 0,
    msb_index(2^k) = k + 1; plus the table in msb_index.c:90-108 (255 -> 8).
    Host-side integer helper (no GPU call)."""
    f = C.CDLL(LQ.LIB_PATH).liquid_msb_index
    f.restype, f.argtypes = C.c_uint, [C.c_uint]
    assert f(0) == 0
    for k in range(32):
        assert f(1 << k) == k + 1
    for x, b in ((3, 2), (126, 7), (127, 7), (128, 8), (129, 8), (253, 8), (255, 8), (0xFFFFFFFF, 32)):
        assert f(x) == b


@pytest.mark.parametrize("env,expect", [(None, 1), ("gpu", 0), ("0", 0), ("host", 1)])
def test_small_call_mode_default(env, expect):
    """Single-sample calls run on the host unless LQ_SMALL_CALLS=gpu (or 0):
    the mode the library reads at load, in a fresh process (no GPU needed)."""
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); "
            "print(L.liquid_mi355x_get_small_calls())")
    e = dict(os.environ)
    e.pop("LQ_SMALL_CALLS", None)
    if env is not None:
        e["LQ_SMALL_CALLS"] = env
    out = subprocess.run([sys.executable, "-c", code, LQ.LIB_PATH], capture_output=True, text=True, env=e,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    assert int(out.stdout.strip()) == expect
