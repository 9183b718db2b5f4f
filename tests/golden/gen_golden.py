#!/usr/bin/env python3
"""Extract the reference's own golden vectors into JSON fixtures.

Runs ONLY in the build container (it reads /root/reference as text); the GPU
box and the test-suite read the committed JSON files, never the reference.

What is extracted (all of it data: coefficient, input and expected-output
arrays, plus the tolerances the reference's runners apply):

  * firfilt  : src/filter/tests/data/firfilt_{rrrf,crcf,cccf}_data_h*.c
               (runner src/filter/tests/firfilt_runtest.c:68-95, tol 1e-3)
  * firdecim : src/filter/tests/data/firdecim_*_data_M*.c
               (runner src/filter/tests/firdecim_runtest.c:78-93, tol 1e-3)
  * fftfilt  : src/filter/tests/data/fftfilt_*_data_h*x256.c
               (runner src/filter/tests/fftfilt_runtest.c:83-120, tol 1e-3,
               block n = 1 << liquid_nextpow2(h_len-1))
  * fft      : src/fft/tests/data/fft_data_*.c
               (runner src/fft/tests/fft_runtest.c:30-67, tol 2e-4 on |y-test|)
  * known-answer arrays embedded in autotests:
      dotprod  src/dotprod/tests/dotprod_{rrrf,crcf,cccf}_autotest.c
      firinterp src/filter/tests/firinterp_autotest.c:29-150
      firpfb   src/filter/tests/firpfb_autotest.c:26-73
  * fft_r2r  : src/fft/tests/data/fft_r2rdata_{8,27,32}.c (DCT/DST I-IV, tol 1e-4)
  * firdes   : rcos / rrcos coefficient arrays (src/filter/tests/firdes_autotest.c:25-95,
               tol 1e-5) and Parks-McClellan designs with their band specs
               (src/filter/tests/firdespm_autotest.c:26-140, tol 1e-4)

Usage:  python tests/golden/gen_golden.py [/root/reference]
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?"
CPLX = re.compile(r"(" + NUM + r")\s*([-+])\s*(" + NUM + r")\s*\*\s*_Complex_I")
ARRAY = re.compile(r"(float complex|float)\s+(\w+)\s*\[\s*\w*\s*\]\s*=\s*\{(.*?)\}\s*;", re.S)
SCALAR = re.compile(r"(float complex|float)\s+(\w+)\s*=\s*([^;{]+);")


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _parse_complex(tok):
    tok = tok.strip()
    m = CPLX.fullmatch(tok)
    if m:
        re_, sign, im = m.groups()
        im = float(im)
        return [float(re_), -im if sign == "-" else im]
    # "a + b * _Complex_I" with spaces around '*', or pure real
    m2 = re.fullmatch(r"(" + NUM + r")", tok)
    if m2:
        return [float(tok), 0.0]
    raise ValueError("cannot parse complex literal: %r" % tok)


def _split_items(body):
    return [t for t in (s.strip() for s in body.split(",")) if t]


def parse_arrays(src):
    src = _strip_comments(src)
    out = {}
    for kind, name, body in ARRAY.findall(src):
        items = _split_items(body)
        if kind == "float complex":
            out[name] = [_parse_complex(t) for t in items]
        else:
            out[name] = [float(t.rstrip("f")) for t in items]
    return out


def parse_function_bodies(src):
    """Map autotest function name -> body text (brace matched)."""
    src = _strip_comments(src)
    res = {}
    for m in re.finditer(r"void\s+(autotest_\w+)\s*\(\s*\)\s*\{", src):
        i = m.end()
        depth = 1
        while depth:
            if src[i] == "{":
                depth += 1
            elif src[i] == "}":
                depth -= 1
            i += 1
        res[m.group(1)] = src[m.end():i - 1]
    return res


def parse_scalars(body):
    out = {}
    for kind, name, expr in SCALAR.findall(body):
        expr = expr.strip().rstrip("f")
        try:
            if kind == "float complex":
                expr2 = re.sub(r"\s+", " ", expr)
                out[name] = _parse_complex(expr2.replace(" * _Complex_I", "*_Complex_I"))
            else:
                out[name] = float(expr)
        except ValueError:
            pass
    return out


def read(path):
    with open(os.path.join(REF, path)) as f:
        return f.read()


def gen_filter_data(family):
    d = os.path.join(REF, "src/filter/tests/data")
    cases = []
    for fn in sorted(os.listdir(d)):
        if not fn.startswith(family + "_") or not fn.endswith(".c"):
            continue
        arr = parse_arrays(read(os.path.join("src/filter/tests/data", fn)))
        stem = fn[:-2]
        typ = stem.split("_")[1]
        case = {"name": stem, "type": typ, "source": "src/filter/tests/data/" + fn,
                "h": arr[stem + "_h"], "x": arr[stem + "_x"], "y": arr[stem + "_y"],
                "tol": 1e-3}
        if family == "firdecim":
            case["M"] = int(re.search(r"_M(\d+)h", stem).group(1))
        cases.append(case)
    return cases


def gen_fft():
    d = os.path.join(REF, "src/fft/tests/data")
    cases = []
    for fn in sorted(os.listdir(d), key=lambda s: (len(s), s)):
        m = re.fullmatch(r"fft_data_(\d+)\.c", fn)
        if not m:
            continue
        n = int(m.group(1))
        arr = parse_arrays(read("src/fft/tests/data/" + fn))
        cases.append({"n": n, "x": arr["fft_test_x%d" % n], "y": arr["fft_test_y%d" % n],
                      "source": "src/fft/tests/data/" + fn, "tol": 2e-4})
    return cases


def gen_known_answers():
    ka = {}
    # dotprod crcf (src/dotprod/tests/dotprod_crcf_autotest.c:29-107)
    b = parse_function_bodies(read("src/dotprod/tests/dotprod_crcf_autotest.c"))
    for fname in ("autotest_dotprod_crcf_rand01", "autotest_dotprod_crcf_rand02"):
        body = b[fname]
        arr = parse_arrays(body)
        sc = parse_scalars(body)
        ka[fname] = {"type": "crcf", "h": arr["h"], "x": arr["x"], "y": sc["test"], "tol": 1e-3,
                     "source": "src/dotprod/tests/dotprod_crcf_autotest.c"}
    # dotprod cccf (src/dotprod/tests/dotprod_cccf_autotest.c:33-78)
    b = parse_function_bodies(read("src/dotprod/tests/dotprod_cccf_autotest.c"))
    body = b["autotest_dotprod_cccf_rand16"]
    arr = parse_arrays(body)
    sc = parse_scalars(body)
    ka["autotest_dotprod_cccf_rand16"] = {"type": "cccf", "h": arr["h"], "x": arr["x"],
                                          "y": sc["test"], "tol": 1e-3,
                                          "source": "src/dotprod/tests/dotprod_cccf_autotest.c"}
    # dotprod rrrf (src/dotprod/tests/dotprod_rrrf_autotest.c:31-257)
    b = parse_function_bodies(read("src/dotprod/tests/dotprod_rrrf_autotest.c"))
    for fname in ("autotest_dotprod_rrrf_rand01", "autotest_dotprod_rrrf_rand02"):
        body = b[fname]
        arr = parse_arrays(body)
        sc = parse_scalars(body)
        ka[fname] = {"type": "rrrf", "h": arr["h"], "x": arr["x"], "y": sc["test"], "tol": 1e-3,
                     "source": "src/dotprod/tests/dotprod_rrrf_autotest.c"}
    body = b["autotest_dotprod_rrrf_basic"]
    arr = parse_arrays(body)
    sc = parse_scalars(body)
    cases = []
    for k in range(4):
        cases.append({"x": arr["x%d" % k], "y": sc["test%d" % k]})
    cases.append({"x": arr["h"], "y": sc["test4"]})
    ka["autotest_dotprod_rrrf_basic"] = {"type": "rrrf", "h": arr["h"], "cases": cases, "tol": 1e-6,
                                         "source": "src/dotprod/tests/dotprod_rrrf_autotest.c"}
    # firinterp (src/filter/tests/firinterp_autotest.c:29-150), M = 4
    b = parse_function_bodies(read("src/filter/tests/firinterp_autotest.c"))
    for fname, typ in (("autotest_firinterp_rrrf_generic", "rrrf"),
                       ("autotest_firinterp_crcf_generic", "crcf")):
        arr = parse_arrays(b[fname])
        ka[fname] = {"type": typ, "M": 4, "h": arr["h"], "x": arr["x"], "y": arr["test"],
                     "tol": 1e-6, "source": "src/filter/tests/firinterp_autotest.c"}
    # firpfb impulse response (src/filter/tests/firpfb_autotest.c:26-73), M = 4 filters
    b = parse_function_bodies(read("src/filter/tests/firpfb_autotest.c"))
    arr = parse_arrays(b["autotest_firpfb_impulse_response"])
    ka["autotest_firpfb_impulse_response"] = {"type": "rrrf", "M": 4, "h": arr["h"],
                                              "x": arr["noise"], "y": arr["test"], "tol": 1e-4,
                                              "source": "src/filter/tests/firpfb_autotest.c"}
    return ka


def gen_fft_r2r():
    """src/fft/tests/data/fft_r2rdata_{8,27,32}.c (runner fft_r2r_autotest.c:27-48, tol 1e-4)"""
    out = []
    codes = {"REDFT00": 10, "REDFT10": 11, "REDFT01": 12, "REDFT11": 13,
             "RODFT00": 20, "RODFT10": 21, "RODFT01": 22, "RODFT11": 23}
    for n in (8, 27, 32):
        arr = parse_arrays(read("src/fft/tests/data/fft_r2rdata_%d.c" % n))
        x = arr["fftdata_r2r_x%d" % n]
        for name, code in codes.items():
            key = "fftdata_r2r_%s_y%d" % (name, n)
            if key in arr:
                out.append({"name": "%s_n%d" % (name, n), "n": n, "type": code, "x": list(x),
                            "y": list(arr[key]), "tol": 1e-4,
                            "source": "src/fft/tests/data/fft_r2rdata_%d.c" % n})
    return out


def gen_firdes():
    out = {}
    b = parse_function_bodies(read("src/filter/tests/firdes_autotest.c"))
    for fname, kind in (("autotest_liquid_firdes_rcos", "rcos"), ("autotest_liquid_firdes_rrcos", "rrcos")):
        body = b[fname]
        arr = parse_arrays(body)
        sc = {k: float(v) for k, v in re.findall(r"\b(beta|offset)\s*=\s*(" + NUM + r")f?", body)}
        k, m = (int(v) for v in re.search(r"unsigned int k\s*=\s*(\d+),\s*m\s*=\s*(\d+)", body).groups())
        out[fname] = {"design": kind, "k": k, "m": m, "beta": sc["beta"], "dt": sc["offset"],
                      "h": list(arr["h0"]), "tol": 1e-5,
                      "source": "src/filter/tests/firdes_autotest.c"}
    b = parse_function_bodies(read("src/filter/tests/firdespm_autotest.c"))
    for fname, body in b.items():
        arr = parse_arrays(body)
        n = int(re.search(r"unsigned int n\s*=\s*(\d+)", body).group(1))
        out[fname] = {"design": "firdespm", "n": n, "bands": list(arr["bands"]),
                      "des": list(arr["des"]), "weights": list(arr["weights"]),
                      "h": list(arr["h0"]), "tol": 1e-4,
                      "source": "src/filter/tests/firdespm_autotest.c"}
    return out


def main():
    fixtures = {
        "firdes": gen_firdes(),
        "fft_r2r": gen_fft_r2r(),
        "firfilt": gen_filter_data("firfilt"),
        "firdecim": gen_filter_data("firdecim"),
        "fftfilt": gen_filter_data("fftfilt"),
        "fft": gen_fft(),
        "known_answers": gen_known_answers(),
    }
    for k, v in fixtures.items():
        path = os.path.join(OUT, k + ".json")
        with open(path, "w") as f:
            json.dump({"generated_by": "tests/golden/gen_golden.py", "reference": "liquid-dsp 1.2.0",
                       "data": v}, f, separators=(",", ":"))
        print("wrote", path, len(v))


if __name__ == "__main__":
    main()
