"""Loader for the committed golden fixtures (tests/golden/*.json)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)["data"]


def arr(v):
    """JSON list -> float32 (real) or complex64 ([re, im] pairs) array."""
    if isinstance(v, list) and v and isinstance(v[0], list):
        a = np.asarray(v, dtype=np.float64)
        return (a[:, 0] + 1j * a[:, 1]).astype(np.complex64)
    if isinstance(v, list) and len(v) == 2 and isinstance(v[0], float) and False:
        pass
    return np.asarray(v, dtype=np.float32)


def scalar(v):
    if isinstance(v, list):
        return complex(v[0], v[1])
    return float(v)


def nrm_err(y, ref):
    """Normwise error max|y-ref| / max|ref| (the parity metric)."""
    y = np.asarray(y)
    ref = np.asarray(ref)
    den = np.max(np.abs(ref)) if ref.size else 1.0
    return float(np.max(np.abs(y.astype(np.complex128) - ref.astype(np.complex128))) / (den if den > 0 else 1.0)) \
        if ref.size else 0.0
