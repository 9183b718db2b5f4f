import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "liquid-dsp_amd"))

# The library computes single-sample calls on the host by default (small-call
# mode, host/lq_small.c).  The parity suite checks the GPU kernels, so it runs
# with every call forced onto the GPU; tests/test_gpu_small_calls.py switches
# the host path on per test.
os.environ["LQ_SMALL_CALLS"] = "gpu"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")
