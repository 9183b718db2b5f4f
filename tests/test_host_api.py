"""Host-only parts of the drop-in API that need no GPU: fft_shift (a
permutation of the caller's array, fft_common.c:336-350, pinned by
src/fft/tests/fft_shift_autotest.c) and liquid_nextpow2 (math.c:143-157)."""
import numpy as np

import liquidmi as LQ


def test_fft_shift_reference_cases():
    # fft_shift_autotest.c:27-72
    x4 = np.arange(4) * (1 + 1j)
    assert np.array_equal(LQ.fft_shift(x4), np.array([2, 3, 0, 1]) * (1 + 1j))
    x8 = np.arange(8) * (1 + 1j)
    assert np.array_equal(LQ.fft_shift(x8), np.array([4, 5, 6, 7, 0, 1, 2, 3]) * (1 + 1j))
    # odd n: the first (n-1)/2 swap with the next (n-1)/2, the last stays
    x5 = np.arange(5).astype(complex)
    assert np.array_equal(LQ.fft_shift(x5), np.array([2, 3, 0, 1, 4]))


def test_nextpow2():
    L = LQ.lib()
    for x, e in [(1, 0), (2, 1), (3, 2), (4, 2), (5, 3), (1024, 10), (1025, 11), (2**31, 31)]:
        assert L.liquid_nextpow2(x) == e
