"""Synthetic BSC trials: exactly floor(n*QBER) flips (src/array_and_matrix_operations.cpp:905-933)."""
import numpy as np

from qkd_ldpc_v_amd import bsc_frames


def test_exact_flip_count_and_accurate_qber():
    for n, q in ((10240, 0.0215), (1024, 0.013), (6, 0.2)):
        a, b, acc = bsc_frames(n, q, 7, seed=3)
        k = int(n * q)
        assert acc == k / n
        assert np.all((a ^ b).sum(axis=1) == k)
        assert set(np.unique(a)) <= {0, 1}


def test_seeded():
    a1, b1, _ = bsc_frames(512, 0.05, 3, seed=9)
    a2, b2, _ = bsc_frames(512, 0.05, 3, seed=9)
    assert np.array_equal(a1, a2) and np.array_equal(b1, b2)
