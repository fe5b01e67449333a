"""Shared test setup.  GPU tests are marked `gpu`; everything else runs on CPU."""
import contextlib
import gzip
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
MATRICES = os.path.join(GOLDEN, "matrices")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@contextlib.contextmanager
def diag_env(**knobs):
    """Set QLDPC_* A/B knobs under the diagnostic switch QLDPC_DIAG=1 (the
    library ignores them otherwise) and restore the environment after."""
    keys = ["QLDPC_DIAG"] + list(knobs)
    old = {k: os.environ.get(k) for k in keys}
    os.environ.update(QLDPC_DIAG="1", **knobs)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def matrix_path(name: str) -> str:
    return os.path.join(MATRICES, name + ".gz")


def manifest() -> dict:
    with open(os.path.join(MATRICES, "MANIFEST.json")) as f:
        return json.load(f)


_cache = {}


def load_fixture(name: str):
    """HMatrix of a committed matrix fixture, through the product loader."""
    if name not in _cache:
        from qkd_ldpc_v_amd import load_matrix

        _cache[name] = load_matrix(matrix_path(name), manifest()[name]["format"])
    return _cache[name]


def kat() -> dict:
    with open(os.path.join(GOLDEN, "kat_johnson.json")) as f:
        return json.load(f)


def bits_equal_nan(a: np.ndarray, b: np.ndarray) -> bool:
    """Bitwise equality of float64 arrays, NaNs equal to each other."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a.view(np.uint64)[~na], b.view(np.uint64)[~nb])


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (run on the MI355X box)")
    return True
