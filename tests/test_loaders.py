"""Matrix readers (reference src/array_and_matrix_operations.cpp:291-886)
through the product library, on the committed fixtures and on malformed files."""
import gzip
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import MATRICES, ROOT, load_fixture, manifest, matrix_path
from qkd_ldpc_v_amd import QLDPCError, load_matrix


def test_fixtures_round_trip_to_reference_bytes():
    for name, meta in manifest().items():
        data = gzip.open(matrix_path(name)).read()
        assert hashlib.sha256(data).hexdigest() == meta["sha256"], name


EXPECTED = {  # name: (n, m, nnz, is_regular)
    "kat_n6_m4.dense": (6, 4, 12, True),
    "u_n7_m3.dense": (7, 3, None, None),
    "s1_n10_m5.sp1": (10, 5, 12, False),
    "c1_n1024_m220.alist": (1024, 220, 5120, False),
    "c2_n10240_m2201.alist": (10240, 2201, 40960, False),
    "c3_n10240_m1801.alist": (10240, 1801, 40960, False),
    "c5_n10240_m2048.sp2": (10240, 2048, 60430, False),
}


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_shapes(name):
    H = load_fixture(name)
    n, m, nnz, reg = EXPECTED[name]
    assert (H.n, H.m) == (n, m)
    if nnz is not None:
        assert H.nnz == nnz
    if reg is not None:
        assert H.is_regular == reg
    # bit_nodes is the ascending transpose of check_nodes for every shipped file
    T = [[] for _ in range(H.n)]
    for j, row in enumerate(H.check_nodes):
        assert row == sorted(row)
        for i in row:
            T[i].append(j)
    assert T == H.bit_nodes


def _py_alist(text):
    lines = [list(map(int, l.split())) for l in text.splitlines()]
    n, m = lines[0]
    cw, rw = lines[2], lines[3]
    bits = [[x - 1 for x in lines[4 + i][: cw[i]]] for i in range(n)]
    checks = [[x - 1 for x in lines[4 + n + j][: rw[j]]] for j in range(m)]
    return bits, checks


def test_alist_against_python_parser():
    text = gzip.open(matrix_path("c2_n10240_m2201.alist")).read().decode()
    bits, checks = _py_alist(text)
    H = load_fixture("c2_n10240_m2201.alist")
    assert H.bit_nodes == bits and H.check_nodes == checks


def test_untp_fixture_indices_in_range():
    idx = list(map(int, gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split()))
    assert len(idx) > 0 and min(idx) >= 0 and max(idx) < 10240 and len(set(idx)) == len(idx)


@pytest.mark.parametrize("content,fmt,msg", [
    ("1 0 2\n0 1 1\n", 0, "can only take values"),
    ("1 0 1\n0 1\n", 0, "Different lengths of rows"),
    ("1 0 0\n0 1 0\n", 0, "Column '3' weight cannot be equal to zero"),
    ("3 2\n", 1, "Insufficient data"),
    ("3 2 1\n1 2\n1 1 1\n2 1\n1\n1\n2\n1 2\n3 0\n", 1, "Wrong sparse alist matrix format"),
    ("3 2\n1 2\n1 1 1\n2 1\n1\n2 3\n1\n1 2\n3 0\n", 1, "does not match the weight in the third line"),
    ("3\n2\n2\n1 2 3\n3 0\n", 2, "exceeded the maximum specified weight"),
    ("3 2\n0 1\n-1 2\n0\n0\n1\n", 3, "cannot be less than zero"),
])
def test_loader_errors(tmp_path, content, fmt, msg):
    p = tmp_path / "bad.mtrx"
    p.write_text(content)
    with pytest.raises(QLDPCError) as e:
        load_matrix(str(p), fmt)
    assert msg in str(e.value)


def test_missing_file():
    with pytest.raises(QLDPCError, match="Failed to open file"):
        load_matrix("/nonexistent/x.mtrx", 1)


def test_host_mirror_program_loads(tmp_path):
    exe = os.path.join(ROOT, "qkd_ldpc_v_amd", "host", "host_mirror_check")
    r = subprocess.run([exe, "load", matrix_path("c2_n10240_m2201.alist"), "1"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.split() == ["10240", "2201", "40960", "0"]
    r = subprocess.run([exe, "load", "/nonexistent", "1"], capture_output=True, text=True)
    assert r.returncode == 1 and "ERROR: Failed to open file" in r.stdout


def test_generated_regular_code():
    """codes.regular_code (the C4 (ii) stand-in): exact degrees, distinct rows
    per bit, ascending adjacency, deterministic per seed."""
    import numpy as np
    import qkd_ldpc_v_amd as Q

    H = Q.regular_code(4000, 861, 4, 777)
    assert (H.n, H.m, H.nnz) == (4000, 861, 16000)
    assert set(np.diff(H.col_ptr)) == {4}
    dc = np.diff(H.row_ptr)
    assert dc.max() - dc.min() <= 1
    for j in range(H.m):
        r = H.col_idx[H.row_ptr[j]:H.row_ptr[j + 1]]
        assert (np.diff(r) > 0).all()
    H2 = Q.regular_code(4000, 861, 4, 777)
    assert np.array_equal(H.col_idx, H2.col_idx)
    assert not np.array_equal(H.col_idx, Q.regular_code(4000, 861, 4, 778).col_idx)
