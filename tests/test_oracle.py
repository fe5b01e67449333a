"""The CPU oracle (oracle/ldpc_oracle.c) against the reference's golden KAT and
against an independent pure-Python restatement (tests/ref_python.py)."""
import math

import numpy as np
import pytest

from conftest import bits_equal_nan, kat, load_fixture
from oracle.pyoracle import Oracle
import ref_python


def _random_code(n, m, dv, seed):
    """Random column-regular H (rows ascending)."""
    rng = np.random.default_rng(seed)
    rows = [[] for _ in range(m)]
    for i in range(n):
        for j in rng.choice(m, size=dv, replace=False):
            rows[j].append(i)
    from qkd_ldpc_v_amd import HMatrix

    return HMatrix.from_check_nodes(n, [sorted(r) for r in rows])


def test_kat_johnson_ex25():
    K = kat()
    H = load_fixture("kat_n6_m4.dense")
    O = Oracle(H)
    llr, s = O.build_frame(np.array(K["alice"]), np.array(K["bob"]), K["qber"])
    p = O.params(K["algorithm"], K["max_iterations"], K["thr_enabled"], K["thr"])
    bits, it, ok, post = O.decode(p, llr, s)
    E = K["expected"]
    assert it == E["iterations"] and ok == E["syndromes_match"]
    assert bits.tolist() == E["bob_solution"] == K["alice"]
    assert bits_equal_nan(post, np.array(E["posterior_iteration_1"]))


def test_build_frame_matches_reference_llr():
    H = load_fixture("c1_n1024_m220.alist")
    O = Oracle(H)
    rng = np.random.default_rng(1)
    a = rng.integers(0, 2, H.n).astype(np.uint8)
    b = a.copy()
    b[:13] ^= 1
    q = 13 / H.n
    llr, s = O.build_frame(a, b, q)
    lp = math.log((1.0 - q) / q)
    assert np.array_equal(llr, np.where(b != 0, -lp, lp))
    assert np.array_equal(s, H.syndrome(a))


ALG_PARAMS = [(0, 0, 0), (1, 0, 0), (2, 0.75, 0), (3, 0.6, 0), (4, 0.8, 0.3), (5, 0.5, 1.1)]


@pytest.mark.parametrize("alg,prim,sec", ALG_PARAMS)
@pytest.mark.parametrize("thr_on", [True, False])
def test_oracle_equals_python_restatement(alg, prim, sec, thr_on):
    H = _random_code(48, 24, 3, seed=alg + 10 * thr_on)
    O = Oracle(H)
    cn, bn = H.check_nodes, H.bit_nodes
    rng = np.random.default_rng(100 + alg)
    for trial in range(4):
        a = rng.integers(0, 2, H.n).astype(np.uint8)
        b = a.copy()
        flips = rng.choice(H.n, size=3 + trial, replace=False)
        b[flips] ^= 1
        q = (3 + trial) / H.n
        llr, s = O.build_frame(a, b, q)
        p = O.params(alg, 12, thr_on, 7.5, prim, sec)
        bits, it, ok, post = O.decode(p, llr, s)
        rb, rit, rok, rpost = ref_python.decode(cn, bn, alg, llr.tolist(), s.tolist(), 12, thr_on, 7.5, prim, sec)
        assert (it, ok) == (rit, rok)
        assert bits.tolist() == rb
        assert bits_equal_nan(post, np.array(rpost))


def test_oracle_reproduces_unsorted_slot_pairing():
    """With unsorted bit_nodes lists the reference pairs check->bit slots by
    occurrence order (src/qkd_ldpc_algorithm.cpp:67-69,116-118); the oracle keeps
    that pairing, so results differ from the sorted matrix."""
    from qkd_ldpc_v_amd import HMatrix

    H = _random_code(40, 20, 3, seed=7)
    rp, ri = H.col_ptr.copy(), H.row_idx.copy()
    for i in range(H.n):
        ri[rp[i]:rp[i + 1]] = ri[rp[i]:rp[i + 1]][::-1]
    Hu = HMatrix(H.n, H.m, H.row_ptr, H.col_idx, rp, ri)
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2, H.n).astype(np.uint8)
    b = a.copy()
    b[[1, 5, 9, 20]] ^= 1
    O, Ou = Oracle(H), Oracle(Hu)
    llr, s = O.build_frame(a, b, 4 / H.n)
    p = O.params(0, 6, True, 100.0)
    r1 = O.decode(p, llr, s)
    r2 = Ou.decode(p, llr, s)
    rb, rit, rok, rpost = ref_python.decode(Hu.check_nodes, Hu.bit_nodes, 0, llr.tolist(), s.tolist(), 6, True, 100.0)
    assert bits_equal_nan(r2[3], np.array(rpost)) and r2[1] == rit
    assert not bits_equal_nan(r1[3], r2[3])


def test_oracle_batch_threads_agree():
    H = load_fixture("c1_n1024_m220.alist")
    O = Oracle(H)
    from qkd_ldpc_v_amd import bsc_frames

    a, b, q = bsc_frames(H.n, 0.03, 12, seed=5)
    llr = np.stack([O.build_frame(a[f], b[f], q)[0] for f in range(12)])
    s = np.stack([O.syndrome(a[f]) for f in range(12)])
    p = O.params(0, 50, True, 100.0)
    b1, i1, k1, p1 = O.decode_batch(p, llr, s, threads=1, posterior=True)
    b4, i4, k4, p4 = O.decode_batch(p, llr, s, threads=4, posterior=True)
    assert np.array_equal(b1, b4) and np.array_equal(i1, i4) and np.array_equal(k1, k4)
    assert bits_equal_nan(p1, p4)
    for f in range(12):
        assert np.array_equal(O.decode(p, llr[f], s[f])[0], b1[f])
