"""Unsorted adjacency: the reference's occurrence pairing on the GPU path.

With check_nodes rows out of ascending order, or bit_nodes lists that are not
the ascending transpose, the reference pairs a check's k-th input with the
k-th time its VN loop visits that check (bit_pos_idx,
src/qkd_ldpc_algorithm.cpp:116-118) and a bit's k-th message with the k-th
check that reached it (check_pos_idx, :67-69), so an edge's b2c is total -
c2b of another edge.  The oracle reproduces that pairing (checked against the
independent restatement in tests/ref_python.py by tests/test_oracle.py); the
GPU path plans the v1 global-slot kernel with a pairing pass for such graphs.
No matrix the reference ships is unsorted: these graphs are permuted copies.
"""
import ctypes

import numpy as np
import pytest

import qkd_ldpc_v_amd as Q
from conftest import bits_equal_nan, load_fixture
from oracle.pyoracle import Oracle
from qkd_ldpc_v_amd import HMatrix
from qkd_ldpc_v_amd._lib import lib, ptr

ALGS = [(Q.SPA, 0.0, 0.0), (Q.SPA_LIN, 0.0, 0.0), (Q.NMSA, 0.78, 0.0), (Q.OMSA, 0.77, 0.0),
        (Q.ANMSA, 0.8, 0.35), (Q.AOMSA, 0.55, 1.2)]


def permuted(H, seed, rows=True, cols=True):
    """H with every check_nodes row and / or bit_nodes list in a random order."""
    rng = np.random.default_rng(seed)
    ci, ri = H.col_idx.copy(), H.row_idx.copy()
    if rows:
        for j in range(H.m):
            a, b = H.row_ptr[j], H.row_ptr[j + 1]
            ci[a:b] = rng.permutation(ci[a:b])
    if cols:
        for i in range(H.n):
            a, b = H.col_ptr[i], H.col_ptr[i + 1]
            ri[a:b] = rng.permutation(ri[a:b])
    return HMatrix(H.n, H.m, H.row_ptr.copy(), ci.astype(np.int32), H.col_ptr.copy(), ri.astype(np.int32))


def host_plan(H, alg=0):
    """Plan of a host-only graph built from check_nodes alone (bit_nodes = their
    ascending transpose) through the C ABI."""
    g = ctypes.c_void_p()
    rc = lib().qldpc_graph_create_host(H.n, H.m, ptr(H.row_ptr), ptr(H.col_idx), ctypes.byref(g))
    if rc != 0:
        return rc, None
    lanes, epl, lds = (ctypes.c_int32() for _ in range(3))
    var = ctypes.c_char_p()
    rc = lib().qldpc_graph_plan(g, 0, alg, ctypes.byref(lanes), ctypes.byref(epl), None, ctypes.byref(lds),
                                ctypes.byref(var))
    lib().qldpc_graph_destroy(g)
    return rc, (var.value.decode() if rc == 0 else None)


def test_unsorted_rows_plan_the_pairing_kernel():
    H = load_fixture("c1_n1024_m220.alist")
    assert host_plan(H)[1] == "v2"
    rc, var = host_plan(permuted(H, 1, rows=True, cols=False))
    assert rc == 0 and var in ("glb_lds", "glb_glb"), var


def test_duplicate_bit_in_a_check_is_refused():
    H = HMatrix.from_check_nodes(4, [[0, 1, 2], [1, 2, 3]])
    bad = HMatrix(H.n, H.m, H.row_ptr, np.array([0, 1, 1, 1, 2, 3], np.int32), H.col_ptr, H.row_idx)
    assert host_plan(bad)[0] != 0


def test_check_nodes_only_entries_refuse_unsorted_lists():
    """The host-only planner takes check_nodes only; Graph(H, devices=...)
    passes bit_nodes too (qldpc_graph_create_checked_on) — see the GPU test."""
    H = load_fixture("c1_n1024_m220.alist")
    Hu = permuted(H, 2, rows=False, cols=True)
    with pytest.raises(ValueError):
        Q.Graph(Hu, host_only=True)


@pytest.mark.gpu
def test_device_list_graph_keeps_occurrence_pairing(gpu_available):
    """Graph(H, devices=[0, 0]) on unsorted bit_nodes: two logical shards, each
    decoding with the reference's occurrence pairing, bit-exact vs the oracle."""
    H = load_fixture("c1_n1024_m220.alist")
    Hu = permuted(H, 2, rows=False, cols=True)
    a, b, q = Q.bsc_frames(Hu.n, 0.03, 9, seed=77)
    lp = Q.log_p(q)
    llr = np.where(b != 0, -lp, lp).astype(np.float64)
    synd = Hu.syndrome(a)
    g = Q.Graph(Hu, devices=[0, 0])
    assert g.info()["devices"] == 2
    p = Q.Params(Q.SPA, 50, True, 100.0)
    out = g.decode(p, llr, synd, posterior=True)
    O = Oracle(Hu)
    ob, oi, ok, op = O.decode_batch(O.params(Q.SPA, 50, True, 100.0), llr, synd, threads=8, posterior=True)
    assert np.array_equal(out.bits, ob) and np.array_equal(out.iterations, oi) and np.array_equal(out.synd_ok, ok)
    assert bits_equal_nan(out.posterior, op)


def _parity(H, alg, prim, sec, batch, qber, max_it, seed):
    a, b, q = Q.bsc_frames(H.n, qber, batch, seed=seed)
    lp = Q.log_p(q)
    llr = np.where(b != 0, -lp, lp).astype(np.float64)
    synd = H.syndrome(a)
    g = Q.Graph(H)
    plan = g.plan(0, alg)
    out = g.decode(Q.Params(alg, max_it, True, 100.0, prim, sec), llr, synd, posterior=True)
    O = Oracle(H)
    ob, oi, ok, op = O.decode_batch(O.params(alg, max_it, True, 100.0, prim, sec), llr, synd, threads=8,
                                    posterior=True)
    for f in range(batch):
        assert np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f], f
        assert bits_equal_nan(out.posterior[f], op[f]), f
    return plan, out


@pytest.mark.gpu
@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_unsorted_c1_matches_oracle(gpu_available, alg, prim, sec):
    H = load_fixture("c1_n1024_m220.alist")
    Hu = permuted(H, 10 + alg)
    plan, out = _parity(Hu, alg, prim, sec, batch=24, qber=0.02, max_it=12, seed=alg)
    assert plan["variant"] in ("glb_lds", "glb_glb"), plan
    # the pairing changes the decode: the sorted graph gives other posteriors
    Hs = load_fixture("c1_n1024_m220.alist")
    a, b, q = Q.bsc_frames(H.n, 0.02, 24, seed=alg)
    lp = Q.log_p(q)
    llr = np.where(b != 0, -lp, lp).astype(np.float64)
    ref = Q.Graph(Hs).decode(Q.Params(alg, 12, True, 100.0, prim, sec), llr, Hs.syndrome(a), posterior=True)
    assert not all(bits_equal_nan(ref.posterior[f], out.posterior[f]) for f in range(24))


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols", [(True, False), (False, True)])
def test_unsorted_one_side_matches_oracle(gpu_available, rows, cols):
    H = load_fixture("c1_n1024_m220.alist")
    _parity(permuted(H, 7, rows=rows, cols=cols), Q.SPA, 0.0, 0.0, batch=16, qber=0.015, max_it=50, seed=3)


@pytest.mark.gpu
def test_unsorted_c2_spa_full_decode(gpu_available):
    H = load_fixture("c2_n10240_m2201.alist")
    _parity(permuted(H, 21), Q.SPA, 0.0, 0.0, batch=8, qber=0.0215, max_it=50, seed=5)
