"""Rate adaptation: adapt_code_rate on the host and
QKD_LDPC_RATE_ADAPT's trials + extended frames + decode on device.

The (QBER, delta, f_EC) points are configs/ADAPTIVE T.json's maps for the
R=0.8 format-3 matrix with its .untp list (code-rate bucket 0.805); the
generator state chains from SIMULATION_SEED through the points like the
reference's setup loop (src/simulation.cpp:394-455)."""
import gzip
import math

import numpy as np
import pytest

import qkd_ldpc_v_amd as Q
from conftest import bits_equal_nan, load_fixture, matrix_path
from oracle import pyoracle as P
from oracle.pyoracle import Oracle

POINTS = [  # (QBER, delta, efficiency), code_rate 0.805 maps of configs/ADAPTIVE T.json
    (0.0076, 0.1, 1.85), (0.0116, 0.09, 1.5), (0.0156, 0.06, 1.39), (0.0196, 0.03, 1.28),
    (0.0236, 0.01, 1.21), (0.0276, 0.11, 1.2), (0.0316, 0.22, 1.22),
]
SEED = 21042025


def untp():
    return np.array(gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split(), np.int32)


@pytest.mark.parametrize("untainted", [True, False])
def test_adapt_code_rate_matches_oracle(untainted):
    H = load_fixture("c5_n10240_m2048.sp2")
    u = untp() if untainted else None
    st_p = Q.xoshiro_state(SEED)
    st_o = st_p.copy()
    got = 0
    for q, d, e in POINTS:
        pp, sp, rate = Q.adapt_code_rate(H.n, H.m, q, d, e, u, st_p)
        po, so = P.adapt_code_rate(H.n, H.m, q, d, e, u, st_o)
        assert np.array_equal(pp, po) and np.array_equal(sp, so) and np.array_equal(st_p, st_o)
        if pp.size:
            got += 1
            assert np.all(np.diff(pp) > 0) and np.all(np.diff(sp) > 0)
            assert not np.intersect1d(pp, sp).size
            assert rate == pytest.approx((H.n - H.m - sp.size) / (H.n - pp.size - sp.size))
            if untainted:
                assert np.array_equal(pp, np.sort(u[:pp.size]))
    assert got >= 3


def test_out_of_range_combination_is_skipped():
    st = Q.xoshiro_state(1)
    before = st.copy()
    p, s, r = Q.adapt_code_rate(10240, 2048, 0.11, 0.01, 1.0, None, st)  # R beyond the achievable range
    assert p.size == 0 and s.size == 0 and np.array_equal(st, before)


@pytest.mark.gpu
@pytest.mark.parametrize("alg,prim,sec", [(Q.AOMSA, 0.7, 0.99), (Q.ANMSA, 0.8, 0.35), (Q.SPA, 0.0, 0.0)])
def test_rate_adapted_pipeline_bitexact(gpu_available, alg, prim, sec):
    import torch

    H = load_fixture("c5_n10240_m2048.sp2")
    g = Q.Graph(H)
    st = Q.xoshiro_state(SEED)
    O = Oracle(H)
    batch = 16
    seeds = Q.trial_seeds(SEED, batch)
    dev = torch.device("cuda:0")
    for q, d, e in POINTS[1:4]:
        pp, sp, _ = Q.adapt_code_rate(H.n, H.m, q, d, e, untp(), st)
        plan = g.rate_plan(pp, sp)
        ds = torch.from_numpy(seeds.view(np.int64)).to(dev)
        ta = torch.empty((batch, H.n), dtype=torch.uint8, device=dev)
        tb = torch.empty_like(ta)
        pa = torch.empty((batch, max(1, pp.size)), dtype=torch.uint8, device=dev)
        pb = torch.empty_like(pa)
        qa = Q.trials_rate_adapt_device(H.n, q, ds, pp.size, ta, tb, pa, pb)
        lp = torch.full((batch,), Q.log_p(qa), dtype=torch.float64, device=dev)
        ax = torch.empty_like(ta)
        llr = torch.empty((batch, H.n), dtype=torch.float64, device=dev)
        syn = torch.empty((batch, H.m), dtype=torch.uint8, device=dev)
        bits = torch.empty_like(ta)
        it = torch.empty(batch, dtype=torch.int32, device=dev)
        ok = torch.empty(batch, dtype=torch.uint8, device=dev)
        km = torch.empty(batch, dtype=torch.uint8, device=dev)
        par = Q.Params(alg, 50, True, 100.0, prim, sec)
        g.qkd_ldpc_rate_adapt_device(plan, par, ta, tb, pa, pb, lp, ax, llr, syn, bits, it, ok, km)
        torch.cuda.synchronize()
        oa, ol = zip(*[P.trial_rate_adapt(H.n, q, int(sd), pp, sp)[:2] for sd in seeds])
        oa, ol = np.stack(oa), np.stack(ol)
        assert np.array_equal(ax.cpu().numpy(), oa)
        assert bits_equal_nan(llr.cpu().numpy(), ol)
        osyn = H.syndrome(oa)
        assert np.array_equal(syn.cpu().numpy(), osyn)
        ob, oi, ook, _ = O.decode_batch(O.params(alg, 50, True, 100.0, prim, sec), ol, osyn, threads=8)
        assert np.array_equal(bits.cpu().numpy(), ob)
        assert np.array_equal(it.cpu().numpy().astype(np.uint32), oi)
        assert np.array_equal(ok.cpu().numpy(), ook)
        assert np.array_equal(km.cpu().numpy(), (ob == oa).all(axis=1).astype(np.uint8))


# The other two code rates of the sweep (configs/ADAPTIVE T.json maps for the
# 0.655 and 0.505 buckets; AOMSA beta / sigma of those buckets)
OTHER_RATES = [
    ("c5b_n10240_m3584", 0.74, 0.94, [(0.0408, 0.1, 1.2), (0.0528, 0.01, 1.16), (0.0688, 0.23, 1.19)]),
    ("c5c_n10240_m5120", 0.72, 0.85, [(0.0774, 0.09, 1.17), (0.0894, 0.01, 1.14), (0.1094, 0.13, 1.15)]),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,beta,sigma,points", OTHER_RATES)
def test_rate_adapted_other_code_rates(gpu_available, name, beta, sigma, points):
    """R=0.65 and R=0.5 format-3 matrices: rate-adapted AOMSA frames built on
    device and decoded, bit-exact against the oracle (posteriors included)."""
    import torch

    H = load_fixture(name + ".sp2")
    u = np.array(gzip.open(matrix_path(name + ".untp")).read().split(), np.int32)
    g = Q.Graph(H)
    O = Oracle(H)
    st = Q.xoshiro_state(5555)
    batch = 12
    seeds = Q.trial_seeds(5555, batch)
    dev = torch.device("cuda:0")
    done = 0
    for q, d, e in points:
        pp, sp, _ = Q.adapt_code_rate(H.n, H.m, q, d, e, u, st)
        if pp.size + sp.size == 0:
            continue
        done += 1
        plan = g.rate_plan(pp, sp)
        ds = torch.from_numpy(seeds.view(np.int64)).to(dev)
        ta = torch.empty((batch, H.n), dtype=torch.uint8, device=dev)
        tb = torch.empty_like(ta)
        pa = torch.empty((batch, max(1, pp.size)), dtype=torch.uint8, device=dev)
        pb = torch.empty_like(pa)
        qa = Q.trials_rate_adapt_device(H.n, q, ds, pp.size, ta, tb, pa, pb)
        lp = torch.full((batch,), Q.log_p(qa), dtype=torch.float64, device=dev)
        ax = torch.empty_like(ta)
        llr = torch.empty((batch, H.n), dtype=torch.float64, device=dev)
        syn = torch.empty((batch, H.m), dtype=torch.uint8, device=dev)
        bits = torch.empty_like(ta)
        it = torch.empty(batch, dtype=torch.int32, device=dev)
        ok = torch.empty(batch, dtype=torch.uint8, device=dev)
        km = torch.empty(batch, dtype=torch.uint8, device=dev)
        par = Q.Params(Q.AOMSA, 50, True, 100.0, beta, sigma)
        g.qkd_ldpc_rate_adapt_device(plan, par, ta, tb, pa, pb, lp, ax, llr, syn, bits, it, ok, km)
        torch.cuda.synchronize()
        oa, ol = zip(*[P.trial_rate_adapt(H.n, q, int(sd), pp, sp)[:2] for sd in seeds])
        oa, ol = np.stack(oa), np.stack(ol)
        assert np.array_equal(ax.cpu().numpy(), oa)
        osyn = H.syndrome(oa)
        assert np.array_equal(syn.cpu().numpy(), osyn)
        ob, oi, ook, op = O.decode_batch(O.params(Q.AOMSA, 50, True, 100.0, beta, sigma), ol, osyn, threads=8,
                                         posterior=True)
        assert np.array_equal(bits.cpu().numpy(), ob)
        assert np.array_equal(it.cpu().numpy().astype(np.uint32), oi)
        assert np.array_equal(ok.cpu().numpy(), ook)
        out = g.decode(par, llr.cpu().numpy(), osyn, posterior=True)
        assert bits_equal_nan(out.posterior, op)
    assert done >= 2


@pytest.mark.gpu
def test_rate_adapted_pipeline_large_frames(gpu_available):
    """n = 102,400 (the C4 stand-in): the rate-adapted frame builder runs with
    1024 threads per frame there (decoder.hpp aux_frame_threads) — extended
    key, LLRs (1e-4 / DBL_MAX included) and Alice syndrome vs the oracle, then
    a short SPA decode of the built frames through the split kernel."""
    import torch

    H = load_fixture("c4s_n102400_m32001.alist")
    g = Q.Graph(H)
    rng = np.random.default_rng(4)
    pick = rng.choice(H.n, size=300, replace=False)
    pp, sp = np.sort(pick[:200]).astype(np.int32), np.sort(pick[200:]).astype(np.int32)
    plan = g.rate_plan(pp, sp)
    batch, q = 3, 0.03
    seeds = Q.trial_seeds(99, batch)
    dev = torch.device("cuda:0")
    ds = torch.from_numpy(seeds.view(np.int64)).to(dev)
    ta = torch.empty((batch, H.n), dtype=torch.uint8, device=dev)
    tb = torch.empty_like(ta)
    pa = torch.empty((batch, pp.size), dtype=torch.uint8, device=dev)
    pb = torch.empty_like(pa)
    qa = Q.trials_rate_adapt_device(H.n, q, ds, pp.size, ta, tb, pa, pb)
    lp = torch.full((batch,), Q.log_p(qa), dtype=torch.float64, device=dev)
    ax = torch.empty_like(ta)
    llr = torch.empty((batch, H.n), dtype=torch.float64, device=dev)
    syn = torch.empty((batch, H.m), dtype=torch.uint8, device=dev)
    bits = torch.empty_like(ta)
    it = torch.empty(batch, dtype=torch.int32, device=dev)
    ok = torch.empty(batch, dtype=torch.uint8, device=dev)
    km = torch.empty(batch, dtype=torch.uint8, device=dev)
    par = Q.Params(Q.SPA, 6, True, 100.0)
    g.qkd_ldpc_rate_adapt_device(plan, par, ta, tb, pa, pb, lp, ax, llr, syn, bits, it, ok, km)
    torch.cuda.synchronize()
    oa, ol = zip(*[P.trial_rate_adapt(H.n, q, int(sd), pp, sp)[:2] for sd in seeds])
    oa, ol = np.stack(oa), np.stack(ol)
    assert np.array_equal(ax.cpu().numpy(), oa)
    assert bits_equal_nan(llr.cpu().numpy(), ol)
    osyn = H.syndrome(oa)
    assert np.array_equal(syn.cpu().numpy(), osyn)
    O = Oracle(H)
    ob, oi, ook, _ = O.decode_batch(O.params(Q.SPA, 6, True, 100.0), ol, osyn, threads=8)
    assert np.array_equal(bits.cpu().numpy(), ob)
    assert np.array_equal(it.cpu().numpy().astype(np.uint32), oi) and np.array_equal(ok.cpu().numpy(), ook)
    assert np.array_equal(km.cpu().numpy(), (ob == oa).all(axis=1).astype(np.uint8))
