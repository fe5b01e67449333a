"""qldpc_run_trials — the simulation loop's batch seam through the C ABI
(Graph.run_trials): run_trial for every seed of one combination
(src/simulation.cpp:540-576, the body of QKD_LDPC_batch_simulation's
pool.detach_loop, :721-746), generated, decoded and compared on device and
sharded over the graph's devices.  Every trial's {iterations_num,
syndromes_match, keys_match} must equal the CPU oracle's run_trial on the same
seed (seeds[t] + seed_add)."""
import gzip
import os

import numpy as np
import pytest

import qkd_ldpc_v_amd as Q
from conftest import load_fixture, matrix_path
from oracle import pyoracle as P
from test_dropin import oracle_trials


def _check(H, g, alg, prim, sec, qber, max_it, seeds, seed_add, plan=None, punct=None, short=None):
    out = g.run_trials(Q.Params(alg, max_it, True, 100.0, prim, sec), qber, seeds, seed_add=seed_add, plan=plan)
    sd = [(int(s) + seed_add) & 0xFFFFFFFFFFFFFFFF for s in seeds]
    want = oracle_trials(H, alg, prim, sec, qber, max_it, sd, punct, short)
    got = [(int(a), int(b), int(c)) for a, b, c in zip(out.iterations, out.synd_ok, out.keys_match)]
    assert got == want
    assert out.accurate_qber == int(H.n * qber) / H.n
    assert np.all(out.runtime_us > 0)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", ["4", "0"])
def test_run_trials_c1_three_shards(gpu_available, monkeypatch, chunk):
    """31 trials over 3 logical shards; chunks of 4 cycle both pipeline slots."""
    if chunk != "0":
        monkeypatch.setenv("QLDPC_DIAG", "1")
        monkeypatch.setenv("QLDPC_TRIAL_CHUNK", chunk)
    H = load_fixture("c1_n1024_m220.alist")
    g = Q.Graph(H, devices=[0, 0, 0])
    seeds = P.trial_seeds(9012025, 31)
    out = _check(H, g, Q.SPA, 0.0, 0.0, 0.03, 50, seeds, 3)
    # the runtime shares follow the decode spans: not one constant
    assert out.runtime_us.max() > out.runtime_us.min()


@pytest.mark.gpu
def test_run_trials_min_sum_c2(gpu_available):
    H = load_fixture("c2_n10240_m2201.alist")
    g = Q.Graph(H)
    _check(H, g, Q.OMSA, 0.77, 0.0, 0.02, 50, P.trial_seeds(1022025, 12), 0)


@pytest.mark.gpu
def test_run_trials_rate_adapt(gpu_available, monkeypatch):
    monkeypatch.setenv("QLDPC_DIAG", "1")
    monkeypatch.setenv("QLDPC_TRIAL_CHUNK", "5")
    H = load_fixture("c5_n10240_m2048.sp2")
    u = np.array(gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split(), np.int32)
    punct, short, _ = Q.adapt_code_rate(H.n, H.m, 0.0156, 0.06, 1.39, u, Q.xoshiro_state(5555))
    g = Q.Graph(H, devices=[0, 0])
    plan = g.rate_plan(punct, short)
    _check(H, g, Q.AOMSA, 0.7, 0.99, 0.0156, 50, P.trial_seeds(5555, 11), 2, plan, punct, short)


@pytest.mark.gpu
def test_run_trials_split_frames_c4(gpu_available):
    """n = 102400: split frames and the trial generator's global-scratch path."""
    H = load_fixture("c4s_n102400_m32001.alist")
    g = Q.Graph(H)
    _check(H, g, Q.SPA, 0.0, 0.0, 0.038, 50, P.trial_seeds(777, 3), 1)


@pytest.mark.gpu
def test_run_trials_errors(gpu_available):
    H = load_fixture("c1_n1024_m220.alist")
    g = Q.Graph(H)
    with pytest.raises(Q.QLDPCError, match="is too small for QBER"):
        g.run_trials(Q.Params(Q.SPA, 50), 0.0005, P.trial_seeds(1, 4))
    out = g.run_trials(Q.Params(Q.SPA, 50), 0.03, np.zeros(0, np.uint64))
    assert out.iterations.size == 0 and out.accurate_qber == int(H.n * 0.03) / H.n


@pytest.mark.gpu
def test_run_trials_pipelined_window_is_the_combinations_own(gpu_available):
    """run_trials_submit puts combination c + 1 on the device before c is
    collected.  Each trial's runtime share comes from its chunk's window, which
    starts after the other slot's chunk in flight has ended: c + 1's window
    must not contain c's decode, so both pipelined sums stay near
    the blocking run's, and the results equal the blocking run's."""
    H = load_fixture("c2_n10240_m2201.alist")
    g = Q.Graph(H)
    p = Q.Params(Q.SPA, 50, True, 100.0)
    seeds = P.trial_seeds(1022025, 2048)
    g.run_trials(p, 0.0215, seeds[:64])  # warm: workspaces, generator tables
    blk = g.run_trials(p, 0.0215, seeds)
    j1 = g.submit_trials(p, 0.0215, seeds)
    j2 = g.submit_trials(p, 0.0215, seeds, seed_add=1)
    o1, o2 = j1.wait(), j2.wait()
    for a, b in ((o1, blk),):
        assert np.array_equal(a.iterations, b.iterations) and np.array_equal(a.keys_match, b.keys_match)
    rb, r1, r2 = blk.runtime_us.sum(), o1.runtime_us.sum(), o2.runtime_us.sum()
    assert r1 < 1.3 * rb and r2 < 1.3 * rb, (rb, r1, r2)
    assert np.all(o2.runtime_us > 0)


@pytest.mark.gpu
def test_run_trials_pipelined_split_graphs(gpu_available):
    """Two split-frame graphs (C4 stand-in, 8-wave parts), two combinations
    each, all submitted before any is collected: the split decodes of one
    device are serialised, so no part group can wait on another launch's
    workgroups ('part group failed to meet'); every job equals
    its blocking run."""
    H = load_fixture("c4s_n102400_m32001.alist")
    ga, gb = Q.Graph(H), Q.Graph(H)
    assert ga.plan(0, Q.SPA)["variant"].startswith("v2_split")
    p = Q.Params(Q.SPA, 50, True, 100.0)
    seeds = P.trial_seeds(777, 24)
    want = ga.run_trials(p, 0.038, seeds)
    jobs = [(ga, ga.submit_trials(p, 0.038, seeds)), (gb, gb.submit_trials(p, 0.038, seeds)),
            (ga, ga.submit_trials(p, 0.038, seeds, seed_add=1)), (gb, gb.submit_trials(p, 0.038, seeds))]
    outs = [j.wait() for _, j in jobs]
    for k in (0, 1, 3):
        assert np.array_equal(outs[k].iterations, want.iterations)
        assert np.array_equal(outs[k].synd_ok, want.synd_ok) and np.array_equal(outs[k].keys_match, want.keys_match)
    assert outs[2].iterations.size == 24


@pytest.mark.gpu
def test_frame_builder_refuses_graph_beyond_its_lds(gpu_available):
    """The device frame builder keeps both keys in LDS as bit words (n <=
    655,360): one bit more is refused with a message, not a launch error."""
    H = Q.regular_code(655392, 109232, 3, 5)
    g = Q.Graph(H)
    with pytest.raises(Q.QLDPCError, match="frame builder keeps the frame's keys in LDS"):
        g.run_trials(Q.Params(Q.SPA, 2), 0.02, P.trial_seeds(1, 1))
    # the rate-adapted builder also holds the extended key: its limit is ~436k bits
    H = Q.regular_code(440064, 73344, 3, 5)
    g = Q.Graph(H)
    plan = g.rate_plan(np.arange(0, 64, 2, dtype=np.int32), np.arange(1, 33, 2, dtype=np.int32))
    with pytest.raises(Q.QLDPCError, match="frame builder keeps the frame's keys in LDS"):
        g.run_trials(Q.Params(Q.SPA, 2), 0.02, P.trial_seeds(1, 1), plan=plan)
    g.run_trials(Q.Params(Q.SPA, 1), 0.02, P.trial_seeds(1, 1))  # plain frames of that size still build
