"""GPU parity: the HIP decoder (through the C ABI) against the CPU oracle and the
reference's golden KAT.  Bar: bit-exact hard bits, iteration counts,
syndromes_match AND posterior LLRs (the SPA math is glibc-exact on device).
Runs on the MI355X box: `pytest -m gpu`."""
import math
import sys

import numpy as np
import pytest

from conftest import bits_equal_nan, kat, load_fixture, matrix_path
from oracle.pyoracle import Oracle
import qkd_ldpc_v_amd as Q

pytestmark = pytest.mark.gpu

DBL_MAX = sys.float_info.max
ALGS = [  # (alg, primary, secondary) — NOPT_R=0,82 / config-map style factors
    (Q.SPA, 0.0, 0.0), (Q.SPA_LIN, 0.0, 0.0), (Q.NMSA, 0.78, 0.0), (Q.OMSA, 0.77, 0.0),
    (Q.ANMSA, 0.8, 0.35), (Q.AOMSA, 0.55, 1.2),
]
_graphs = {}


def graph(name, variant="auto"):
    """Device graph of a fixture; variant "v1" forces the first-generation
    planner (QLDPC_VARIANT is read when the graph is created, under the
    diagnostic switch QLDPC_DIAG=1)."""
    import os

    key = (name, variant)
    if key not in _graphs:
        old = {k: os.environ.pop(k, None) for k in ("QLDPC_VARIANT", "QLDPC_DIAG")}
        if variant != "auto":
            os.environ.update(QLDPC_DIAG="1", QLDPC_VARIANT=variant)
        try:
            _graphs[key] = Q.Graph(load_fixture(name))
        finally:
            for k, v in old.items():
                os.environ.pop(k, None)
                if v is not None:
                    os.environ[k] = v
    return _graphs[key]


def frames(H, qber, batch, seed):
    a, b, q = Q.bsc_frames(H.n, qber, batch, seed=seed)
    lp = Q.log_p(q)
    llr = np.where(b != 0, -lp, lp).astype(np.float64)
    return a, b, llr, H.syndrome(a)


def assert_parity(name, alg, prim, sec, qber, batch, max_it=50, thr_on=True, thr=100.0, seed=0, threads=16,
                  llr=None, synd=None, variant="auto"):
    H = load_fixture(name)
    if llr is None:
        _, _, llr, synd = frames(H, qber, batch, seed)
    g = graph(name, variant)
    out = g.decode(Q.Params(alg, max_it, thr_on, thr, prim, sec), llr, synd, posterior=True)
    O = Oracle(H)
    ob, oi, ok, op = O.decode_batch(O.params(alg, max_it, thr_on, thr, prim, sec), llr, synd, threads=threads,
                                    posterior=True)
    bad = [f for f in range(llr.shape[0])
           if not (np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f]
                   and bits_equal_nan(out.posterior[f], op[f]))]
    assert not bad, (f"{name} alg={alg}: {len(bad)}/{llr.shape[0]} frames differ; first {bad[0]}: "
                     f"gpu it={out.iterations[bad[0]]} ok={out.synd_ok[bad[0]]} / oracle it={oi[bad[0]]} "
                     f"ok={ok[bad[0]]}; bit diffs={int((out.bits[bad[0]] != ob[bad[0]]).sum())}")
    return out, oi


def test_device_exact_math_bitwise(gpu_available):
    import torch

    rng = np.random.default_rng(11)
    xs = np.concatenate([
        (rng.random(200000) * 2 - 1) * 60.0,
        (rng.random(200000) * 2 - 1) * 2.0,
        1.0 - np.ldexp(rng.random(100000), -rng.integers(0, 60, 100000)),
        -(1.0 - np.ldexp(rng.random(100000), -rng.integers(0, 60, 100000))),
        rng.integers(0, 2**63, 200000, dtype=np.int64).view(np.float64),
        np.array([0.0, -0.0, 1.0, -1.0, 22.0, -22.0, np.inf, -np.inf, np.nan, DBL_MAX, 5e-324]),
    ])
    refs = {0: math.tanh, 2: math.expm1}
    d_in = torch.from_numpy(xs).cuda()
    d_out = torch.empty_like(d_in)
    for fn, name in ((0, "tanh"), (1, "atanh"), (2, "expm1"), (3, "log1p"), (6, "tanh_dec"), (7, "atanh_dec"),
                     (8, "tanh_half_clip_t"), (9, "atanh2_clip")):
        Q._lib.check(Q.lib().qldpc_selftest_math_device(fn, xs.size, d_in.data_ptr(), d_out.data_ptr(), None),
                     "selftest")
        torch.cuda.synchronize()
        got = d_out.cpu().numpy()
        f = {0: math.tanh, 1: math.atanh, 2: math.expm1, 3: math.log1p, 6: math.tanh, 7: math.atanh,
             8: lambda v: math.tanh(v / 2.),  # 8: the SPA scan's table form of tanh(b2c / 2.)
             9: lambda v: v if v != v else max(-100.0, min(100.0, 2. * math.atanh(v)))}[fn]  # 9: clipped 2 atanh

        def ref(x):
            try:
                return f(x)
            except (ValueError, OverflowError):
                if fn in (1, 7):
                    return math.copysign(math.inf, x) if abs(x) == 1 else math.nan
                if fn == 9:
                    return math.copysign(100.0, x) if abs(x) == 1 else math.nan
                if fn == 3:
                    return -math.inf if x == -1 else math.nan
                return math.inf
        want = np.array([ref(float(x)) for x in xs])
        assert bits_equal_nan(got, want), f"{name}: {int((~((got == want) | (np.isnan(got) & np.isnan(want)))).sum())} diffs"


def test_kat_johnson_on_gpu(gpu_available):
    K = kat()
    H = load_fixture("kat_n6_m4.dense")
    g = graph("kat_n6_m4.dense")
    lp = Q.log_p(K["qber"])
    llr = np.where(np.array(K["bob"]) != 0, -lp, lp)
    s = H.syndrome(np.array(K["alice"], np.uint8))
    out = g.decode(Q.Params(K["algorithm"], K["max_iterations"], K["thr_enabled"], K["thr"]), llr, s, posterior=True)
    E = K["expected"]
    assert int(out.iterations[0]) == E["iterations"] and bool(out.synd_ok[0]) == E["syndromes_match"]
    assert out.bits[0].tolist() == E["bob_solution"]
    assert bits_equal_nan(out.posterior[0], np.array(E["posterior_iteration_1"]))


def test_planner_picks_wave_aligned_kernel(gpu_available):
    for name in ("c1_n1024_m220.alist", "c2_n10240_m2201.alist", "c3_n10240_m1801.alist"):
        for alg, _, _ in ALGS:
            assert graph(name).plan(0, alg)["variant"] == "v2", name
        assert graph(name, "v1").plan(0, Q.SPA)["variant"] == "reg_lds", name


@pytest.mark.parametrize("variant", ["auto", "v1"])
@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c1_1k_all_algorithms(gpu_available, alg, prim, sec, variant):
    # QBER above the code's threshold region: a mix of converging and failing frames
    assert_parity("c1_n1024_m220.alist", alg, prim, sec, qber=0.03, batch=96, seed=alg, variant=variant)


@pytest.mark.parametrize("variant", ["auto", "v1"])
@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c2_10k_all_algorithms(gpu_available, alg, prim, sec, variant):
    assert_parity("c2_n10240_m2201.alist", alg, prim, sec, qber=0.026, batch=24, seed=10 + alg, variant=variant)


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c2_unpaletted_llrs(gpu_available, alg, prim, sec):
    """Frames with more than 4 distinct LLR values (soft channel inputs): the V2
    kernel gathers llr[] from HBM instead of the LDS palette."""
    H = load_fixture("c2_n10240_m2201.alist")
    a, b, llr, s = frames(H, 0.024, 16, 70 + alg)
    rng = np.random.default_rng(71 + alg)
    llr = llr * rng.uniform(0.6, 1.4, llr.shape)
    llr[::2, :5] = [1e-4, -1e-4, 0.0, -0.0, DBL_MAX]  # specials in half the frames
    assert_parity("c2_n10240_m2201.alist", alg, prim, sec, qber=0, batch=16, llr=llr, synd=s)


@pytest.mark.parametrize("name,batch", [("c1_n1024_m220.alist", 24), ("c2_n10240_m2201.alist", 8),
                                        ("c4s_n102400_m32001.alist", 4)])
def test_spa_iteration0_uniform_llr_table(gpu_available, name, batch):
    """SPA iteration 0 on +-L frames takes per-frame tables (t0, A[d]) instead
    of per-edge tanh/atanh: both ends of its L range, L past the tanh
    saturation (t0 = 1, messages = +-thr), threshold off, iteration caps 1-3
    and an all-positive frame (one-entry palette).  Outside the range (and
    with a third LLR value) the general pass runs; results must agree."""
    H = load_fixture(name)
    a, b, _, s = frames(H, 0.03, batch, 90)
    sign = np.where(b != 0, -1.0, 1.0)
    sign[0] = 1.0  # no channel errors in frame 0
    for L in (2.0**-20, 2.0**-21, 0.37, 3.5, 43.99, 44.0, 60.0, 2.0**10, 2.0**10 * 1.5):
        for max_it, thr_on in ((1, True), (2, True), (3, False), (12, True)):
            assert_parity(name, Q.SPA, 0, 0, qber=0, batch=batch, max_it=max_it, thr_on=thr_on,
                          llr=sign * L, synd=s)
    llr = sign * 2.5
    llr[1, 7] = 1e-4  # a third value: general iteration 0 for that frame only
    assert_parity(name, Q.SPA, 0, 0, qber=0, batch=batch, max_it=8, llr=llr, synd=s)


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c2_rate_adapted_palette(gpu_available, alg, prim, sec):
    """Punctured (1e-4) and shortened (DBL_MAX) positions on the V2 kernel: four
    distinct LLRs per frame, i.e. a full palette."""
    H = load_fixture("c2_n10240_m2201.alist")
    rng = np.random.default_rng(80 + alg)
    a, b, llr, s = frames(H, 0.02, 12, 81 + alg)
    pos = rng.permutation(H.n)
    punct, short = pos[:300], pos[300:500]
    a[:, short] = 0
    b[:, short] = 0
    s = H.syndrome(a)
    lp = Q.log_p(0.02)
    llr = np.where(b != 0, -lp, lp)
    llr[:, punct] = 1e-4
    llr[:, short] = DBL_MAX
    for thr_on in (True, False):
        assert_parity("c2_n10240_m2201.alist", alg, prim, sec, qber=0, batch=12, thr_on=thr_on, llr=llr, synd=s)


def test_c2_spa_headline_config(gpu_available):
    out, oi = assert_parity("c2_n10240_m2201.alist", Q.SPA, 0, 0, qber=0.0215, batch=48, seed=1022025)
    assert out.synd_ok.mean() > 0.9  # the config's operating point decodes


@pytest.mark.parametrize("alg,prim,sec", [(Q.OMSA, 0.77, 0.0), (Q.NMSA, 0.78, 0.0)])
def test_c3_10k(gpu_available, alg, prim, sec):
    assert_parity("c3_n10240_m1801.alist", alg, prim, sec, qber=0.015, batch=32, seed=10022025)


@pytest.mark.parametrize("vng", ["1", "0"])
@pytest.mark.parametrize("alg,prim,sec", ALGS[2:])
def test_minsum_bit_gather_and_vn_phases(gpu_available, alg, prim, sec, vng, monkeypatch):
    """Min-sum family on dv <= 4 codes: the bit gather (default, messages
    rebuilt per bit from row aggregates) and the VN-phase path (QLDPC_VNG=0,
    read per launch) both bit-exact, incl. iteration caps and threshold off."""
    monkeypatch.setenv("QLDPC_DIAG", "1")
    monkeypatch.setenv("QLDPC_VNG", vng)
    assert_parity("c3_n10240_m1801.alist", alg, prim, sec, qber=0.02, batch=24, seed=77)
    assert_parity("c2_n10240_m2201.alist", alg, prim, sec, qber=0.03, batch=16, seed=78, max_it=3)
    assert_parity("c1_n1024_m220.alist", alg, prim, sec, qber=0.04, batch=32, seed=79, thr_on=False)
    # irregular (dv 2..26) hybrid shape: padded per-bit edge chunks, bits in degree order
    assert_parity("c5_n10240_m2048.sp2", alg, prim, sec, qber=0.03, batch=12, seed=80)
    assert_parity("c5_n10240_m2048.sp2", alg, prim, sec, qber=0.05, batch=8, seed=81, max_it=2)
    H = load_fixture("c5_n10240_m2048.sp2")  # rate-adapted style frame: full palette, DBL_MAX, 1e-4
    rng = np.random.default_rng(82)
    a, b, llr, s = frames(H, 0.02, 8, 83)
    pos = rng.permutation(H.n)
    a[:, pos[300:420]] = 0
    b[:, pos[300:420]] = 0
    s = H.syndrome(a)
    lp = Q.log_p(0.02)
    llr = np.where(b != 0, -lp, lp)
    llr[:, pos[:300]] = 1e-4
    llr[:, pos[300:420]] = DBL_MAX
    assert_parity("c5_n10240_m2048.sp2", alg, prim, sec, qber=0, batch=8, llr=llr, synd=s)


def _irregular_dv4_code(n=4096, m=900, seed=5):
    """Random code whose bits have degree 0..4 (isolated bits included) and
    rows of degree 12..20: the dv <= 4 bit gather with missing terms."""
    rng = np.random.default_rng(seed)
    rows = [set() for _ in range(m)]
    for b in range(n):
        d = int(rng.choice([0, 1, 2, 3, 4], p=[0.02, 0.08, 0.3, 0.3, 0.3]))
        for r in rng.choice(m, size=d, replace=False):
            rows[int(r)].add(b)
    for r in range(m):  # every row at least 2 edges (a 1-edge row keeps min2 = DBL_MAX)
        while len(rows[r]) < 2:
            rows[r].add(int(rng.integers(n)))
    return Q.HMatrix.from_check_nodes(n, [sorted(r) for r in rows])


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_bit_gather_irregular_low_degree(gpu_available, alg, prim, sec):
    H = _irregular_dv4_code()
    g = Q.Graph(H)
    O = Oracle(H)
    for qber, max_it, thr_on, seed in ((0.03, 50, True, 1), (0.06, 4, True, 2), (0.03, 50, False, 3)):
        _, _, llr, synd = frames(H, qber, 16, seed)
        out = g.decode(Q.Params(alg, max_it, thr_on, 100.0, prim, sec), llr, synd, posterior=True)
        ob, oi, ok, op = O.decode_batch(O.params(alg, max_it, thr_on, 100.0, prim, sec), llr, synd, threads=16,
                                        posterior=True)
        for f in range(llr.shape[0]):
            assert np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f]
            assert bits_equal_nan(out.posterior[f], op[f])
    # (the plan shape is asserted after the bits, so a changed plan never skips them)
    assert g.plan(0, alg)["variant"] == "v2", g.plan(0, alg)


@pytest.mark.parametrize("alg,prim,sec", ALGS)
@pytest.mark.parametrize("name,qber", [("c5b_n10240_m3584.sp2", 0.045), ("c5c_n10240_m5120.sp2", 0.085)])
def test_c5_other_code_rates_all_algorithms(gpu_available, name, qber, alg, prim, sec):
    """R=0.65 (m=3584) and R=0.5 (m=5120, a bit of degree 66) format-3 codes on
    the hybrid shape; R=0.5's min-sum row aggregates live in global scratch."""
    assert_parity(name, alg, prim, sec, qber=qber, batch=8, seed=60 + alg)
    assert_parity(name, alg, prim, sec, qber=qber, batch=4, seed=70 + alg, max_it=2, thr_on=False)
    plan = graph(name).plan(0, alg)
    assert plan["variant"] == "v2_hybrid"
    if name.startswith("c5b") and alg >= 2:
        # R=0.65: the 16-byte row aggregates (56 KiB) stay in LDS beside the totals
        assert plan["lds_bytes"] > 130 * 1024, plan


M2K = [("m2k_n10240_m1024.sp2", 0.006), ("m2k_n10240_m1536.sp2", 0.012), ("m2k_n10240_m2560.sp2", 0.028),
       ("m2k_n10240_m3072.sp2", 0.036), ("m2k_n10240_m4096.sp2", 0.055), ("m2k_n10240_m4608.sp2", 0.065)]


@pytest.mark.parametrize("alg,prim,sec", ALGS)
@pytest.mark.parametrize("name,qber", M2K)
def test_format3_codes_all_rates_all_algorithms(gpu_available, name, qber, alg, prim, sec):
    """The other irregular format-3 codes the reference ships with untainted
    lists (sparse_matrices/matrices_2_10k_all, R = 0.9 .. 0.55), whatever
    shape the planner gives them."""
    assert_parity(name, alg, prim, sec, qber=qber, batch=8, seed=80 + alg)


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c5_irregular_hybrid_variant(gpu_available, alg, prim, sec):
    assert_parity("c5_n10240_m2048.sp2", alg, prim, sec, qber=0.025, batch=12, seed=50 + alg)
    assert graph("c5_n10240_m2048.sp2").plan(0, alg)["variant"] == "v2_hybrid"


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c5_irregular_v1_global_message_variant(gpu_available, alg, prim, sec):
    assert_parity("c5_n10240_m2048.sp2", alg, prim, sec, qber=0.025, batch=6, seed=60 + alg, variant="v1")
    assert graph("c5_n10240_m2048.sp2", "v1").plan(0, alg)["variant"] == "glb_lds"


@pytest.mark.parametrize("alg,prim,sec", [(Q.SPA, 0, 0), (Q.AOMSA, 0.55, 1.2)])
def test_c4_100k_all_global_variant(gpu_available, alg, prim, sec):
    assert_parity("c4s_n102400_m32001.alist", alg, prim, sec, qber=0.038, batch=3, max_it=6, seed=4, variant="v1")
    assert graph("c4s_n102400_m32001.alist", "v1").plan(0, alg)["variant"] == "glb_glb"


# n = 100k: a frame is split over several workgroups of one XCD (capi.hip plan_v2_split)
@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c4_100k_split_variant(gpu_available, alg, prim, sec):
    assert_parity("c4s_n102400_m32001.alist", alg, prim, sec, qber=0.038, batch=10, max_it=8, seed=40 + alg)
    assert graph("c4s_n102400_m32001.alist").plan(0, alg)["variant"] == "v2_split"


def test_c4_100k_split_full_decode(gpu_available):
    # 50 iterations: converging frames exit early, the rest run to the cap
    out, oi = assert_parity("c4s_n102400_m32001.alist", Q.SPA, 0, 0, qber=0.038, batch=6, max_it=50, seed=9)
    assert out.iterations.min() < 50


@pytest.mark.parametrize("max_it,qber", [(1, 0.038), (2, 0.038), (3, 0.038), (50, 1e-6), (50, 0.003)])
@pytest.mark.parametrize("alg,prim,sec", [(Q.SPA, 0, 0), (Q.OMSA, 0.77, 0.0), (Q.AOMSA, 0.55, 1.2)])
def test_c4_split_deferred_exit_edges(gpu_available, alg, prim, sec, max_it, qber):
    """Split frames test for the exit after the message pass (decoder_v2.hip
    QL_SPLIT_DEFER; the frame leaves before the gather with the totals of the
    scan that found it done).  Edges: iteration caps 1-3 (the last iteration
    a scan only), frames without errors (AOMSA exits in iteration 0, SPA /
    OMSA in iteration 1) and frames that converge in a few iterations —
    bits, iterations, syndromes_match and posteriors vs the oracle."""
    out, oi = assert_parity("c4s_n102400_m32001.alist", alg, prim, sec, qber=qber, batch=4, max_it=max_it,
                            seed=700 + max_it)
    if qber < 1e-5:
        assert out.synd_ok.all()


@pytest.mark.parametrize("wp", [0, 16])
@pytest.mark.parametrize("alg,prim,sec", [(Q.SPA, 0, 0), (Q.OMSA, 0.77, 0.0), (Q.AOMSA, 0.55, 1.2)])
def test_c4_generated_dv4_many_parts(gpu_available, monkeypatch, alg, prim, sec, wp):
    """the generated n=102400 dv=4 code (409,600
    edges).  The planner takes 16-wave parts, one per CU, with 12 scratch
    message slots per lane (8 parts, four frames per XCD; 21 8-wave parts and
    three frames without them).  wp = 16 forces the 16-wave family (the same
    plan here)."""
    H = Q.regular_code(102400, 22001, 4, 777)
    if wp:
        monkeypatch.setenv("QLDPC_DIAG", "1")
        monkeypatch.setenv("QLDPC_SPLIT_WP", str(wp))
    g = Q.Graph(H)
    monkeypatch.delenv("QLDPC_SPLIT_WP", raising=False)
    O = Oracle(H)
    _, _, llr, synd = frames(H, 0.022, 6, 4242)
    out = g.decode(Q.Params(alg, 50, True, 100.0, prim, sec), llr, synd, posterior=True)
    ob, oi, ok, op = O.decode_batch(O.params(alg, 50, True, 100.0, prim, sec), llr, synd, threads=16, posterior=True)
    for f in range(llr.shape[0]):
        assert np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f]
        assert bits_equal_nan(out.posterior[f], op[f])
    # the plan this test meant to cover (asserted after the bits: a changed plan never skips them;
    # the planner's shapes alone are CPU tests, tests/test_capi.py)
    plan = g.plan(0, alg)
    assert plan["variant"] == "v2_split" and plan["lanes"] == 8 * 1024, plan
    assert g.split_plan() == {"parts": 8, "part_lanes": 1024, "scratch_slots": 12}
    assert plan["workgroups"] == 256, plan  # one 16-wave part per CU


@pytest.mark.parametrize("alg,prim,sec", ALGS)
@pytest.mark.parametrize("name,wp,scratch,parts", [("c4s", "16", "1", 6), ("c4s", "8", "1", 12), ("c4g", "8", "0", 21),
                                                   ("c4g", "8", "1", 16)])
def test_c4_split_scratch_slots_forced(gpu_available, monkeypatch, alg, prim, sec, name, wp, scratch, parts):
    """Split families the planner does not pick by default (QLDPC_SPLIT_WP and
    QLDPC_SPLIT_SCRATCH, read when the graph is created; the defaults are the
    stand-in's 15 8-wave parts without scratch slots and C4 (ii)'s 8 16-wave
    parts with 12 per lane): the stand-in with scratch slots in 16- and
    8-wave parts, C4 (ii) in 8-wave parts without and with them — bits,
    iterations, syndromes_match and posteriors vs the oracle."""
    H = load_fixture("c4s_n102400_m32001.alist") if name == "c4s" else Q.regular_code(102400, 22001, 4, 777)
    monkeypatch.setenv("QLDPC_DIAG", "1")
    monkeypatch.setenv("QLDPC_SPLIT_WP", wp)
    monkeypatch.setenv("QLDPC_SPLIT_SCRATCH", scratch)
    g = Q.Graph(H)
    monkeypatch.delenv("QLDPC_SPLIT_SCRATCH")
    monkeypatch.delenv("QLDPC_SPLIT_WP")
    qber = 0.038 if name == "c4s" else 0.022
    _, _, llr, synd = frames(H, qber, 6, 300 + alg)
    out = g.decode(Q.Params(alg, 14, True, 100.0, prim, sec), llr, synd, posterior=True)
    O = Oracle(H)
    ob, oi, ok, op = O.decode_batch(O.params(alg, 14, True, 100.0, prim, sec), llr, synd, threads=16, posterior=True)
    for f in range(llr.shape[0]):
        assert np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f]
        assert bits_equal_nan(out.posterior[f], op[f])
    assert g.split_plan() == {"parts": parts, "part_lanes": 64 * int(wp), "scratch_slots": 12 if scratch == "1" else 0}


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_c4_100k_split_full_parts(gpu_available, monkeypatch, alg, prim, sec):
    """The C4 stand-in plans 8-wave parts without scratch slots, two per CU
    (decoder_v2.hip PL = 512: LDS message slots at a 512-lane stride, the
    graph's per-part arrays at the 1024-lane stride with waves 8..15 empty;
    test_c4_100k_split_variant).  QLDPC_SPLIT_WP=16 with QLDPC_SPLIT_SCRATCH=0
    (read when the graph is created) forces the fourth family, 16-wave parts
    without scratch slots, one per CU (8 parts) — bit-exact with the oracle,
    posteriors included."""
    H = load_fixture("c4s_n102400_m32001.alist")
    monkeypatch.setenv("QLDPC_DIAG", "1")
    monkeypatch.setenv("QLDPC_SPLIT_WP", "16")
    monkeypatch.setenv("QLDPC_SPLIT_SCRATCH", "0")
    g = Q.Graph(H)
    monkeypatch.delenv("QLDPC_SPLIT_WP")
    monkeypatch.delenv("QLDPC_SPLIT_SCRATCH")
    _, _, llr, synd = frames(H, 0.038, 8, 170 + alg)
    out = g.decode(Q.Params(alg, 12, True, 100.0, prim, sec), llr, synd, posterior=True)
    O = Oracle(H)
    ob, oi, ok, op = O.decode_batch(O.params(alg, 12, True, 100.0, prim, sec), llr, synd, threads=16, posterior=True)
    for f in range(llr.shape[0]):
        assert np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f]
        assert bits_equal_nan(out.posterior[f], op[f])
    plan = g.plan(0, alg)  # (after the bits; the default 15 x 8-wave plan is a CPU test)
    assert plan["lanes"] == 8 * 1024, plan
    assert plan["workgroups"] == 256, plan


@pytest.mark.parametrize("env", [{"QLDPC_SPLIT_X": "0"}, {"QLDPC_SPLIT_K": "10"}])
@pytest.mark.parametrize("alg,prim,sec", [(Q.SPA, 0, 0), (Q.OMSA, 0.77, 0.0)])
def test_c4_100k_split_other_layouts(gpu_available, monkeypatch, alg, prim, sec, env):
    """The split layouts other than the default (read when the graph is
    created): the term-major stage (QLDPC_SPLIT_X=0, the A/B arm of
    DecodeArgs::xoff) and K = 10 parts of 16 waves instead of the planner's 15
    of 8 — same
    bits, iterations and posteriors as the oracle and as the default graph."""
    H = load_fixture("c4s_n102400_m32001.alist")
    monkeypatch.setenv("QLDPC_DIAG", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g0 = Q.Graph(H)
    for k in env:
        monkeypatch.delenv(k)
    _, _, llr, synd = frames(H, 0.038, 6, 90 + alg)
    p = Q.Params(alg, 10, True, 100.0, prim, sec)
    out0 = g0.decode(p, llr, synd, posterior=True)
    out1 = graph("c4s_n102400_m32001.alist").decode(p, llr, synd, posterior=True)
    O = Oracle(H)
    ob, oi, ok, op = O.decode_batch(O.params(alg, 10, True, 100.0, prim, sec), llr, synd, threads=16, posterior=True)
    for out in (out0, out1):
        for f in range(llr.shape[0]):
            assert np.array_equal(out.bits[f], ob[f]) and out.iterations[f] == oi[f] and out.synd_ok[f] == ok[f]
            assert bits_equal_nan(out.posterior[f], op[f])
    assert g0.plan(0, alg)["lanes"] == (10 * 1024 if "QLDPC_SPLIT_K" in env else 15 * 512)


@pytest.mark.parametrize("batch", [1, 2])
def test_c4_100k_split_few_frames(gpu_available, batch):
    # fewer frames than XCDs: most part groups draw no frame and leave
    assert_parity("c4s_n102400_m32001.alist", Q.OMSA, 0.77, 0, qber=0.038, batch=batch, max_it=5, seed=70 + batch)


@pytest.mark.parametrize("max_it", [1, 2, 3])
@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_iteration_cap_edges(gpu_available, alg, prim, sec, max_it):
    assert_parity("c1_n1024_m220.alist", alg, prim, sec, qber=0.02, batch=32, max_it=max_it, seed=7)
    assert_parity("c2_n10240_m2201.alist", alg, prim, sec, qber=0.024, batch=8, max_it=max_it, seed=17)


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_threshold_disabled(gpu_available, alg, prim, sec):
    assert_parity("c1_n1024_m220.alist", alg, prim, sec, qber=0.035, batch=32, thr_on=False, seed=8)


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_rate_adapted_special_llrs(gpu_available, alg, prim, sec):
    """QKD_LDPC_RATE_ADAPT frames (src/qkd_ldpc_algorithm.cpp:1148-1174):
    punctured positions carry ALMOST_ZERO=1e-4, shortened positions DBL_MAX."""
    import gzip

    H = load_fixture("c5_n10240_m2048.sp2")
    untp = np.array(gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split(), np.int64)
    rng = np.random.default_rng(12)
    batch = 8
    punct = np.sort(untp[:400])
    rest = np.setdiff1d(np.arange(H.n), punct)
    short = np.sort(rng.choice(rest, 300, replace=False))
    a, b, llr, s = frames(H, 0.03, batch, 13)
    a[:, short] = 0
    b[:, short] = 0
    a[:, punct] = rng.integers(0, 2, (batch, punct.size))
    b[:, punct] = rng.integers(0, 2, (batch, punct.size))
    lp = Q.log_p(0.03)
    llr = np.where(b != 0, -lp, lp)
    llr[:, punct] = 1e-4
    llr[:, short] = DBL_MAX
    s = H.syndrome(a)
    for thr_on in (True, False):
        assert_parity("c5_n10240_m2048.sp2", alg, prim, sec, qber=0, batch=batch, thr_on=thr_on, llr=llr, synd=s)


def test_full_batch_properties(gpu_available):
    """BASELINE C2 size (4096 frames): every frame reported as decoded satisfies
    the syndrome, and a seeded sample matches the oracle bit for bit."""
    H = load_fixture("c2_n10240_m2201.alist")
    a, b, llr, s = frames(H, 0.0215, 4096, 99)
    out = graph("c2_n10240_m2201.alist").decode(Q.Params(Q.SPA, 50, True, 100.0), llr, s)
    okf = out.synd_ok.astype(bool)
    assert np.array_equal(H.syndrome(out.bits[okf]), s[okf])
    assert np.all(out.iterations[~okf] == 50) and np.all((out.iterations >= 1) & (out.iterations <= 50))
    sample = np.random.default_rng(0).choice(4096, 24, replace=False)
    O = Oracle(H)
    ob, oi, ok, _ = O.decode_batch(O.params(Q.SPA, 50, True, 100.0), llr[sample], s[sample], threads=16)
    assert np.array_equal(out.bits[sample], ob) and np.array_equal(out.iterations[sample], oi)
    # keys match where decoding succeeded at this operating point (bob_solution == alice)
    assert (out.bits[okf] == a[okf]).all(axis=1).mean() > 0.99


def test_device_qkd_ldpc_pipeline(gpu_available):
    """QKD_LDPC's whole per-trial window on device == host frame build + decode."""
    import torch

    H = load_fixture("c2_n10240_m2201.alist")
    g = graph("c2_n10240_m2201.alist")
    a, b, llr, s = frames(H, 0.0215, 64, 5)
    q = int(H.n * 0.0215) / H.n
    dev = torch.device("cuda:0")
    ta, tb = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    lp = torch.full((64,), Q.log_p(q), dtype=torch.float64, device=dev)
    llr_ws = torch.empty((64, H.n), dtype=torch.float64, device=dev)
    syn_ws = torch.empty((64, H.m), dtype=torch.uint8, device=dev)
    bits = torch.empty((64, H.n), dtype=torch.uint8, device=dev)
    it = torch.empty(64, dtype=torch.int32, device=dev)
    ok = torch.empty(64, dtype=torch.uint8, device=dev)
    km = torch.empty(64, dtype=torch.uint8, device=dev)
    p = Q.Params(Q.SPA, 50, True, 100.0)
    g.qkd_ldpc_device(p, ta, tb, lp, llr_ws, syn_ws, bits, it, ok, km)
    torch.cuda.synchronize()
    assert bits_equal_nan(llr_ws.cpu().numpy(), llr)
    assert np.array_equal(syn_ws.cpu().numpy(), s)
    host = g.decode(p, llr, s)
    assert np.array_equal(bits.cpu().numpy(), host.bits)
    assert np.array_equal(it.cpu().numpy().astype(np.uint32), host.iterations)
    assert np.array_equal(km.cpu().numpy(), (host.bits == a).all(axis=1).astype(np.uint8))
    # no LLR workspace (the bench's form): the register decoder reads the
    # builder's palette codes, the f64 LLRs are never written, same results
    bits.zero_(), it.zero_(), km.zero_()
    g.qkd_ldpc_device(p, ta, tb, lp, None, syn_ws, bits, it, ok, km)
    torch.cuda.synchronize()
    assert np.array_equal(bits.cpu().numpy(), host.bits)
    assert np.array_equal(it.cpu().numpy().astype(np.uint32), host.iterations)
    assert np.array_equal(km.cpu().numpy(), (host.bits == a).all(axis=1).astype(np.uint8))


def test_repeat_calls_deterministic(gpu_available):
    H = load_fixture("c3_n10240_m1801.alist")
    _, _, llr, s = frames(H, 0.016, 200, 3)
    g = graph("c3_n10240_m1801.alist")
    p = Q.Params(Q.OMSA, 50, True, 100.0, 0.77)
    r1 = g.decode(p, llr, s, posterior=True)
    r2 = g.decode(p, llr, s, posterior=True)
    assert np.array_equal(r1.bits, r2.bits) and bits_equal_nan(r1.posterior, r2.posterior)


def test_cpp_mirror_six_decoders_and_batch(gpu_available, tmp_path):
    """The C++ mirror (reference names/signatures) end to end: each per-frame
    decoder and decode_batch agree, and both equal the oracle."""
    import subprocess

    from conftest import ROOT

    name = "c1_n1024_m220.alist"
    H = load_fixture(name)
    _, _, llr, s = frames(H, 0.03, 6, 123)
    fr = tmp_path / "frames.bin"
    with open(fr, "wb") as f:
        f.write(np.int32(llr.shape[0]).tobytes())
        for i in range(llr.shape[0]):
            f.write(llr[i].astype(np.float64).tobytes())
            f.write(s[i].astype(np.int32).tobytes())
    out = tmp_path / "out.bin"
    exe = f"{ROOT}/qkd_ldpc_v_amd/host/host_mirror_check"
    r = subprocess.run([exe, "decoders", matrix_path(name), "1", str(fr), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
    raw = np.fromfile(out, np.uint8)
    rec = 5 + H.n
    O = Oracle(H)
    for k, (alg, prim, sec) in enumerate(ALGS):
        ob, oi, ok, _ = O.decode_batch(O.params(alg, 50, True, 100.0, prim, sec), llr, s, threads=4)
        for f in range(llr.shape[0]):
            b = raw[(k * llr.shape[0] + f) * rec:(k * llr.shape[0] + f + 1) * rec]
            assert int(b[:4].view(np.uint32)[0]) == oi[f] and b[4] == ok[f]
            assert np.array_equal(b[5:], ob[f])


def test_cpp_mirror_kat(gpu_available):
    import subprocess

    from conftest import ROOT

    exe = f"{ROOT}/qkd_ldpc_v_amd/host/host_mirror_check"
    r = subprocess.run([exe, "kat", matrix_path("kat_n6_m4.dense")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "iterations=1 syndromes_match=1 keys_match=1", r.stdout


@pytest.mark.parametrize("alg,prim,sec", ALGS)
def test_nonfinite_and_consistent_frames(gpu_available, alg, prim, sec):
    """Edge inputs: NaN / +-inf channel LLRs in some frames (NaN survives the
    clip), frames whose channel decision already satisfies the
    syndrome (Bob == Alice), and an all-zero key."""
    H = load_fixture("c2_n10240_m2201.alist")
    a, b, llr, s = frames(H, 0.02, 8, 90 + alg)
    llr[0, 5] = np.nan
    llr[1, 7] = np.inf
    llr[2, 9] = -np.inf
    llr[3, [11, 12, 13]] = [np.nan, np.inf, -np.inf]
    lp = Q.log_p(0.02)
    llr[4] = np.where(a[4] != 0, -lp, lp)  # consistent frame
    llr[5] = lp                             # all-zero key, zero syndrome
    s[5] = 0
    assert_parity("c2_n10240_m2201.alist", alg, prim, sec, qber=0, batch=8, llr=llr, synd=s)


def test_zero_batch_and_single_frame(gpu_available):
    H = load_fixture("c1_n1024_m220.alist")
    g = graph("c1_n1024_m220.alist")
    _, _, llr, s = frames(H, 0.02, 1, 3)
    out = g.decode(Q.Params(Q.SPA, 50, True, 100.0), llr[:0], s[:0])
    assert out.bits.shape == (0, H.n)
    assert_parity("c1_n1024_m220.alist", Q.SPA, 0, 0, qber=0, batch=1, llr=llr, synd=s)


@pytest.mark.parametrize("name,alg,prim,sec", [("c1_n1024_m220.alist", Q.SPA, 0.0, 0.0),
                                               ("c3_n10240_m1801.alist", Q.OMSA, 0.77, 0.0)])
def test_host_threads_share_one_graph(gpu_available, name, alg, prim, sec):
    """qldpc_decode_batch called concurrently by host threads on ONE graph (the
    reference's thread pool over trials, src/simulation.cpp:740-746): calls of
    different sizes (the staging buffers grow under other threads), with and
    without posteriors; every frame must equal the oracle's."""
    import threading

    H = load_fixture(name)
    total = 8 * 6 * 5
    _, _, llr, synd = frames(H, 0.02 if alg == Q.SPA else 0.015, total, seed=99)
    O = Oracle(H)
    prm = (alg, 50, True, 100.0, prim, sec)
    ob, oi, ok, op = O.decode_batch(O.params(*prm), llr, synd, threads=16, posterior=True)
    g = Q.Graph(H)
    errors = []

    def worker(t):
        try:
            f = t * 30
            for call, size in enumerate((1, 7, 2, 12, 3, 5)):
                sl = slice(f, f + size)
                out = g.decode(Q.Params(*prm), llr[sl], synd[sl], posterior=(call % 2 == 0))
                for j, fr in enumerate(range(sl.start, sl.stop)):
                    same = (np.array_equal(out.bits[j], ob[fr]) and out.iterations[j] == oi[fr]
                            and out.synd_ok[j] == ok[fr]
                            and (out.posterior is None or bits_equal_nan(out.posterior[j], op[fr])))
                    if not same:
                        errors.append((t, call, fr))
                f += size
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, f"{len(errors)} frames/calls differ; first {errors[:3]}"


@pytest.mark.parametrize("name,alg,prim,sec,qber", [("c2_n10240_m2201.alist", Q.SPA, 0.0, 0.0, 0.0215),
                                                     ("c3_n10240_m1801.alist", Q.OMSA, 0.77, 0.0, 0.016)])
def test_frame_claim_order(gpu_available, monkeypatch, name, alg, prim, sec, qber):
    """The claim order (order.hip) is a permutation of the batch in ascending
    weight |H * z XOR s| of the channel decision z = (llr <= 0) — paletted and
    soft-LLR frames alike, on relabelled graphs — and decoding in index order
    (QLDPC_ORDER=0) gives identical results."""
    import torch

    H = load_fixture(name)
    g = graph(name)
    batch = 300
    _, _, llr, s = frames(H, qber, batch, 17)
    rng = np.random.default_rng(3)
    llr[::7] *= rng.uniform(0.5, 2.0, size=llr[::7].shape)  # soft LLRs: beyond the 4-value palette
    dev = torch.device("cuda:0")
    p = Q.Params(alg, 50, True, 100.0, prim, sec)

    def run():
        tl, ts = torch.from_numpy(llr).to(dev), torch.from_numpy(s).to(dev)
        bits = torch.empty((batch, H.n), dtype=torch.uint8, device=dev)
        it = torch.empty(batch, dtype=torch.int32, device=dev)
        ok = torch.empty(batch, dtype=torch.uint8, device=dev)
        post = torch.empty((batch, H.n), dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)
        g.decode_device(p, tl, ts, bits, it, ok, post, stream=stream)
        torch.cuda.synchronize()
        order, weight = g.last_claim_order(stream)
        return (bits.cpu().numpy(), it.cpu().numpy(), ok.cpu().numpy(), post.cpu().numpy()), order, weight

    r1, order, weight = run()
    assert order is not None and np.array_equal(np.sort(order), np.arange(batch))
    w = (H.syndrome((llr <= 0).astype(np.uint8)) != s).sum(axis=1)
    bad = np.nonzero(weight != w)[0]
    assert bad.size == 0, (f"{bad.size} weights differ; frames {bad[:12].tolist()} gpu {weight[bad[:12]].tolist()} "
                           f"host {w[bad[:12]].tolist()}; gpu weights {weight[:8].tolist()} host {w[:8].tolist()}")
    assert np.all(np.diff(w[order]) >= 0)
    monkeypatch.setenv("QLDPC_DIAG", "1")
    monkeypatch.setenv("QLDPC_ORDER", "0")
    r0, order0, _ = run()
    assert order0 is None
    for x, y in zip(r1[:3], r0[:3]):
        assert np.array_equal(x, y)
    assert bits_equal_nan(r1[3], r0[3])
