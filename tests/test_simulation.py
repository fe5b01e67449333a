"""Config-driven simulation driver: configuration parsing
(current and legacy schemas), combination building, the results CSV, and — on
the GPU — whole simulations whose statistics are recomputed from the oracle."""
import gzip
import json
import math
import os
import shutil

import numpy as np
import pytest

import qkd_ldpc_v_amd as Q
from conftest import ROOT, load_fixture, matrix_path
from oracle import pyoracle as P
from oracle.pyoracle import Oracle
from qkd_ldpc_v_amd import simulation as S

CFG_DIR = os.path.join(ROOT, "tests", "golden", "configs")


def cfg_path(name):
    return os.path.join(CFG_DIR, name + ".json")


def mtrx_dir(tmp_path, fixture, with_untp=None):
    d = tmp_path / "matrices"
    d.mkdir(exist_ok=True)
    stem = fixture.rsplit(".", 1)[0]
    (d / (stem + ".mtrx")).write_bytes(gzip.open(matrix_path(fixture)).read())
    if with_untp:
        (d / (stem + ".untp")).write_bytes(gzip.open(matrix_path(with_untp)).read())
    return str(d)


def test_parse_current_and_legacy_configs():
    c = S.Config.load(cfg_path("adaptive_t"))
    assert (c.decoding_algorithm, c.trials_number, c.simulation_seed) == (5, 10, 5555)
    assert c.rate_adaptation and c.untainted_puncturing and not c.use_adaptation_ranges
    assert len(c.adaptation_maps) == 26 and [m["code_rate"] for m in c.adaptation_maps] == sorted(
        m["code_rate"] for m in c.adaptation_maps)
    assert c.primary["maps"][0] == {"code_rate": 0.505, "value": 0.72}
    legacy = S.Config.load(cfg_path("legacy_10k_spa_fer001"))
    assert legacy.decoding_algorithm == 0 and not legacy.rate_adaptation and len(legacy.qber_ranges) == 22
    oldest = S.Config.load(cfg_path("legacy_1k"))
    assert oldest.decoding_algorithm == 0 and oldest.simulation_seed == 9012025


def test_config_errors_mirror_the_reference(tmp_path):
    c = json.load(open(cfg_path("adaptive_t")))
    c["trials_number"] = 0
    p = tmp_path / "bad.json"
    p.write_text(json.dumps(c))
    with pytest.raises(S.ConfigError, match="Number of trials must be > 0!"):
        S.Config.load(str(p))
    c = json.load(open(cfg_path("adaptive_t")))
    del c["decoding_algorithm_max_iterations"]
    p.write_text(json.dumps(c))
    with pytest.raises(S.ConfigError, match="missing configuration parameter"):
        S.Config.load(str(p))


@pytest.mark.parametrize("field,value,msg", [
    ("code_rate", 1.0, "Code rate\\(R\\) must be: 0 < R < 1!"),
    ("delta", {"begin": 0.2, "end": 0.1, "step": 0.01}, "Invalid delta begin or end parameters"),
    ("delta", {"begin": 0.0, "end": 0.1, "step": 0.01}, "Invalid delta begin or end parameters"),
    ("delta", {"begin": 0.05, "end": 0.1, "step": 0.0}, "Delta step must be > 0!"),
    ("delta", {"begin": 0.05, "end": 0.1, "step": 0.2}, "Delta step is too large."),
    ("efficiency", {"begin": 0.9, "end": 1.2, "step": 0.1}, "Invalid efficiency begin or end parameters"),
    ("efficiency", {"begin": 1.3, "end": 1.2, "step": 0.1}, "Invalid efficiency begin or end parameters"),
    ("efficiency", {"begin": 1.0, "end": 1.2, "step": 0.0}, "Efficiency step must be > 0!"),
    ("efficiency", {"begin": 1.0, "end": 1.2, "step": 0.5}, "Efficiency step is too large."),
])
def test_adaptation_ranges_validation_mirrors_the_reference(tmp_path, field, value, msg):
    """code_rate_adaptation_parameters_ranges checks of src/config.cpp:327-354."""
    c = json.load(open(cfg_path("adaptive_t")))
    ra = c["code_rate_adaptation_parameters"]
    ra["use_adaptation_parameters_ranges"] = True
    good = {"code_rate": 0.8, "delta": {"begin": 0.05, "end": 0.1, "step": 0.01},
            "efficiency": {"begin": 1.0, "end": 1.2, "step": 0.1}}
    ra["code_rate_adaptation_parameters_ranges"] = [good]
    p = tmp_path / "ok.json"
    p.write_text(json.dumps(c))
    assert S.Config.load(str(p)).adaptation_ranges[0]["delta"] == (0.05, 0.1, 0.01)
    bad = dict(good)
    bad[field] = value
    ra["code_rate_adaptation_parameters_ranges"] = [good, bad]
    p.write_text(json.dumps(c))
    with pytest.raises(S.ConfigError, match=msg):
        S.Config.load(str(p))


def test_driver_log_p_is_the_c_library_log():
    """The a-priori LLR magnitude qldpc_run_trials (the driver's seam) uses is
    log((1-q)/q) by the C library, qldpc_log_p, as the reference computes it
    (src/qkd_ldpc_algorithm.cpp:1043): at n=10240, n_err=229 numpy's log differs
    from it by one ulp on some hosts, which would change every LLR of the frame."""
    for n, ne in ((10240, 229), (10240, 689), (102400, 2290), (102400, 5764), (1024, 13)):
        q = ne / n
        want = Q.log_p(q)
        import ctypes
        libm = ctypes.CDLL("libm.so.6")
        libm.log.restype = ctypes.c_double
        libm.log.argtypes = [ctypes.c_double]
        assert want == libm.log((1.0 - q) / q)


def test_rate_adapted_combinations_match_oracle_chain(tmp_path):
    cfg = S.Config.load(cfg_path("adaptive_t"))
    d = mtrx_dir(tmp_path, "c5_n10240_m2048.sp2", "c5_n10240_m2048.untp")
    mats, combos = S.prepare(cfg, S.matrix_files(d))
    H = load_fixture("c5_n10240_m2048.sp2")
    unt = np.array(gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split(), np.int32)
    st = Q.xoshiro_state(cfg.simulation_seed)
    want = []
    for m in cfg.adaptation_maps:
        if m["code_rate"] != 0.805:
            continue
        p, s = P.adapt_code_rate(H.n, H.m, m["QBER"], m["delta"], m["efficiency"], unt, st)
        if p.size or s.size:
            want.append((m["QBER"], p, s))
    assert len(combos) == len(want) > 0
    for c, (q, p, s) in zip(combos, want):
        assert c.config_qber == q and np.array_equal(c.punctured, p) and np.array_equal(c.shortened, s)
        assert (c.primary, c.secondary) == (0.7, 0.99)  # beta / sigma maps at code rate 0.805
        assert c.bits_to_remove >= p.size + s.size


def test_missing_untp_is_searched_and_written(tmp_path):
    """get_punctured_bits_untainted (:1076-1123): no .untp -> the search runs on
    the setup generator before the combinations' draws, and the file is
    written (one line, indices each followed by a space) and read back next time."""
    cfg = S.Config.load(cfg_path("adaptive_t"))
    d = mtrx_dir(tmp_path, "c5_n10240_m2048.sp2")
    mats, combos = S.prepare(cfg, S.matrix_files(d))
    untp = [f for f in os.listdir(d) if f.endswith(".untp")]
    assert len(untp) == 1
    text = open(os.path.join(d, untp[0])).read()
    H = load_fixture("c5_n10240_m2048.sp2")
    st = Q.xoshiro_state(cfg.simulation_seed)
    unt = Q.select_punctured_untainted(H, st)
    assert text == "".join(f"{v} " for v in unt) and "\n" not in text
    want = []
    for m in cfg.adaptation_maps:
        if m["code_rate"] != 0.805:
            continue
        p, s = P.adapt_code_rate(H.n, H.m, m["QBER"], m["delta"], m["efficiency"], unt, st)
        if p.size or s.size:
            want.append((m["QBER"], p, s))
    assert len(combos) == len(want) > 0
    for c, (q, p, s) in zip(combos, want):
        assert c.config_qber == q and np.array_equal(c.punctured, p) and np.array_equal(c.shortened, s)
    # second run: the written file is read, no search draws
    mats2, combos2 = S.prepare(cfg, S.matrix_files(d))
    st2 = Q.xoshiro_state(cfg.simulation_seed)
    first = next(m for m in cfg.adaptation_maps if m["code_rate"] == 0.805)
    p2, s2 = P.adapt_code_rate(H.n, H.m, first["QBER"], first["delta"], first["efficiency"], unt, st2)
    assert np.array_equal(combos2[0].shortened, s2)


def test_range_values_and_qber_buckets():
    assert S._range_values(0.01, 0.05, 0.01) == [0.01 + j * 0.01 for j in range(5)]
    assert S._range_values(0.3, 0.3, 0.1) == [0.3]
    cfg = S.Config.load(cfg_path("legacy_10k_spa_fer001"))
    qs = S._rate_qber_values(cfg, 1 - 2201 / 10240)  # the C2 matrix's bucket (0.795)
    assert qs == [0.0215]


def test_results_csv_format(tmp_path):
    cfg = S.Config.load(cfg_path("adaptive_t"))
    cfg.enable_throughput_measurement = False
    r = {"sim_number": 0, "matrix_filename": "x.mtrx", "is_regular": False, "n": 10240, "m": 2048,
         "config_qber": 0.0116, "accurate_qber": 0.0115234375, "iter_mean": 12.345, "iter_std": 1.5, "iter_min": 7,
         "iter_max": 20, "ratio_success_dec": 1.0, "ratio_success_ldpc": 0.9, "delta": 0.09, "efficiency": 1.5,
         "punct_fraction": 0.05, "short_fraction": 0.04, "adapted_rate": 0.83, "primary": 0.7, "secondary": 0.99}
    path = S.write_results(cfg, [r], "00h-00m-01s", str(tmp_path))
    lines = open(path).read().splitlines()
    assert os.path.basename(path) == ("ldpc(trial_num=10,dec_alg=AOMSA,max_dec_alg_iters=100,priv_maint=ON,"
                                      "rate_adapt=ON[punct=untainted],seed=5555,sim_duration=00h-00m-01s).csv")
    assert lines[0].endswith(";FER;DELTA;EFFICIENCY;PUNCT_FRACTION;SHORT_FRACTION;R_ADAPTED;BETA;SIGMA")
    assert lines[1] == ("0;x.mtrx;irregular;0,800;2048;10240;0,0116;0,0115;12,35;1,50;7;20;1;0,9;0,1;"
                        "0,090;1,500;0,050;0,040;0,830;0,700;0,990")


def test_bits_to_remove_properties():
    H = load_fixture("c1_n1024_m220.alist")
    k = S._bits_to_remove(H)
    assert 0 < k <= H.m
    p = np.array([3, 10, 500], np.int32)
    s = np.array([4, 11], np.int32)
    assert S._bits_to_remove(H, p, s) >= 5


def _oracle_stats(H, alg, prim, sec, thr, max_it, q, seeds, sim, punct=None, short=None):
    O = Oracle(H)
    llrs, alices = [], []
    for sd in seeds:
        sd = (int(sd) + sim) & 0xFFFFFFFFFFFFFFFF
        if punct is None:
            a, b, qa = P.trial(H.n, q, sd)
            lp = Q.log_p(qa)  # the C library log, as the driver and the reference (:1043)
            llrs.append(np.where(b != 0, -lp, lp))
            alices.append(a)
        else:
            a, l, qa = P.trial_rate_adapt(H.n, q, sd, punct, short)
            llrs.append(l)
            alices.append(a)
    A, L = np.stack(alices), np.stack(llrs)
    bits, it, ok, _ = O.decode_batch(O.params(alg, max_it, True, thr, prim, sec), L, H.syndrome(A), threads=8)
    km = (bits == A).all(axis=1)
    return it, ok.astype(bool), km, qa


@pytest.mark.gpu
def test_simulation_end_to_end_matches_oracle(gpu_available, tmp_path):
    c = json.load(open(cfg_path("legacy_1k")))
    c["trials_number"] = 40
    c["code_rate_QBER_maps"] = [{"code_rate": 0.9, "QBER_begin": 0.02, "QBER_end": 0.03, "QBER_step": 0.01}]
    c["enable_throughput_measurement"] = True
    c["throughput_measurement_parameters"] = {"consider_RTT": False, "RTT": 0}
    cp = tmp_path / "c1.json"
    cp.write_text(json.dumps(c))
    cfg = S.Config.load(str(cp))
    d = mtrx_dir(tmp_path, "c1_n1024_m220.alist")
    mats, combos = S.prepare(cfg, S.matrix_files(d))
    assert [x.config_qber for x in combos] == [0.02, 0.03]
    res = S.run(cfg, mats, combos, log=lambda *a: None)
    for r in res:  # per-trial throughput distribution (src/simulation.cpp:626-681), not one amortised value
        assert 0 < r["tp_min"] <= r["tp_mean"] <= r["tp_max"] and r["tp_std"] > 0 and r["tp_min"] < r["tp_max"]
    H = load_fixture("c1_n1024_m220.alist")
    seeds = Q.trial_seeds(cfg.simulation_seed, cfg.trials_number)
    for sim, (r, cb) in enumerate(zip(res, combos)):
        it, ok, km, qa = _oracle_stats(H, 0, 0, 0, cfg.threshold, cfg.max_iterations, cb.config_qber, seeds, sim)
        assert r["ratio_success_dec"] == ok.mean() and r["ratio_success_ldpc"] == (ok & km).mean()
        assert r["accurate_qber"] == qa
        if ok.any():
            assert r["iter_mean"] == pytest.approx(it[ok].mean()) and r["iter_max"] == it[ok].max()
    path = S.write_results(cfg, res, "00h-00m-00s", str(tmp_path / "results"))
    assert len(open(path).read().splitlines()) == 3


@pytest.mark.gpu
def test_rate_adapted_simulation_matches_oracle(gpu_available, tmp_path):
    c = json.load(open(cfg_path("adaptive_t")))
    c["trials_number"] = 12
    cp = tmp_path / "a.json"
    cp.write_text(json.dumps(c))
    cfg = S.Config.load(str(cp))
    d = mtrx_dir(tmp_path, "c5_n10240_m2048.sp2", "c5_n10240_m2048.untp")
    mats, combos = S.prepare(cfg, S.matrix_files(d))
    combos = combos[:3]
    res = S.run(cfg, mats, combos, log=lambda *a: None)
    H = load_fixture("c5_n10240_m2048.sp2")
    seeds = Q.trial_seeds(cfg.simulation_seed, cfg.trials_number)
    for sim, (r, cb) in enumerate(zip(res, combos)):
        it, ok, km, qa = _oracle_stats(H, 5, cb.primary, cb.secondary, cfg.threshold, cfg.max_iterations,
                                       cb.config_qber, seeds, sim, cb.punctured, cb.shortened)
        assert r["ratio_success_dec"] == ok.mean() and r["ratio_success_ldpc"] == (ok & km).mean()
        if ok.any():
            assert r["iter_mean"] == pytest.approx(it[ok].mean())


def test_throughput_stats_restates_process_trials_results():
    """THROUGHPUT_* (src/simulation.cpp:626-681): per-trial bits/s, mean and
    population std over TRIALS_NUMBER, RTT added to each runtime, truncated."""
    rt = np.array([10.0, 20.0, 40.0, 80.0])
    mean, std, lo, hi = S.throughput_stats(8000, rt, 4)
    tp = 8000 * 1e6 / rt
    assert (mean, lo, hi) == (int(tp.mean()), int(tp.min()), int(tp.max()))
    assert std == int(math.sqrt(((tp - tp.mean()) ** 2).mean()))
    assert lo <= mean <= hi and std > 0
    m2, _, lo2, hi2 = S.throughput_stats(8000, rt, 4, rtt_ms=0.4)
    assert hi2 == int(8000 * 1e6 / (10.0 + 400.0)) and m2 < mean and lo2 < lo
    # runtimes are whole microseconds (trial_result::runtime), rounded to
    # nearest and >= 1 — the C++ batch seam's rule (simulation_batch.cpp)
    assert S.throughput_stats(8000, np.array([9.6, 20.4, 39.5, 80.0]), 4) == (mean, std, lo, hi)
    assert S.throughput_stats(1000, np.array([0.2]), 1)[2] == int(1000 * 1e6 / 1.0)
