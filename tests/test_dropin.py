"""The C++ drop-in: the replacement TU for the reference's
src/qkd_ldpc_algorithm.cpp (qkd_ldpc_v_amd/host/dropin/qkd_ldpc_algorithm.cpp),
compiled against the reference-shaped declarations of tests/dropin/api and
driven by a restatement of run_trial (tests/dropin/run_trial_check.cpp: its
exact two calls, src/simulation.cpp:563-574).  The per-trial results
(iterations_num, syndromes_match, keys_match) must equal the CPU oracle's on
the same trials (run_trial's generator: Xoshiro256++(seed), fill_random_bits,
inject_errors; the punctured draws continue from the same generator).

Built by `make` (the binary travels to the GPU box with the tree)."""
import gzip
import os
import subprocess

import numpy as np
import pytest

import qkd_ldpc_v_amd as Q
from conftest import ROOT, load_fixture, matrix_path
from oracle import pyoracle as P
from oracle.pyoracle import Oracle

BIN = os.path.join(ROOT, "tests", "dropin", "run_trial_check")


def _bin():
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} is not built (make)")
    return BIN


def run(args, tmp_path):
    r = subprocess.run([_bin()] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.split("\n")


def write_list(tmp_path, name, values):
    p = tmp_path / name
    p.write_text("\n".join(str(int(v)) for v in values) + "\n")
    return p


def oracle_trials(H, alg, prim, sec, qber, max_it, seeds, punct=None, short=None):
    """(iterations, syndromes_match, keys_match) per trial from the oracle."""
    O = Oracle(H)
    p = O.params(alg, max_it, True, 100.0, prim, sec)
    out = []
    for sd in seeds:
        if punct is None:
            a, b, q = P.trial(H.n, qber, int(sd))
            lp = np.log((1.0 - q) / q)
            llr = np.where(b != 0, -lp, lp)
            ref = a
        else:
            ref, llr, q = P.trial_rate_adapt(H.n, qber, int(sd), punct, short)
        s = H.syndrome(ref)
        bits, it, ok, _ = O.decode_batch(p, llr[None, :], s[None, :], threads=1)
        out.append((int(it[0]), int(ok[0]), int(np.array_equal(bits[0], ref))))
    return out


def parse(lines, tag=""):
    return [tuple(int(x) for x in ln[len(tag):].split()) for ln in lines if ln.startswith(tag) and ln.strip()]


def test_dropin_binary_loads_matrices_without_gpu():
    out = subprocess.run([_bin(), "load", matrix_path("c2_n10240_m2201.alist"), "1"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and out.stdout.split() == ["10240", "2201", "40960"]


@pytest.mark.gpu
@pytest.mark.parametrize("alg,prim,sec", [(Q.SPA, 0.0, 0.0), (Q.SPA_LIN, 0.0, 0.0), (Q.NMSA, 0.78, 0.0),
                                          (Q.OMSA, 0.77, 0.0), (Q.ANMSA, 0.8, 0.35), (Q.AOMSA, 0.55, 1.2)])
def test_run_trial_qkd_ldpc(gpu_available, tmp_path, alg, prim, sec):
    """Adaptation off: run_trial -> QKD_LDPC, the six decoders on C1."""
    name = "c1_n1024_m220.alist"
    H = load_fixture(name)
    seeds = P.trial_seeds(9012025 + alg, 12)
    sf = write_list(tmp_path, "seeds.txt", seeds)
    got = parse(run(["trials", matrix_path(name), 1, alg, prim, sec, 0.03, 50, sf], tmp_path))
    assert got == oracle_trials(H, alg, prim, sec, 0.03, 50, seeds)


@pytest.mark.gpu
def test_run_trial_qkd_ldpc_c2_spa(gpu_available, tmp_path):
    name = "c2_n10240_m2201.alist"
    H = load_fixture(name)
    seeds = P.trial_seeds(1022025, 6)
    sf = write_list(tmp_path, "seeds.txt", seeds)
    got = parse(run(["trials", matrix_path(name), 1, Q.SPA, 0, 0, 0.0215, 50, sf], tmp_path))
    assert got == oracle_trials(H, Q.SPA, 0.0, 0.0, 0.0215, 50, seeds)


@pytest.mark.gpu
@pytest.mark.parametrize("alg,prim,sec", [(Q.AOMSA, 0.7, 0.99), (Q.SPA, 0.0, 0.0)])
def test_run_trial_qkd_ldpc_rate_adapt(gpu_available, tmp_path, alg, prim, sec):
    """Adaptation on: run_trial -> QKD_LDPC_RATE_ADAPT(..., prng) on the R=0.8
    format-3 code with untainted puncturing (configs/ADAPTIVE T.json point
    QBER 1.56%, delta 0.06, f_EC 1.39)."""
    name = "c5_n10240_m2048.sp2"
    H = load_fixture(name)
    u = np.array(gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split(), np.int32)
    punct, short, _ = Q.adapt_code_rate(H.n, H.m, 0.0156, 0.06, 1.39, u, Q.xoshiro_state(5555))
    assert punct.size > 0 and short.size > 0
    seeds = P.trial_seeds(5555, 6)
    files = [write_list(tmp_path, "seeds.txt", seeds), write_list(tmp_path, "p.txt", punct),
             write_list(tmp_path, "s.txt", short)]
    got = parse(run(["trials", matrix_path(name), 3, alg, prim, sec, 0.0156, 50] + files, tmp_path))
    assert got == oracle_trials(H, alg, prim, sec, 0.0156, 50, seeds, punct, short)


def _permuted_copy(H, tmp_path, seed=7):
    """H with its bit ids permuted (same n, m, nnz; different edges), written in
    format 3 (read_sparse_matrix_2: rows then columns, 0-based)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(H.n)
    rows = [sorted(int(perm[c]) for c in r) for r in H.check_nodes]
    cols = [[] for _ in range(H.n)]
    for j, r in enumerate(rows):
        for c in r:
            cols[c].append(j)
    p = tmp_path / "permuted.sp2"
    with open(p, "w") as f:
        f.write(f"{H.n} {H.m}\n")
        for r in rows:
            f.write(" ".join(map(str, r)) + "\n")
        for c in cols:
            f.write(" ".join(map(str, c)) + "\n")
    return p


@pytest.mark.gpu
def test_graph_cache_same_address_new_edges(gpu_available, tmp_path):
    """The reference's config-after-config loop: a second H of the same shape
    but different edges, loaded into the SAME H_matrix object (same address).
    The content-keyed cache must build a new device graph, not reuse the first."""
    name = "c1_n1024_m220.alist"
    HA = load_fixture(name)
    pB = _permuted_copy(HA, tmp_path)
    HB = Q.load_matrix(str(pB), 3)
    assert (HB.n, HB.m, HB.nnz) == (HA.n, HA.m, HA.nnz) and not np.array_equal(HB.col_idx, HA.col_idx)
    seeds = P.trial_seeds(4242, 8)
    sf = write_list(tmp_path, "seeds.txt", seeds)
    lines = run(["reuse", matrix_path(name), 1, pB, 3, Q.SPA, 0, 0, 0.03, 50, sf], tmp_path)
    assert parse(lines, "A ") == oracle_trials(HA, Q.SPA, 0.0, 0.0, 0.03, 50, seeds)
    assert parse(lines, "B ") == oracle_trials(HB, Q.SPA, 0.0, 0.0, 0.03, 50, seeds)


@pytest.mark.gpu
def test_graph_cache_catches_unsampled_inplace_edit(gpu_available, tmp_path):
    """An in-place edit of H that leaves the O(1) fast key unchanged (two
    unsampled rows swap their check ids) is caught by the cache's periodic
    full-content check (every 32nd hit of an entry): a new device graph."""
    lines = run(["inplace", matrix_path("c2_n10240_m2201.alist"), 1], tmp_path)
    f = [ln for ln in lines if ln.startswith("inplace")][0].split()
    assert f[2] == "1", lines
    assert 1 <= int(f[4]) <= 32, lines


def test_dropin_refuses_non_bit_syndrome():
    """The reference's decoders read syndrome[j] as a sign (any non-zero: -1,
    src/qkd_ldpc_algorithm.cpp:57) and compare it by value (:101); the kernels
    take bits, so the drop-in refuses a syndrome holding anything but 0 / 1,
    before any device work (no GPU needed)."""
    r = subprocess.run([_bin(), "badsyndrome", matrix_path("c1_n1024_m220.alist"), "1"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 1 and "syndrome[1] = 2 is not a bit" in r.stdout, r.stdout + r.stderr


def test_graph_cache_fast_key_is_cheap():
    """The cache's per-call key is O(1): a fingerprint of 128 sampled lists,
    well under the full-content pass (which only a miss takes)."""
    r = subprocess.run([_bin(), "keycost", matrix_path("c2_n10240_m2201.alist"), "1", "300"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    f = r.stdout.split()
    fast, full = float(f[2]), float(f[4])
    assert fast * 5 < full, (fast, full)


# ---- the batch seam: QKD_LDPC_batch_simulation over the drop-in TUs ----------
BATCH = os.path.join(ROOT, "tests", "dropin", "batch_check")


def _batch_bin():
    if not os.path.exists(BATCH):
        pytest.fail(f"{BATCH} is not built (make)")
    return BATCH


def _stats_of(trials, n_trials):
    """process_trials_results' decoding statistics (src/simulation.cpp:580-624)."""
    it = np.array([t[0] for t in trials], np.float64)
    ok = np.array([t[1] for t in trials], bool)
    km = np.array([t[2] for t in trials], bool)
    succ = it[ok]
    mean = succ.mean() if succ.size else 0.0
    std = np.sqrt(((succ - mean) ** 2).sum() / succ.size) if succ.size else 0.0
    return (ok.sum() / n_trials, (ok & km).sum() / n_trials, int(succ.max()) if succ.size else 0,
            int(succ.min()) if succ.size else 0, mean, std)


def _run_batch(tmp_path, name, fmt, alg, prim, sec, qbers, max_it, trials, sim_seed, threads, H, punct=None,
               short=None, devices="0,0,0"):
    qf = tmp_path / "q.txt"
    qf.write_text("\n".join(repr(float(q)) for q in qbers) + "\n")
    files = [qf]
    if punct is not None:
        files += [write_list(tmp_path, "p.txt", punct), write_list(tmp_path, "s.txt", short)]
    args = [_batch_bin(), "batch", matrix_path(name), fmt, alg, prim, sec, files[0], max_it, trials, sim_seed,
            threads] + files[1:]
    env = dict(os.environ, QKD_LDPC_HIP_DEVICES=devices, QLDPC_DIAG="1", QLDPC_TRIAL_CHUNK="5")
    r = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.split("\n")
    seeds = P.trial_seeds(sim_seed, trials)
    for sim, q in enumerate(qbers):
        sd = [(int(s) + sim) & 0xFFFFFFFFFFFFFFFF for s in seeds]
        want = oracle_trials(H, alg, prim, sec, q, max_it, sd, punct, short)
        seam = [tuple(int(x) for x in ln.split()[3:6]) for ln in lines if ln.startswith(f"S {sim} ")]
        pert = [tuple(int(x) for x in ln.split()[3:6]) for ln in lines if ln.startswith(f"T {sim} ")]
        assert seam == want, f"batch seam, combination {sim}"
        assert pert == want, f"per-trial drop-in from {threads} threads, combination {sim}"
        rt = [int(ln.split()[6]) for ln in lines if ln.startswith(f"S {sim} ")]
        assert min(rt) >= 1
        R = [ln.split() for ln in lines if ln.startswith(f"R {sim} ")]
        assert len(R) == 1
        dec, ldpc, it_max, it_min, it_mean, it_std = _stats_of(want, trials)
        r_ = R[0]
        assert float(r_[2]) == dec and float(r_[3]) == ldpc and int(r_[4]) == it_max and int(r_[5]) == it_min
        assert float(r_[6]) == pytest.approx(it_mean, rel=1e-12) and float(r_[7]) == pytest.approx(it_std, rel=1e-9)
        assert float(r_[8]) == int(H.n * q) / H.n
        tp_mean, tp_std, tp_min, tp_max = (int(x) for x in r_[9:13])
        assert 0 < tp_min <= tp_mean <= tp_max and tp_std >= 0
    return lines


@pytest.mark.gpu
def test_batch_seam_qkd_ldpc_three_shards(gpu_available, tmp_path):
    """QKD_LDPC_batch_simulation through the drop-in (adaptation off): every
    trial of two combinations from the batch seam on a 3-logical-shard graph
    (chunks of 5 trials, so both pipeline slots cycle), and from run_trial
    called by 8 concurrent threads through the per-trial drop-in, equals the
    oracle's run_trial; the aggregated sim_results equal the oracle's."""
    name = "c1_n1024_m220.alist"
    H = load_fixture(name)
    _run_batch(tmp_path, name, 1, Q.NMSA, 0.78, 0.0, [0.02, 0.03], 50, 23, 9012025, 8, H)


@pytest.mark.gpu
def test_batch_seam_rate_adapt_three_shards(gpu_available, tmp_path):
    """Adaptation on: the trials run QKD_LDPC_RATE_ADAPT (punctured draws from
    the trial generator) on the R=0.8 format-3 code, AOMSA, 3 logical shards."""
    name = "c5_n10240_m2048.sp2"
    H = load_fixture(name)
    u = np.array(gzip.open(matrix_path("c5_n10240_m2048.untp")).read().split(), np.int32)
    punct, short, _ = Q.adapt_code_rate(H.n, H.m, 0.0156, 0.06, 1.39, u, Q.xoshiro_state(5555))
    _run_batch(tmp_path, name, 3, Q.AOMSA, 0.7, 0.99, [0.0156], 50, 13, 5555, 8, H, punct, short)


@pytest.mark.gpu
def test_batch_seam_spa_c1_one_device(gpu_available, tmp_path):
    """SPA with the default device list (every GPU of the box)."""
    name = "c1_n1024_m220.alist"
    H = load_fixture(name)
    _run_batch(tmp_path, name, 1, Q.SPA, 0.0, 0.0, [0.025], 50, 16, 777, 4, H, devices="0")
