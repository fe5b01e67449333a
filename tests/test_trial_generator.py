"""Trial generator: the reference's run_trial keys.

CPU: the oracle's generator (libstdc++'s own uniform_int_distribution and
std::shuffle over a restated Xoshiro256++) against an independent pure-Python
restatement of the same algorithms, and the product's host seed sequence
against the oracle.  GPU: qldpc_trials_device against the oracle, bit for bit.
Upstream Xoshiro-cpp is not in the image: the generator itself is parity
unpinned against it (published algorithm, SplitMix64 seeding)."""
import numpy as np
import pytest

import qkd_ldpc_v_amd as Q
from oracle import pyoracle as P

M64 = (1 << 64) - 1


class PyXoshiro:
    def __init__(self, seed):
        x = seed & M64
        self.s = []
        for _ in range(4):
            x = (x + 0x9E3779B97F4A7C15) & M64
            z = x
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            self.s.append(z ^ (z >> 31))

    @staticmethod
    def rotl(v, k):
        return ((v << k) | (v >> (64 - k))) & M64

    def __call__(self):
        s = self.s
        r = (self.rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = self.rotl(s[3], 45)
        return r


def py_below(g, rng):  # libstdc++ _S_nd<unsigned __int128>
    p = g() * rng
    lo = p & M64
    if lo < rng:
        thr = ((1 << 64) - rng) % rng
        while lo < thr:
            p = g() * rng
            lo = p & M64
    return p >> 64


def py_trial(n, qber, seed):
    g = PyXoshiro(seed)
    a = [py_below(g, 2) for _ in range(n)]
    ne = int(float(n) * qber)
    b = list(a)
    pos = list(range(n))
    i = 1
    if n % 2 == 0:
        d = py_below(g, 2)
        pos[1], pos[d] = pos[d], pos[1]
        i = 2
    while i != n:
        b0 = i + 1
        x = py_below(g, b0 * (b0 + 1))
        p1, p2 = x // (b0 + 1), x % (b0 + 1)
        pos[i], pos[p1] = pos[p1], pos[i]
        pos[i + 1], pos[p2] = pos[p2], pos[i + 1]
        i += 2
    for e in range(ne):
        b[pos[e]] ^= 1
    return np.array(a, np.uint8), np.array(b, np.uint8), ne / n


def py_trial_prefix(n, qber, seed):
    """The device generator's form (trials.hip): the same draws, but the
    shuffle keeps only the k = floor(n*qber) prefix inject_errors reads — a
    swap at position pos >= k only writes a[p] = pos when p < k (a[pos] is
    still pos then)."""
    g = PyXoshiro(seed)
    a = [py_below(g, 2) for _ in range(n)]
    k = int(float(n) * qber)
    pre = list(range(k))

    def swap(pos, p):
        if pos < k:
            pre[pos], pre[p] = pre[p], pre[pos]
        elif p < k:
            pre[p] = pos

    if k > 0:
        i = 1
        if n % 2 == 0:
            swap(1, py_below(g, 2))
            i = 2
        while i != n:
            b0 = i + 1
            x = py_below(g, b0 * (b0 + 1))
            swap(i, x // (b0 + 1))
            swap(i + 1, x % (b0 + 1))
            i += 2
    b = list(a)
    for p in pre:
        b[p] ^= 1
    return np.array(a, np.uint8), np.array(b, np.uint8)


@pytest.mark.parametrize("n,qber,seed", [(1024, 0.0215, 5), (1023, 0.05, 2**63 + 11), (2048, 0.0005, 77),
                                         (1025, 0.3, 9), (10240, 0.013, 1022025)])
def test_prefix_shuffle_equals_full_shuffle(n, qber, seed):
    """The k-prefix shuffle the device runs gives the full shuffle's keys."""
    a, b, _ = py_trial(n, qber, seed)
    pa, pb = py_trial_prefix(n, qber, seed)
    assert np.array_equal(a, pa) and np.array_equal(b, pb)


def py_trial_segmented(n, qber, seed, n_punct=0):
    """The segment-parallel device generator's form (trials.hip): every draw's
    meaning comes from its index in the trial's stream (Alice's n bits, the
    shuffle's S draws, the punctured pairs); a shuffle step at a position
    i < k goes to pbuf[i] and is replayed in order, one at i >= k only
    contributes a[p] = i for p < k, where the largest i wins (the draw
    kernel's atomic max); a rejected draw would flag the trial."""
    g = PyXoshiro(seed)
    k = int(float(n) * qber)
    S = n // 2 if n % 2 == 0 else (n - 1) // 2
    a = [g() >> 63 for _ in range(n)]
    pbuf = [0] * max(k, 1)
    last = [0] * max(k, 1)
    rejected = False

    def record(pos, p):
        if pos < k:
            pbuf[pos] = p
        elif p < k:
            last[p] = max(last[p], pos)

    for t in range(S):
        if n % 2 == 0 and t == 0:
            record(1, g() >> 63)
            continue
        i = 2 * t if n % 2 == 0 else 2 * t + 1
        b1 = i + 2
        rng = (i + 1) * b1
        x = g()
        lo = (x * rng) & M64
        if lo < rng and lo < ((1 << 64) - rng) % rng:
            rejected = True
        hi = (x * rng) >> 64
        p1 = int(float(hi) / float(b1))  # the kernel's f64 quotient (exact below 2^51)
        record(i, p1)
        record(i + 1, hi - p1 * b1)
    pa, pb = [], []
    for _ in range(n_punct):
        pa.append(g() >> 63)
        pb.append(g() >> 63)
    pre = list(range(k))
    for pos in range(1, k):
        p = pbuf[pos]
        pre[p], pre[pos] = pos, pre[p]
    b = list(a)
    for j in range(k):
        b[last[j] if last[j] else pre[j]] ^= 1
    return np.array(a, np.uint8), np.array(b, np.uint8), rejected, pa, pb


@pytest.mark.parametrize("n,qber,seed", [(1024, 0.0215, 5), (1023, 0.05, 2**63 + 11), (2048, 0.0005, 77),
                                         (1025, 0.3, 9), (10240, 0.013, 1022025), (6, 0.34, 3), (7, 0.15, 1),
                                         (2, 0.5, 4)])
def test_segmented_generator_equals_full_shuffle(n, qber, seed):
    """The segment-parallel generator's prefix replay + last-writer merge gives
    the full shuffle's keys (no rejection on these streams)."""
    a, b, _ = py_trial(n, qber, seed)
    sa, sb, rej, _, _ = py_trial_segmented(n, qber, seed)
    assert not rej
    assert np.array_equal(a, sa) and np.array_equal(b, sb)


def test_f64_quotient_is_exact_below_2_51():
    """split_two (trials.hip): floor(fl(x / b1)) == x // b1 for x < 2^51."""
    rng = np.random.default_rng(5)
    xs = [int(v) for v in rng.integers(0, 1 << 51, 200000, dtype=np.int64)]
    bs = [int(v) for v in rng.integers(2, 1 << 26, 200000, dtype=np.int64)]
    for x, b1 in zip(xs, bs):
        assert int(float(x) / float(b1)) == x // b1
    for b1 in (3, 7, 102401, 102402, (1 << 25) + 1):  # quotients just below an integer
        for q in (1, 12345, (1 << 51) // b1 - 1):
            x = q * b1 - 1
            assert int(float(x) / float(b1)) == x // b1


def test_f32_quotient_estimate_within_one():
    """split_two's f32 path (trials.hip, b1 < 2^20): the truncated estimate
    fl(fl(fma(hi, 2^32, fl(lo))) * r) with r within one ulp of 1 / b1 (the
    hardware reciprocal's bound) is within one of floor(x / b1), so one
    remainder correction gives the exact (x / b1, x % b1)."""
    rng = np.random.default_rng(11)
    f32 = np.float32
    for b1 in list(rng.integers(3, 1 << 20, 3000)) + [3, 4, 102402, (1 << 20) - 1]:
        b1 = int(b1)
        xs = [int(v) for v in rng.integers(0, b1 * (b1 - 1), 40, dtype=np.int64)] + [b1 * (b1 - 1) - 1, b1 - 1, 0]
        r0 = f32(1.0) / f32(b1)
        for r in (r0, np.nextafter(r0, f32(0)), np.nextafter(r0, f32(1))):
            for x in xs:
                xf = f32(float(x >> 32) * 4294967296.0 + float(f32(x & 0xFFFFFFFF)))
                q = int(f32(xf * r))
                assert abs(q - x // b1) <= 1, (b1, x)


@pytest.mark.parametrize("n,qber,seed", [(1024, 0.0215, 5), (1023, 0.05, 2**63 + 11), (10240, 0.013, 1022025)])
def test_oracle_trial_matches_python_restatement(n, qber, seed):
    a, b, q = P.trial(n, qber, seed)
    pa, pb, pq = py_trial(n, qber, seed)
    assert np.array_equal(a, pa) and np.array_equal(b, pb) and q == pq
    assert int((a != b).sum()) == int(n * qber)


@pytest.mark.parametrize("seed,draws", [(1, 0), (1, 1), (9012025, 1024), (1022025, 10240), (2**64 - 7, 102400)])
def test_xoshiro_jump_matrix(seed, draws):
    """The device generator's second wave starts from J_n . s (GF(2) jump,
    trials.hip): the host jump equals stepping the generator `draws` times."""
    g = PyXoshiro(seed)
    for _ in range(draws):
        g()
    out = np.zeros(4, np.uint64)
    Q._lib.check(Q.lib().qldpc_xoshiro_jump(seed, draws, out.ctypes.data), "qldpc_xoshiro_jump")
    assert [int(v) for v in out] == g.s


def test_seed_sequences_agree():
    g = PyXoshiro(1022025)
    want = np.array([g() for _ in range(16)], np.uint64)
    assert np.array_equal(P.trial_seeds(1022025, 16), want)
    assert np.array_equal(P.xoshiro(1022025, 16), want)
    assert np.array_equal(Q.trial_seeds(1022025, 16), want)


@pytest.mark.gpu
@pytest.mark.parametrize("n,qber,batch", [(1024, 0.013, 24), (1024, 0.0015, 130), (10240, 0.0215, 24),
                                           (10241, 0.05, 24), (102400, 0.038, 4), (102400, 0.13, 2),
                                           (102400, 0.2, 2)])
def test_device_trials_bitexact(gpu_available, n, qber, batch):
    """(batch 130: three groups of 64 trials, the last partial; n = 10241 and
    1024 with batch 24: the byte-store path and a single segment group; the
    finish kernel resolves k <= 12288 prefix swaps in parallel, replays
    k = 13312 on one thread in LDS and k = 20480 in global memory)"""
    import torch

    seeds = Q.trial_seeds(9012025, batch)
    d_seeds = torch.from_numpy(seeds.view(np.int64)).cuda()
    da = torch.empty((batch, n), dtype=torch.uint8, device="cuda")
    db = torch.empty_like(da)
    q = Q.trials_device(n, qber, d_seeds, da, db, seed_add=3)
    torch.cuda.synchronize()
    A, B = da.cpu().numpy(), db.cpu().numpy()
    for f in range(batch):
        a, b, qo = P.trial(n, qber, (int(seeds[f]) + 3) & M64)
        assert np.array_equal(A[f], a) and np.array_equal(B[f], b), f"trial {f} differs"
        assert q == qo


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("n,qber,batch,n_punct", [(10240, 0.0215, 70, 0), (1023, 0.05, 5, 0), (10240, 0.0156, 9, 37)])
def test_device_trials_serial_rerun_bitexact(gpu_available, monkeypatch, n, qber, batch, n_punct, mode):
    """QLDPC_TRIAL_SERIAL=1 sends every trial through the finish kernel's
    sequential rerun — the path a trial with a rejected shuffle draw takes —
    and =2 through the one-thread replay of the prefix swaps (the path of
    12288 < k <= 16384) instead of the parallel resolution: both must give
    the same keys and punctured draws as the oracle."""
    import torch

    monkeypatch.setenv("QLDPC_DIAG", "1")
    monkeypatch.setenv("QLDPC_TRIAL_SERIAL", mode)
    seeds = Q.trial_seeds(1022025, batch)
    d_seeds = torch.from_numpy(seeds.view(np.int64)).cuda()
    da = torch.empty((batch, n), dtype=torch.uint8, device="cuda")
    db = torch.empty_like(da)
    if n_punct:
        pa = torch.empty((batch, n_punct), dtype=torch.uint8, device="cuda")
        pb = torch.empty_like(pa)
        Q.trials_rate_adapt_device(n, qber, d_seeds, n_punct, da, db, pa, pb, seed_add=2)
    else:
        Q.trials_device(n, qber, d_seeds, da, db, seed_add=2)
    torch.cuda.synchronize()
    A, B = da.cpu().numpy(), db.cpu().numpy()
    for f in range(batch):
        a, b, _, spa, spb = py_trial_segmented(n, qber, (int(seeds[f]) + 2) & M64, n_punct)
        assert np.array_equal(A[f], a) and np.array_equal(B[f], b), f"trial {f} differs"
        if n_punct:
            assert pa[f].cpu().tolist() == spa and pb[f].cpu().tolist() == spb


def test_too_small_for_qber_is_an_error():
    with pytest.raises(Q.QLDPCError, match="too small for QBER"):
        Q._lib.check(Q.lib().qldpc_trials_device(10, 0.01, 0, None, 0, None, None, None, None), "trials")
