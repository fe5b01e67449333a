"""Synthetic BSC trials (host input generation, not timed).

The reference's trial (src/simulation.cpp:540-557; fill_random_bits /
inject_errors, src/array_and_matrix_operations.cpp:889-933): Alice's key is
i.i.d. Bernoulli(1/2); Bob's key is Alice's with exactly floor(n * QBER) bits
flipped at distinct uniformly random positions; the accurate QBER is
floor(n*QBER)/n.  This generator reproduces that distribution with numpy's
PCG64 (seeded, vectorised over frames) for tests and the smoke check; the
reference-identical trials (Xoshiro256++ seeds, libstdc++ draw consumption)
are `qkd_ldpc_v_amd.trials_device` / `trials_rate_adapt_device` (trials.hip),
which bench.py and the simulation driver use.
"""
from __future__ import annotations

import numpy as np


def bsc_frames(n: int, qber: float, batch: int, seed: int = 0):
    """Return (alice uint8[batch,n], bob uint8[batch,n], accurate_qber)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    num_errors = int(float(n) * qber)  # static_cast<size_t>(n * QBER), :913
    alice = rng.integers(0, 2, size=(batch, n), dtype=np.uint8)
    bob = alice.copy()
    if num_errors > 0:
        # distinct positions per frame: argpartition of uniform keys
        keys = rng.random((batch, n), dtype=np.float32)
        pos = np.argpartition(keys, num_errors - 1, axis=1)[:, :num_errors]
        rows = np.repeat(np.arange(batch), num_errors)
        bob[rows, pos.ravel()] ^= 1
    return alice, bob, num_errors / n
