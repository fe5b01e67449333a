"""Seeded regular LDPC codes for configurations whose matrix file is absent
upstream (the n=102400 R=0.79 dv=4 file is listed in
`sparse_matrices/.MISSING_LARGE_BLOBS:3`, so the benchmark also runs a
build-generated code of the same shape).

Construction: socket model.  Row degrees are as equal as E = n*dv allows (the
first E mod m rows get one more edge), the E row sockets are shuffled by a
numpy PCG64 generator with the given seed, bit b takes sockets [dv*b, dv*b+dv),
and a bit that drew one row twice swaps the repeat with a socket of another
bit until every bit has dv distinct rows.  Deterministic for (n, m, dv, seed).
Not a reference algorithm: the decoder's parity against the oracle does not
depend on which code it runs."""
import numpy as np

from .graph import HMatrix


def regular_code(n: int, m: int, dv: int, seed: int) -> HMatrix:
    if n <= 0 or m <= 0 or dv <= 0 or dv > m:
        raise ValueError("need n, m > 0 and 0 < dv <= m")
    E = n * dv
    deg = np.full(m, E // m, np.int64)
    deg[:E % m] += 1
    rng = np.random.Generator(np.random.PCG64(seed))
    sockets = rng.permutation(np.repeat(np.arange(m, dtype=np.int64), deg)).reshape(n, dv)
    for _ in range(100 * n):
        srt = np.sort(sockets, axis=1)
        bad = np.nonzero((srt[:, 1:] == srt[:, :-1]).any(axis=1))[0]
        if bad.size == 0:
            break
        for b in bad:
            row = sockets[b]
            vals, cnt = np.unique(row, return_counts=True)
            if not (cnt > 1).any():  # fixed by an earlier swap
                continue
            dup = int(vals[cnt > 1][0])
            j = int(np.nonzero(row == dup)[0][1])
            while True:  # a partner bit c and slot i such that the swap keeps both distinct
                c = int(rng.integers(n))
                i = int(rng.integers(dv))
                r2 = int(sockets[c, i])
                if c != b and r2 not in row and dup not in sockets[c]:
                    sockets[b, j], sockets[c, i] = r2, dup
                    break
    else:
        raise RuntimeError("socket repair did not converge")
    rows = [[] for _ in range(m)]
    for b in range(n):
        for r in sockets[b]:
            rows[int(r)].append(b)
    return HMatrix.from_check_nodes(n, [sorted(r) for r in rows])
