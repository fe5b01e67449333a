"""Debug: posterior differences of one parity case (GPU vs oracle)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import qkd_ldpc_v_amd as Q
from conftest import load_fixture
from oracle.pyoracle import Oracle
name = sys.argv[1] if len(sys.argv) > 1 else "c1_n1024_m220.alist"
alg = int(sys.argv[2]) if len(sys.argv) > 2 else 0
qber = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05
H = load_fixture(name)
a, b, q = Q.bsc_frames(H.n, qber, 8, seed=0)
lp = Q.log_p(q)
llr = np.where(b != 0, -lp, lp).astype(np.float64)
s = H.syndrome(a)
g = Q.Graph(H)
print("plan", g.plan(0, alg))
try:
    print("labels", g.labels()[1])
except Exception as e:
    print("labels n/a", e)
for it in (1, 2):
    out = g.decode(Q.Params(alg, it, True, 100.0, 0.78, 0.35), llr, s, posterior=True)
    O = Oracle(H)
    ob, oi, ok, op = O.decode_batch(O.params(alg, it, True, 100.0, 0.78, 0.35), llr, s, threads=4, posterior=True)
    for f in range(2):
        d = set(np.nonzero(out.posterior[f].view(np.uint64) != op[f].view(np.uint64))[0].tolist())
        rows = [j for j, r in enumerate(H.check_nodes) if all(c in d for c in r)]
        print("max_it", it, "frame", f, "ndiff", len(d), "rows fully differing", rows)
        if it == 1:
            for j in rows[:6]:
                r = H.check_nodes[j]
                par = int(np.sum(llr[f][r] <= 0)) & 1
                print("   row", j, "deg", len(r), "s", int(s[f][j]), "par", par,
                      "gpu-oracle", [round(float(out.posterior[f][c] - op[f][c]), 4) for c in r[:4]])
