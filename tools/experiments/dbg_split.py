"""Debug: C4 split decode posterior vs oracle (which bits differ)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_v_amd as Q
from oracle.pyoracle import Oracle
H = Q.load_matrix(os.path.join(ROOT, "tests/golden/matrices/c4s_n102400_m32001.alist.gz"), 1)
a, b, q = Q.bsc_frames(H.n, 0.03, 2, seed=90)
sign = np.where(b != 0, -1.0, 1.0)
g = Q.Graph(H)
print("plan", g.plan(0, Q.SPA), os.environ.get("QLDPC_AB_BUILD"))
O = Oracle(H)
s = H.syndrome(a)
for L, it in ((3.5, 1), (3.5, 1), (3.5, 2), (3.5, 5)):
    llr = sign * L
    out = g.decode(Q.Params(Q.SPA, it, True, 100.0), llr, s, posterior=True)
    ob, oi, ok, op = O.decode_batch(O.params(Q.SPA, it, True, 100.0), llr, s, threads=8, posterior=True)
    for f in range(2):
        d = np.nonzero(out.posterior[f] != op[f])[0]
        print("L", L, "it", it, "f", f, "iters", out.iterations[f], oi[f], "bitdiff", int((out.bits[f] != ob[f]).sum()),
              "postdiff", len(d), "gpu", out.posterior[f][:4], "ora", op[f][:4])
