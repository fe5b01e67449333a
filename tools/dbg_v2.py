"""Debug helper (GPU box): where does the V2 decoder first differ from the oracle?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import qkd_ldpc_v_amd as Q  # noqa: E402
from conftest import load_fixture  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

for name, q in (("c2_n10240_m2201.alist", 0.026), ("c3_n10240_m1801.alist", 0.02), ("c1_n1024_m220.alist", 0.03)):
    H = load_fixture(name)
    g = Q.Graph(H)
    print(name, g.plan(0, 0), flush=True)
    a, b, qq = Q.bsc_frames(H.n, q, 4, seed=5)
    lp = Q.log_p(qq)
    llr = np.where(b != 0, -lp, lp)
    s = H.syndrome(a)
    O = Oracle(H)
    for alg, prim, sec in ((0, 0, 0), (3, 0.77, 0), (5, 0.55, 1.2)):
        for mi in (1, 2, 3, 50):
            out = g.decode(Q.Params(alg, mi, True, 100.0, prim, sec), llr, s, posterior=True)
            ob, oi, ok, op = O.decode_batch(O.params(alg, mi, True, 100.0, prim, sec), llr, s, threads=4,
                                            posterior=True)
            d = out.posterior != op
            print(f"  alg {alg} max_it {mi}: post diffs {int(d.sum())} bits diffs {int((out.bits != ob).sum())} "
                  f"it {out.iterations.tolist()} vs {oi.tolist()}", flush=True)
            if d.any():
                f, i = np.argwhere(d)[0]
                rows = np.where(H.col_idx == i)[0]
                print("    first diff frame", f, "bit", i, out.posterior[f, i], op[f, i], "edges", rows[:6])
