"""Probe: bsc frames, syndromes swapped between variants."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import qkd_ldpc_v_amd as Q
from conftest import load_fixture

H = load_fixture("c2_n10240_m2201.alist")
a, b, q = Q.bsc_frames(H.n, 0.0215, 8, seed=17)
lp = Q.log_p(q)
llr = np.where(b != 0, -lp, lp)
dev = torch.device("cuda:0")
g = Q.Graph(H)
for name, s in (("Hb", H.syndrome(b)), ("Ha", H.syndrome(a)), ("zero", np.zeros((8, H.m), np.uint8))):
    z = (llr <= 0).astype(np.uint8)
    exp = (H.syndrome(z) != s).sum(axis=1)
    for L in (llr, np.where(b != 0, -2.0, 2.0)):
        tl, ts = torch.from_numpy(L.copy()).to(dev), torch.from_numpy(s.copy()).to(dev)
        bits = torch.empty((8, H.n), dtype=torch.uint8, device=dev)
        it = torch.empty(8, dtype=torch.int32, device=dev)
        ok = torch.empty(8, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev)
        g.decode_device(Q.Params(3, 5, True, 100.0, 0.77), tl, ts, bits, it, ok, stream=st)
        torch.cuda.synchronize()
        o, wt = g.last_claim_order(st)
        print(name, "lp", L[0, 0], "gpu", wt[:5].tolist(), "expected", exp[:5].tolist(), flush=True)
