"""Probe: claim-order weights vs batch size."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import qkd_ldpc_v_amd as Q
from conftest import load_fixture

H = load_fixture("c2_n10240_m2201.alist")
a, b, q = Q.bsc_frames(H.n, 0.0215, 300, seed=17)
lp = Q.log_p(q)
llr = np.where(b != 0, -lp, lp)
s = H.syndrome(a)
exp = (H.syndrome((llr <= 0).astype(np.uint8)) != s).sum(axis=1)
dev = torch.device("cuda:0")
for fresh in (False, True):
    g = Q.Graph(H)
    for batch in ((8, 16, 32, 48, 64, 128, 300) if not fresh else (300, 8)):
        tl, ts = torch.from_numpy(llr[:batch].copy()).to(dev), torch.from_numpy(s[:batch].copy()).to(dev)
        bits = torch.empty((batch, H.n), dtype=torch.uint8, device=dev)
        it = torch.empty(batch, dtype=torch.int32, device=dev)
        ok = torch.empty(batch, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev)
        g.decode_device(Q.Params(3, 5, True, 100.0, 0.77), tl, ts, bits, it, ok, stream=st)
        torch.cuda.synchronize()
        o, wt = g.last_claim_order(st)
        bad = np.nonzero(wt != exp[:batch])[0]
        print("fresh", fresh, "batch", batch, "bad", bad.size, bad[:8].tolist(), "gpu", wt[:3].tolist(),
              "exp", exp[:3].tolist(), flush=True)
