"""Probe: claim-order weights on crafted frames (expected: 0, 0, |Hb|, |s|)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import qkd_ldpc_v_amd as Q
from conftest import load_fixture

H = load_fixture(sys.argv[1] if len(sys.argv) > 1 else "c2_n10240_m2201.alist")
rng = np.random.default_rng(1)
b = rng.integers(0, 2, (4, H.n)).astype(np.uint8)
llr = np.where(b != 0, -2.0, 2.0)
llr[1] = 2.0
s = H.syndrome(b)
s[1] = 0
s[2] = 0
llr[3] = 3.0
exp = (H.syndrome((llr <= 0).astype(np.uint8)) != s).sum(axis=1)
dev = torch.device("cuda:0")
g = Q.Graph(H)
for batch in (4, 2):
    tl, ts = torch.from_numpy(llr[:batch].copy()).to(dev), torch.from_numpy(s[:batch].copy()).to(dev)
    bits = torch.empty((batch, H.n), dtype=torch.uint8, device=dev)
    it = torch.empty(batch, dtype=torch.int32, device=dev)
    ok = torch.empty(batch, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    g.decode_device(Q.Params(int(os.environ.get("ALG", "3")), 5, True, 100.0, 0.77), tl, ts, bits, it, ok, stream=st)
    torch.cuda.synchronize()
    o, wt = g.last_claim_order(st)
    print("batch", batch, "gpu", wt.tolist(), "expected", exp[:batch].tolist(), "|s|", s.sum(1)[:batch].tolist(),
          "|Hz|", H.syndrome((llr <= 0).astype(np.uint8)).sum(1)[:batch].tolist(), flush=True)
