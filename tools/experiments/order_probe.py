"""Probe: claim-order weights vs the host's |H z xor s| with relabelling on/off."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import qkd_ldpc_v_amd as Q
from conftest import load_fixture

name = sys.argv[1] if len(sys.argv) > 1 else "c2_n10240_m2201.alist"
H = load_fixture(name)
a, b, q = Q.bsc_frames(H.n, 0.0215, 64, seed=17)
lp = Q.log_p(q)
llr = np.where(b != 0, -lp, lp).astype(np.float64)
s = H.syndrome(a)
w = (H.syndrome((llr <= 0).astype(np.uint8)) != s).sum(axis=1)
dev = torch.device("cuda:0")
for rl in ("1", "0"):
    os.environ["QLDPC_RELABEL"] = rl
    g = Q.Graph(H)
    for soft in (False, True):
        L = llr * (1.0 + 0.01 * np.arange(H.n)) if soft else llr
        tl, ts = torch.from_numpy(L).to(dev), torch.from_numpy(s).to(dev)
        bits = torch.empty((64, H.n), dtype=torch.uint8, device=dev)
        it = torch.empty(64, dtype=torch.int32, device=dev)
        ok = torch.empty(64, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev)
        g.decode_device(Q.Params(int(os.environ.get("ALG", "0")), 50, True, 100.0, 0.77), tl, ts, bits, it, ok, stream=st)
        torch.cuda.synchronize()
        o, wt = g.last_claim_order(st)
        print(f"relabel={rl} soft={soft} gpu {wt[:6].tolist()} host {w[:6].tolist()} equal={np.array_equal(wt, w)}",
              flush=True)
