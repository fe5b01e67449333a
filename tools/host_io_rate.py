#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer entry (qldpc_decode_batch): C2 SPA
frames built on the host (f64 LLRs + syndromes), decoded through the C ABI
with host arrays in and out.  Prints one JSON line.  Not the bench value."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_v_amd as Q  # noqa: E402

H = Q.load_matrix(os.path.join(ROOT, "tests", "golden", "matrices", "c2_n10240_m2201.alist.gz"), 1)
batch = 4096
a, b, q = Q.bsc_frames(H.n, 0.0215, batch, seed=1)
lp = Q.log_p(q)
llr = np.ascontiguousarray(np.where(b != 0, -lp, lp))
s = H.syndrome(a)
g = Q.Graph(H)
p = Q.Params(Q.SPA, 50, True, 100.0)
g.decode(p, llr[:256], s[:256])  # warm
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    out = g.decode(p, llr, s)
dt = (time.perf_counter() - t0) / reps
print(json.dumps({"entry": "qldpc_decode_batch (host buffers)", "workload": "C2 SPA 50-iter, 4096 frames",
                  "seconds_per_batch": dt, "info_bits_per_s": batch * (H.n - H.m) / dt,
                  "h2d_bytes": llr.nbytes + s.nbytes, "d2h_bytes": out.bits.nbytes + 5 * batch,
                  "mean_iterations": float(out.iterations.mean())}))
