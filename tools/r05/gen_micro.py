"""Trial generator kernel times (rocprofv3 --kernel-trace --stats over this
script): C2 / C4 shapes at several batch sizes, to separate per-wave latency
(batch 64: one wave per segment) from throughput (batch 4096)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import qkd_ldpc_v_amd as Q  # noqa: E402

for n, qber, batch in [(10240, 0.0215, 64), (10240, 0.0215, 512), (10240, 0.0215, 4096), (10240, 0.0005, 4096),
                       (102400, 0.038, 128), (102400, 0.038, 64)]:
    seeds = Q.trial_seeds(1022025, batch)
    d = torch.from_numpy(seeds.view(np.int64)).cuda()
    a = torch.empty((batch, n), dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    for _ in range(3):
        Q.trials_device(n, qber, d, a, b)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(5):
        Q.trials_device(n, qber, d, a, b)
    ev1.record()
    torch.cuda.synchronize()
    print(f"n={n} qber={qber} batch={batch}: {ev0.elapsed_time(ev1) / 5:.3f} ms per call", flush=True)
