"""Light-cone SA step latency probe: ms per step for several (p, c) and
replica counts on a d=3 RRG with N=1e6 (configs[1] sizes)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

n, d = 1_000_000, 3
adj = mjx.random_regular_graph(d, n, seed=7)
for (p, c) in ((1, 1), (2, 1), (3, 1)):
    for R in (64, 4096):
        sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone")
        sa.steps(5)
        torch.cuda.synchronize()
        K = 1000
        t0 = time.perf_counter()
        sa.steps(K)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"p={p} c={c} R={R}: {1e3 * el / K * 1e3:.1f} us/step", flush=True)
        del sa
