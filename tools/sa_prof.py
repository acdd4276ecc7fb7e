"""Phase timers of k_sa_spec (diagnostic build with -DMJX_SA_PROF): per-wave
s_memtime cycles per phase, summed over waves, for configs[1] (d=3, N=1e6,
p=2, c=1) at several replica counts."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

raw = mjx._lib.load()                      # (the variant under tools/ab_lib.py)
names = ["tape+rows(i,A0)+tree", "rows(C)+sectors+lvl1", "gc words+lvl2", "hash lookups", "resolve+flips+drain",
         "hash clear", "hash inserts", "fence"]
n, d, p, c = 1_000_000, 3, 2, 1
adj = mjx.random_regular_graph(d, n, seed=7)
for R in [int(x) for x in os.environ.get("SA_RS", "4096,16384").split(",")]:
    for kern in ({}, {"spec_half": True}) if os.environ.get("HALF") else ({},):
        sa = mjx.SAReplicas(adj, p, c, np.arange(R), kernel=kern)
        sa.steps(2000)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 8)()
        raw.mjx_sa_prof_read(buf, 1)
        K = 1000
        t0 = time.perf_counter()
        sa.steps(K)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        raw.mjx_sa_prof_read(buf, 1)
        tot = sum(buf[:8])
        waves = (R // 64) * 8 * (2 if kern else 1)
        batches = K / 8
        print(f"R={R} {kern} layout={sa.layout}: {1e6 * el / K:.2f} us/step; per wave per batch (cycles): "
              + ", ".join(f"{nm} {buf[q] / waves / batches:.0f}" for q, nm in enumerate(names))
              + f"; total {tot / waves / batches:.0f}", flush=True)
        del sa
