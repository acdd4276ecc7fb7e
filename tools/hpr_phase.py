#!/usr/bin/env python3
"""Per-phase cycle split of k_hpr_update at C3 (needs a libmjx.so built with
MJX_EXTRA_CFLAGS=-DMJX_HPR_PROF): staging / compute / epilogue, summed over
waves, as a fraction of the total."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mjx
from mjx import _lib

n, d, p, c = 100000, 4, 2, 2
lib = _lib.load()
edges = mjx.random_regular_edges(d, n, seed=3)
plan = mjx.HPRPlan(edges, n, d)
chi = torch.rand((2 * plan.E, 256), dtype=torch.float32, device="cuda")
chi /= chi.sum(1, keepdim=True)
b = torch.rand((n, 2), dtype=torch.float32, device="cuda")
b /= b.sum(1, keepdim=True)
out = torch.empty_like(chi)
buf = (ctypes.c_ulonglong * 32)()
for _ in range(3):
    mjx.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4, out=out)
torch.cuda.synchronize()
lib.mjx_hpr_prof_read(buf, 1)
K = 10
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    mjx.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4, out=out)
e1.record()
torch.cuda.synchronize()
lib.mjx_hpr_prof_read(buf, 0)
v = [buf[i] / K for i in range(4)]
tot = sum(v)
waves = (n + 15) // 16 * 4
print(f"HPr_dp {e0.elapsed_time(e1) / K:.3f} ms; per wave cycles: stage {v[0]/waves:.0f} compute {v[1]/waves:.0f} "
      f"row-sum sync {v[2]/waves:.0f} epilogue {v[3]/waves:.0f}; fractions " + " ".join(f"{x / tot:.2f}" for x in v), flush=True)
