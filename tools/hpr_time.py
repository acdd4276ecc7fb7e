#!/usr/bin/env python3
"""Quick timing of the HPR kernels at config 3 (d=4, N=1e5, p=2, c=2)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mjx

n, d, p, c = int(os.environ.get("N", 100000)), 4, 2, 2
for dtype in ((torch.float32,) if os.environ.get("ONLY_F32") else (torch.float32, torch.float64)):
    edges = mjx.random_regular_edges(d, n, seed=3)
    plan = mjx.HPRPlan(edges, n, d)
    nc = 4 ** (p + c)
    chi = torch.rand((2 * plan.E, nc), dtype=dtype, device="cuda")
    chi /= chi.sum(1, keepdim=True)
    b = torch.rand((n, 2), dtype=dtype, device="cuda")
    b /= b.sum(1, keepdim=True)
    out = torch.empty_like(chi)
    for _ in range(3):
        mjx.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K = 20
    e0.record()
    for _ in range(K):
        mjx.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    byts = 3 * 2 * plan.E * nc * chi.element_size()
    print(f"{dtype}: HPr_dp {ms:.3f} ms  {2*plan.E/ms*1e3:.3e} msgs/s  {byts/ms/1e6:.0f} GB/s algorithmic", flush=True)
    z = torch.empty(4 * plan.E, dtype=dtype, device="cuda")
    mg = torch.empty((n, 2), dtype=dtype, device="cuda")
    e0.record()
    for _ in range(K):
        mjx.marginals_comp(out, plan, p, c, zwork=z, out=mg)
    e1.record()
    torch.cuda.synchronize()
    print(f"{dtype}: marginals {e0.elapsed_time(e1)/K:.3f} ms", flush=True)
