#!/usr/bin/env python3
"""Timing of the decay-split (q layout) HPR update and marginals at configs[2]
(d=4, N=1e5, p=c=2, fp32) -- the kernels of hpr_run's loop -- by HIP events
over K launches (the bench's hpr.loop_state_q measurement, standalone)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402
from mjx import _lib as L, _device as D  # noqa: E402

n, d, p, c = int(os.environ.get("N", 100000)), 4, 2, 2
K = int(os.environ.get("K", 50))
plan = mjx.HPRPlan(mjx.random_regular_edges(d, n, seed=3), n, d)
nc = 4 ** (p + c)
g = torch.Generator(device="cuda").manual_seed(0)
chi = torch.rand((2 * plan.E, nc), dtype=torch.float32, device="cuda", generator=g)
chi /= chi.sum(1, keepdim=True)
b = torch.rand((n, 2), dtype=torch.float32, device="cuda", generator=g)
b /= b.sum(1, keepdim=True)
st = mjx.HPRState(plan, p, c, chi, b, dtype=torch.float32, layout="q")
code, sptr, sz = L.MJX_F32, st._sc.data_ptr(), st._sc.element_size()
lmbd = 25 * n
wp, wm = math.exp(-lmbd / n), math.exp(lmbd / n)
bufs = (st.chi, st.chi_b)
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]


def run():
    s_ = D.stream_handle()
    e[0].record()
    for k in range(K):
        L.call("mjx_hpr_update_q", code, bufs[k % 2].data_ptr(), bufs[1 - k % 2].data_ptr(), st.biases.data_ptr(),
               plan.nbr.data_ptr(), plan.in_row.data_ptr(), plan.out_row.data_ptr(), n, d, p, c, 1, wp, wm, 0.4,
               sptr, s_)
    e[1].record()
    for k in range(K):
        L.call("mjx_hpr_marginals_q", code, bufs[k % 2].data_ptr(), plan.out_row.data_ptr(), n, d, p, c, 1e-15,
               sptr + sz, st._ii.data_ptr(), st.zwork.data_ptr(), st.marg.data_ptr(), s_)
    e[2].record()


for rep in range(3):
    run()
    torch.cuda.synchronize()
    print(f"q layout: update {e[0].elapsed_time(e[1]) / K:.4f} ms, marginals {e[1].elapsed_time(e[2]) / K:.4f} ms",
          flush=True)
