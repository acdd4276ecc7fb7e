#!/usr/bin/env python3
"""Per-phase cycle split of the decay-split pipelined update k_hpr_update_q2
at configs[2] (d=4, N=1e5, p=c=2, fp32), on a variant built with
-DMJX_HPR_PROF (tools/ab_lib.py --build hprprof -DMJX_HPR_PROF mjx_hpr_f32.hip):
per wave and tile, s_memtime cycles of the DMA/index issue, the DP, the
vmcnt wait for the next tile's rows, the two barriers and the epilogue; the DP
per wave index (x_a) shows the imbalance the first barrier absorbs."""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402
from mjx import _lib as L, _device as D  # noqa: E402

n, d, p, c = 100000, 4, 2, 2
K = 20
lib = L.load()
plan = mjx.HPRPlan(mjx.random_regular_edges(d, n, seed=3), n, d)
nc = 4 ** (p + c)
g = torch.Generator(device="cuda").manual_seed(0)
chi = torch.rand((2 * plan.E, nc), dtype=torch.float32, device="cuda", generator=g)
chi /= chi.sum(1, keepdim=True)
b = torch.rand((n, 2), dtype=torch.float32, device="cuda", generator=g)
b /= b.sum(1, keepdim=True)
st = mjx.HPRState(plan, p, c, chi, b, dtype=torch.float32, layout="q")
code, sptr = L.MJX_F32, st._sc.data_ptr()
wp, wm = math.exp(-25.0), math.exp(25.0)
bufs = (st.chi, st.chi_b)


def run(k):
    for j in range(k):
        L.call("mjx_hpr_update_q", code, bufs[j % 2].data_ptr(), bufs[1 - j % 2].data_ptr(), st.biases.data_ptr(),
               plan.nbr.data_ptr(), plan.in_row.data_ptr(), plan.out_row.data_ptr(), n, d, p, c, 1, wp, wm, 0.4,
               sptr, D.stream_handle())


buf = (ctypes.c_ulonglong * 32)()
run(3)
torch.cuda.synchronize()
lib.mjx_hpr_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.mjx_hpr_prof_read(ctypes.cast(buf, ctypes.c_void_p), 1)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run(K)
e1.record()
torch.cuda.synchronize()
lib.mjx_hpr_prof_read(ctypes.cast(buf, ctypes.c_void_p), 0)
ntiles = (n + 15) // 16
waves = ntiles * 8                                  # wave-tiles per launch
names = ["issue", "DP", "vmcnt wait", "barrier 1", "epilogue", "barrier 2"]
v = [buf[4 + k] / K / waves for k in range(6)]
tot = sum(v)
print(f"k_hpr_update_q2 {e0.elapsed_time(e1) / K:.4f} ms per launch (profiling build); cycles per wave and tile: "
      + ", ".join(f"{nm} {x:.0f} ({x / tot:.2f})" for nm, x in zip(names, v)) + f"; total {tot:.0f}", flush=True)
per = [buf[10 + w] / K / ntiles for w in range(8)]
print("DP cycles per tile by wave (x_a index): " + " ".join(f"{x:.0f}" for x in per), flush=True)
