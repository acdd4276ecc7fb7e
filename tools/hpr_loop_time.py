"""hpr_run's loop iteration at configs[2] (d=4, N=1e5, p=c=2, fp32, decay-split
layout) in hipGraph-replayed batches of 16, the device-continued CPU stream
beside it (the bench's hpr.loop_state_q.loop_ms_per_iter), with the node step
fused (mjx_hpr_node_step) and as three launches, alternating on one box."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, p, c = 100_000, 4, 2, 2
plan = mjx.HPRPlan(mjx.random_regular_edges(d, n, seed=3), n, d)
g = torch.Generator().manual_seed(0)
chi = torch.rand((2 * plan.E, 4 ** (p + c)), dtype=torch.float64, generator=g)
chi /= chi.sum(1, keepdim=True)
b = torch.rand((n, 2), dtype=torch.float64, generator=g)
b /= b.sum(1, keepdim=True)
for rep in range(3):
    for fuse in (True, False):
        st = mjx.HPRState(plan, p, c, chi, b, dtype=torch.float32, layout="q")
        st.fuse_node = fuse
        gcpu = torch.Generator().manual_seed(1)
        st.steps_batched(16, gcpu)
        st.steps_batched(16, gcpu)
        st.rng_attach(gcpu)
        drawn = st.draw_batch_device(16)
        nb = 20
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nb):
            st.launch_batch(drawn)
            drawn = st.draw_batch_device(16, st.t)
            st.collect_batch()
        torch.cuda.synchronize()
        print(f"fused node step {fuse}: {1e3 * (time.perf_counter() - t0) / (16 * nb):.4f} ms per iteration",
              flush=True)
        del st
