#!/usr/bin/env python3
"""RRG d=4 replica-packed sweep at growing N (R=4096): does throughput fall
with the state size (TLB reach / cache) like the N=1e7 ER case?  Also times
SA init (s0 draws) at configs[1]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import mjx
    R, W = 4096, 64
    for n in (1_000_000, 4_000_000, 10_000_000):
        g = mjx.random_regular_graph_device(4, n, seed=1)
        s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda")
        out, tmp = torch.empty_like(s0), torch.empty_like(s0)
        mjx.rollout(g, s0, 2, words=W, out=out, tmp=tmp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            mjx.rollout(g, s0, 2, words=W, out=out, tmp=tmp)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        B = 4 * 4 * n + 512 * n * 6
        print(f"RRG d=4 N={n:.0e} R=4096: {ms:.3f} ms/step  {2 * B / (ms / 1e3) / 1e9:.0f} GB/s", flush=True)
        del g, s0, out, tmp
        torch.cuda.empty_cache()
    adj = mjx.random_regular_graph(3, 1_000_000, seed=7)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sa = mjx.SAReplicas(adj, 2, 1, np.arange(4096))
        torch.cuda.synchronize()
        print(f"SA init (N=1e6, R=4096, d=3, p=2, c=1): {time.perf_counter() - t0:.4f} s", flush=True)
        del sa


if __name__ == "__main__":
    main()
