#!/usr/bin/env python3
"""Time the CSR replica-packed sweep at configs[3] (ER mean degree 5, N=1e7,
R=4096, 2 sweeps + count) and the RRG bench sweep, and check the CSR result
against the ELL-equivalent generic path on a small graph."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=10):
    import torch
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import torch
    import mjx
    n, R = 10_000_000, 4096
    W = R // 64
    rp, col = mjx.erdos_renyi(n, 5.0 / (n - 1), seed=3)
    g = mjx.Graph.csr(rp, col)
    gen = torch.Generator(device="cuda").manual_seed(0)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda", generator=gen)
    out, tmp = torch.empty_like(s0), torch.empty_like(s0)
    cnt = torch.zeros(R, dtype=torch.int64, device="cuda")
    B = 4 * int(rp[-1]) + 8 * (n + 1) + W * 8 * n * (rp[-1] / n + 2)

    def step():
        cnt.zero_()
        mjx.rollout(g, s0, 2, words=W, out=out, tmp=tmp, counts=cnt)

    step()
    for _ in range(3):
        ms = timed(step)
        print(f"ER N=1e7 R=4096: {ms:.3f} ms/step, {2 * B / (ms / 1e3) / 1e9:.0f} GB/s algorithmic, "
              f"{n * R * 2 / (ms / 1e3):.3e} node-updates/s", flush=True)


if __name__ == "__main__":
    main()
