#!/usr/bin/env python3
"""Time the degree-class replica-packed rollout at configs[3] (ER mean degree 5,
N=1e7, R=4096, 2 sweeps) with and without the fused per-replica count, after
checking the count against a torch popcount of the output."""
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
    g = mjx.erdos_renyi_device(n, 5.0 / (n - 1), seed=0 + 31)   # bench.py bench_er: seed (0) + 31 on rank 0
    g.class_ell()                    # the bench's degree-class layout (configs[3])
    gen = torch.Generator(device="cuda").manual_seed(0)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda", generator=gen)
    out, tmp = torch.empty_like(s0), torch.empty_like(s0)
    cnt = torch.zeros(R, dtype=torch.int64, device="cuda")

    def step(c):
        cnt.zero_()
        mjx.rollout(g, s0, 2, words=W, out=out, tmp=tmp, counts=cnt if c else None)

    step(True)
    ref = cnt.clone()
    ones = torch.stack([((out.view(n, W) >> b) & 1).sum(0) for b in range(64)], 1).reshape(-1)
    assert torch.equal(ones, ref), "fused count differs from a torch popcount of the output"
    for _ in range(3):
        a, b = timed(lambda: step(True)), timed(lambda: step(False))
        print(f"ER N=1e7 R=4096 class-ELL, 2 sweeps: {a:.3f} ms with the fused count, {b:.3f} ms without "
              f"(+{100 * (a / b - 1):.1f} %)", flush=True)


if __name__ == "__main__":
    main()
