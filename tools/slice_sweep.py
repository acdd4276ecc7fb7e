#!/usr/bin/env python3
"""A/B of replica slicing for the replica-packed rollout (bench workload:
d=4 RRG, N=1e6, R=4096, 2 sweeps + fused count), interleaved rounds in one
process (cdna_hip_programming.md 5.4 rule 24); checks every variant's output
against slices=1."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mjx
    n, d, R, T = 1_000_000, 4, 4096, 2
    W = R // 64
    g = mjx.Graph.ell(mjx.random_regular_graph(d, n, seed=0))
    gen = torch.Generator(device="cuda").manual_seed(0)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda", generator=gen)
    out, tmp = torch.empty_like(s0), torch.empty_like(s0)
    cnt = torch.zeros(R, dtype=torch.int64, device="cuda")
    variants = [1, 2, 4, 8, 16]
    ref = mjx.rollout(g, s0, T, words=W, slices=1).clone()
    rc = torch.zeros(R, dtype=torch.int64, device="cuda")
    mjx.rollout(g, s0, T, words=W, counts=rc, slices=1)
    times = {S: [] for S in variants}
    for S in variants:
        cnt.zero_()
        o = mjx.rollout(g, s0, T, words=W, out=out, tmp=tmp, counts=cnt, slices=S)
        assert torch.equal(o, ref) and torch.equal(cnt, rc), S
    for rnd in range(5):
        for S in variants:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                cnt.zero_()
                mjx.rollout(g, s0, T, words=W, out=out, tmp=tmp, counts=cnt, slices=S)
            e1.record()
            torch.cuda.synchronize()
            times[S].append(e0.elapsed_time(e1) / 10)
    B = 4 * d * n + (R // 8) * n * (d + 2)
    for S in variants:
        t = sorted(times[S])
        print(f"slices={S:2d}  ms/step median {t[len(t)//2]:.4f} min {t[0]:.4f}  "
              f"algorithmic GB/s {B * T / (t[len(t)//2] / 1e3) / 1e9:.0f}", flush=True)


if __name__ == "__main__":
    main()
