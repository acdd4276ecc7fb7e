#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes (one counter group per pass).

Runs, on cuda:0, exactly the bench.py sweep (d=4 RRG, N=1e6, R=4096
replica-packed, 2 sweeps per rollout, fused count on the last one) a few
times, preceded by a calibration copy of a known byte count (torch's
vectorised copy, 16 B per lane) that tools/pmc_parse.py uses to check the
gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md, HBM section).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--replicas", type=int, default=4096)
    ap.add_argument("--T", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--calib-mb", type=int, default=1024)
    args = ap.parse_args()
    import torch
    import mjx
    n, d, R = args.n, args.d, args.replicas
    W = (R + 63) // 64
    adj = mjx.random_regular_graph(d, n, seed=0)
    dev = torch.device("cuda", 0)
    # calibration: a copy of calib-mb MiB (read + write), well past the 256 MiB Infinity Cache
    nb = args.calib_mb << 20
    a = torch.ones(nb // 8, dtype=torch.int64, device=dev)
    b = torch.empty_like(a)
    torch.cuda.synchronize()
    b.copy_(a)
    torch.cuda.synchronize()
    del a, b
    g = mjx.Graph.ell(adj)
    gen = torch.Generator(device=dev).manual_seed(0)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device=dev, generator=gen)
    out = torch.empty_like(s0)
    tmp = torch.empty_like(s0)
    counts = torch.zeros(W * 64, dtype=torch.int64, device=dev)
    for _ in range(args.reps):
        counts.zero_()
        mjx.rollout(g, s0, args.T, words=W, out=out, tmp=tmp, counts=counts)
    torch.cuda.synchronize()
    print(f"pmc_run done: n={n} d={d} R={R} T={args.T} reps={args.reps} calib={nb} B", flush=True)


if __name__ == "__main__":
    main()
