#!/usr/bin/env python3
"""Per-sweep timing of the replica-packed dynamics kernels at the bench sizes:
d=4 RRG N=1e6 (configs[1]) and ER mean degree 5 N=1e7 (configs[3]), R=4096,
one sweep with and without the fused per-replica count.  HIP events on the
stream the kernels run on; algorithmic bytes as in DESIGN.md section 3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=20):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def probe(name, g, n, nnz, extra_bytes, W, dev):
    import torch
    import mjx
    gen = torch.Generator(device=dev).manual_seed(0)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device=dev, generator=gen)
    out = torch.empty_like(s0)
    cnt = torch.zeros(W * 64, dtype=torch.int64, device=dev)
    B = 4 * nnz + extra_bytes + 8 * W * (nnz + 2 * n)
    for label, c in (("plain", None), ("count", cnt)):
        ms = timed(lambda: mjx.rollout(g, s0, 1, words=W, out=out, counts=c))
        print(f"{name} {label}: {ms * 1e3:8.1f} us/sweep  {B / (ms / 1e3) / 1e9:7.0f} GB/s algorithmic  "
              f"{n * W * 64 / (ms / 1e3):.3e} node-updates/s", flush=True)
    del s0, out


def main():
    import torch
    import mjx
    dev = torch.device("cuda", 0)
    W = 64
    adj = mjx.random_regular_graph(4, 1_000_000, seed=0)
    probe("RRG d=4 N=1e6", mjx.Graph.ell(adj), 1_000_000, 4_000_000, 0, W, dev)
    n = 10_000_000
    g = mjx.erdos_renyi_device(n, 5.0 / (n - 1), seed=31)
    nnz = int(g.col.numel())
    g.class_ell()
    torch.cuda.synchronize()
    for layout in ("class", "csr"):
        g.rp_layout = layout
        probe(f"ER deg5 N=1e7 [{layout}]", g, g.n, nnz, 8 * (g.n + 1), W, dev)


if __name__ == "__main__":
    main()
