#!/usr/bin/env python3
"""configs[3] (ER mean degree 5, N=1e7, R=4096, 2 sweeps + fused count) on
the bench's own graph (bench.py bench_er: seed 0 + 31) in two node numberings:
the generator's, where the degree-class sweep writes and reads its own rows
through ``order`` (random 512-B rows), and the degree-sorted one (node k =
order[k]: an isomorphic graph whose class runs are contiguous, so writes and
own-row reads stream).  Checks the two rollouts are the same up to the
relabelling, then times both (and R = 8192 in the sorted numbering)."""
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
    n = 10_000_000
    g = mjx.erdos_renyi_device(n, 5.0 / (n - 1), seed=0 + 31)
    order = g.order.long()
    rank = torch.empty_like(order)
    rank[order] = torch.arange(n, device=order.device)
    deg = (g.row_ptr[1:] - g.row_ptr[:-1])[order]
    rp2 = torch.zeros(n + 1, dtype=torch.int64, device=order.device)
    rp2[1:] = torch.cumsum(deg, 0)
    # row k of the new graph = row order[k] of the old one, columns renamed by rank
    starts = g.row_ptr[:-1][order]
    idx = torch.repeat_interleave(starts - rp2[:-1], deg) + torch.arange(int(rp2[-1]), device=order.device)
    col2 = rank[g.col.long()[idx]].to(torch.int32)
    g2 = mjx.Graph.csr_device(rp2, col2)
    assert torch.equal(g2.order.long(), torch.arange(n, device=order.device))
    g.class_ell()
    g2.class_ell()
    print("sorted order is the identity; classes:", g2.class_ell()[2].shape[0], flush=True)
    for R in (4096, 8192):
        W = R // 64
        gen = torch.Generator(device="cuda").manual_seed(5)
        s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda", generator=gen)
        out, tmp = torch.empty_like(s0), torch.empty_like(s0)
        cnt = torch.zeros(R, dtype=torch.int64, device="cuda")
        graphs = [("sorted", g2)] if R > 4096 else [("generator", g), ("sorted", g2)]
        if R == 4096:
            # same dynamics up to the relabelling: rollout(g2, s0[order]) == rollout(g, s0)[order]
            a = mjx.rollout(g, s0, 2, words=W).view(n, W)
            b = mjx.rollout(g2, s0.view(n, W)[order].reshape(-1).contiguous(), 2, words=W).view(n, W)
            assert torch.equal(a[order], b), "relabelled rollout differs"
            del a, b
            print("relabelled rollout equal", flush=True)
        for name, gg in graphs:
            def step(c=True):
                cnt.zero_()
                mjx.rollout(gg, s0, 2, words=W, out=out, tmp=tmp, counts=cnt if c else None)
            step()
            for _ in range(3):
                a, b = timed(step), timed(lambda: step(False))
                print(f"R={R} {name:9s} numbering: 2 sweeps + count {a:.3f} ms, plain {b:.3f} ms "
                      f"({n * R * 2 / a / 1e9:.3f}e12 node-updates/s)", flush=True)
        del s0, out, tmp


if __name__ == "__main__":
    main()
