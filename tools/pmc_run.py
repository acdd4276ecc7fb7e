#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc passes (one counter group per pass).

Runs, on cuda:0, exactly the bench.py sweep (d=4 RRG, N=1e6, R=4096
replica-packed, 2 sweeps per rollout, fused count on the last one) a few
times, then (unless --no-hpr) the C3 HPR iteration (d=4 RRG, N=1e5,
p=c=2, fp32: HPr_dp + marginals_comp, in the reference layout and in the
loop state's decay-split layout), (unless --no-sa) 1000 light-cone SA steps
at configs[1] (the speculative batches), (unless --no-er) the configs[3]
ER degree-class sweeps (N=1e7, 4096 replicas), and (unless --no-giant) a few sweeps
of the C5 partitioned N=1e9 d=6 graph on one rank, preceded by a calibration copy of a known byte count (torch's
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
    ap.add_argument("--no-hpr", action="store_true")
    ap.add_argument("--no-giant", action="store_true")
    ap.add_argument("--giant-n", type=int, default=1_000_000_000)
    ap.add_argument("--no-sa", action="store_true")
    ap.add_argument("--sa-steps", type=int, default=1000)
    ap.add_argument("--no-er", action="store_true")
    ap.add_argument("--er-n", type=int, default=10_000_000)
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
    del s0, out, tmp, g
    if not args.no_hpr:
        hn, hd, p, c = 100_000, 4, 2, 2
        plan = mjx.HPRPlan(mjx.random_regular_edges(hd, hn, seed=3), hn, hd)
        nc = 4 ** (p + c)
        chi = torch.rand((2 * plan.E, nc), dtype=torch.float32, device=dev, generator=gen)
        chi /= chi.sum(1, keepdim=True)
        b = torch.rand((hn, 2), dtype=torch.float32, device=dev, generator=gen)
        b /= b.sum(1, keepdim=True)
        hout = torch.empty_like(chi)
        z = torch.empty(4 * plan.E, dtype=torch.float32, device=dev)
        mg = torch.empty((hn, 2), dtype=torch.float32, device=dev)
        for _ in range(args.reps):
            mjx.HPr_dp(chi, b, plan, p, c, 1, 25 * hn, 0.4, out=hout)
            mjx.marginals_comp(hout, plan, p, c, zwork=z, out=mg)
        # the loop state's decay-split layout (HPRState layout="q")
        st = mjx.HPRState(plan, p, c, chi, b, dtype=torch.float32, layout="q")
        for k in range(args.reps):
            st.step(u=torch.rand(hn, dtype=torch.float64, generator=torch.Generator().manual_seed(k)))
        torch.cuda.synchronize()
        del chi, hout, plan, st
        print("pmc_run hpr done", flush=True)
    if not args.no_sa:
        # configs[1] light-cone SA (d=3, N=1e6, p=2, c=1, 4096 replicas): the
        # speculative batches on the cone layout; one launch per 1024-step tape chunk
        import numpy as np
        sa = mjx.SAReplicas(mjx.random_regular_graph(3, 1_000_000, seed=7), 2, 1, np.arange(4096), mode="lightcone")
        sa.steps(args.sa_steps)
        torch.cuda.synchronize()
        del sa
        # the LDS-resident whole-CU kernels at SA_RRG.py's shapes (d=4, n=1e4, 64
        # replicas on their own graphs): p=c=1 (configs[0], k_sa_lds_wg1) and the
        # script's p=3, c=1 (k_sa_lds_wg), and the one-wave pair kernel beside them
        gl = [mjx.random_regular_graph(4, 10_000, seed=7000 + k) for k in range(64)]
        for (p_, c_, kern) in ((1, 1, None), (3, 1, None), (3, 1, {"lds_wave": True})):
            sa = mjx.SAReplicas(gl, p_, c_, np.arange(64), layout="lds", kernel=kern)
            sa.steps(20 * args.sa_steps)
            torch.cuda.synchronize()
            del sa
        print("pmc_run sa done", flush=True)
    if not args.no_er:
        # configs[3]: ER mean degree 5, N=1e7, 4096 replicas: the degree-class
        # sweeps of bench.py's er leg (2 sweeps + fused count per step)
        ge = mjx.erdos_renyi_device(args.er_n, 5.0 / (args.er_n - 1), seed=31)
        ge.class_ell()
        es = torch.randint(-2 ** 62, 2 ** 62, (args.er_n * W,), dtype=torch.int64, device=dev, generator=gen)
        eo, et = torch.empty_like(es), torch.empty_like(es)
        for _ in range(args.reps):
            counts.zero_()
            mjx.rollout(ge, es, args.T, words=W, out=eo, tmp=et, counts=counts)
        torch.cuda.synchronize()
        del ge, es, eo, et
        print("pmc_run er done", flush=True)
    if not args.no_giant:
        sh = mjx.ShardedRRG(6, args.giant_n, seed=12345, mode="binned")
        sh.drop_adjacency()
        sh.buf[sh.cur].copy_(torch.randint(-2 ** 62, 2 ** 62, sh.buf[sh.cur].shape, dtype=torch.int64,
                                           device=dev, generator=gen))
        for _ in range(args.reps):
            sh.sweep()
        torch.cuda.synchronize()
        print("pmc_run giant done", flush=True)
    print(f"pmc_run done: n={n} d={d} R={R} T={args.T} reps={args.reps} calib={nb} B", flush=True)


if __name__ == "__main__":
    main()
