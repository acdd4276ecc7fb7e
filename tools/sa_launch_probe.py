"""configs[1] (d=3, N=1e6, p=2, c=1, R=4096) light-cone SA: the fixed cost
of one sa.steps(K) call.  One instance per rng; calls of K in SA_KS taken in
rotating order for SA_REPS cycles; the per-call time against K is fitted by
least squares (fixed cost + K * per-step cost)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, p, c, R = 1_000_000, 3, 2, 1, 4096
adj = mjx.random_regular_graph(d, n, seed=7)
Ks = [int(x) for x in os.environ.get("SA_KS", "250,500,1000,2000,4000").split(",")]
reps = int(os.environ.get("SA_REPS", "3"))
tape = int(os.environ.get("SA_TAPE", "8192"))
for rng in os.environ.get("SA_RNGS", "philox,mt19937").split(","):
    sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone", rng=rng, tape=tape)
    sa.steps(10000)
    torch.cuda.synchronize()
    xs, ys = [], []
    for rep in range(reps):
        for j in range(len(Ks)):
            K = Ks[(j + rep) % len(Ks)]
            t0 = time.perf_counter()
            sa.steps(K)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            xs.append(K)
            ys.append(1e6 * el)
            print(f"{rng} rep {rep} K={K}: {1e6 * el:.0f} us = {1e6 * el / K:.3f} us/step", flush=True)
    A = np.stack([np.ones(len(xs)), np.array(xs, dtype=float)], axis=1)
    (fix, slope), *_ = np.linalg.lstsq(A, np.array(ys), rcond=None)
    print(f"{rng} tape={tape}: fixed {fix:.0f} us per call + {slope:.3f} us per step", flush=True)
    del sa
    torch.cuda.empty_cache()
