"""Light-cone SA throughput vs replica count at configs[1] (d=3, N=1e6,
p=2, c=1): tells a latency-bound step (proposals/s grow with R) from a
memory-transaction-bound one (proposals/s flat)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, p, c = 1_000_000, 3, 2, 1
adj = mjx.random_regular_graph(d, n, seed=7)
Rs = [int(x) for x in os.environ.get("SA_RS", "1024,4096,16384,65536").split(",")]
K = int(os.environ.get("SA_K", "1000"))
layouts = os.environ.get("SA_LAYOUTS", "cone,levels").split(",")
rng = os.environ.get("SA_RNG", "mt19937")              # "philox": the non-parity proposal stream
for R, lay in [(R, lay) for R in Rs for lay in layouts]:
    sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone", layout=lay, rng=rng)
    sa.steps(2000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sa.steps(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{lay}{'' if rng == 'mt19937' else ' ' + rng} R={R}: {1e6 * el / K:.2f} us/step, {R * K / el:.3e} proposals/s", flush=True)
    del sa
    torch.cuda.empty_cache()
