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
# SA_SPLITS: waves per word column of the speculative kernel (0 = the library's choice; 16 = half-filled waves at K = 8)
splits = [int(x) for x in os.environ.get("SA_SPLITS", "0").split(",")]
for R, lay, sp in [(R, lay, sp) for R in Rs for lay in layouts for sp in splits]:
    sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone", layout=lay, rng=rng,
                        kernel={"split": sp} if sp else None)
    sa.steps(2000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sa.steps(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{lay}{'' if rng == 'mt19937' else ' ' + rng}{f' split={sp}' if sp else ''} R={R}: {1e6 * el / K:.2f} us/step, "
          f"{R * K / el:.3e} proposals/s", flush=True)
    del sa
    torch.cuda.empty_cache()
