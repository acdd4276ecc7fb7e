"""configs[1] (d=3, N=1e6, p=2, c=1, R=4096) light-cone SA: the cost of the
proposal tape's chunking.  Times sa.steps(K) for each (rng, tape capacity,
K) in SA_CASES, in alternating repetitions on one box, so the MT19937 path
(tape drawn a chunk ahead on a side stream, chunks 128, 512, ..., tape/2)
can be set beside the Philox path (one tape of `tape` rows per launch) and
beside itself at other chunkings."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, p, c, R = 1_000_000, 3, 2, 1, 4096
adj = mjx.random_regular_graph(d, n, seed=7)
cases = [x.split(":") for x in os.environ.get(
    "SA_CASES", "mt19937:2048:2000,mt19937:8192:2000,philox:2048:2000,philox:512:2000").split(",")]
reps = int(os.environ.get("SA_REPS", "3"))
sas = {}
for case in cases:                     # rng:tape:K[:spec_k]
    rng, tape, K = case[:3]
    kern = {"spec_k": int(case[3])} if len(case) > 3 else None
    sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone", rng=rng, tape=int(tape), kernel=kern)
    sa.steps(10000)
    sas[tuple(case)] = sa
torch.cuda.synchronize()
res = {k: [] for k in sas}
for rep in range(reps):
    for key, sa in sas.items():
        K = int(key[2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sa.steps(K)
        torch.cuda.synchronize()
        res[key].append(1e6 * (time.perf_counter() - t0) / K)
        print(f"rep {rep} {':'.join(key)}: {res[key][-1]:.3f} us/step", flush=True)
for key, v in res.items():
    print(f"{':'.join(key):24s}: median {np.median(v):.3f} us/step "
          f"= {R / np.median(v) * 1e6:.3e} proposals/s", flush=True)
