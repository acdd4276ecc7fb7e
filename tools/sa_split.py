"""Light-cone SA step time vs waves per word column (kernel option ``split``) at
configs[1], cone layout, one-trip step (no speculative batches)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, p, c, R = 1_000_000, 3, 2, 1, 4096
adj = mjx.random_regular_graph(d, n, seed=7)
ref = None
for sp in (1, 2, 4, 8, 16):
    sa = mjx.SAReplicas(adj, p, c, np.arange(R), mode="lightcone", layout="cone",
                        kernel={"split": sp, "no_spec": True})
    tr = sa.steps(200, trace=True)
    acc = tr["accept"].cpu().numpy()
    if ref is None:
        ref = acc
    assert np.array_equal(acc, ref), f"split {sp} differs"
    torch.cuda.synchronize()
    K = 1000
    t0 = time.perf_counter()
    sa.steps(K)
    torch.cuda.synchronize()
    print(f"split={sp}: {1e6 * (time.perf_counter() - t0) / K:.1f} us/step", flush=True)
    del sa
