"""Step time of the light-cone SA at SA_RRG.py's shapes (d=4, N=1e4, 64
replicas on distinct graphs): p=c=1 (configs[0]) and p=3, c=1 (the script),
LDS-resident replicas vs the HBM cone layout."""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
import mjx  # noqa: E402

n, d, R = 10_000, 4, 64
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
for (p, c) in ((1, 1), (3, 1)):
    for layout in ("lds", "lds-pair", "lds-single", "cone"):
        K = 20000 if (layout.startswith("lds") or p == 1) else 1000
        kern = {"lds-single": {"lds_single": True}, "lds-pair": {"lds_pair": True}}.get(layout)
        sa = mjx.SAReplicas(graphs, p, c, list(range(R)), layout=layout.split("-")[0], kernel=kern)
        sa.steps(K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sa.steps(K)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"p={p} c={c} {layout}: {1e6 * el / K:.3f} us/step, {R * K / el:.3g} proposals/s, "
              f"done {int((sa.done != 0).sum())}/{R}", flush=True)
