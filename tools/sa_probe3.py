"""Step time of the light-cone SA at SA_RRG.py's shapes (d=4, N=1e4, 64
replicas on distinct graphs): p=c=1 (configs[0]) and p=3, c=1 (the script),
LDS-resident replicas (every LDS kernel) vs the HBM cone layout.

    python tools/sa_probe3.py [--no-cone] [--R 64] [--n 10000]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
import mjx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--no-cone", action="store_true")
ap.add_argument("--R", type=int, default=64)
ap.add_argument("--n", type=int, default=10_000)
ap.add_argument("--pc", default="1,1;3,1")
args = ap.parse_args()
n, d, R = args.n, 4, args.R
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
VARIANTS = {
    # name: (layout, kernel options)
    "lds": ("lds", None),                                   # the default LDS kernel for (p, c)
    "lds-wg16": ("lds", {"split": 16}),                     # whole CU a proposal per wave, 16 waves (p+c-1 >= 2)
    "lds-wg8": ("lds", {"split": 8}),                       # the same, 8 waves
    "lds-wg4": ("lds", {"split": 4}),                       # whole CU, 4 waves (p+c-1 >= 2)
    "lds-cu": ("lds", {"lds_cu": True}),                    # whole CU, level-synchronous (d 3/4, T 2/3)
    "lds-cu16": ("lds", {"lds_cu": True, "split": 16}),     # the same with 16 waves
    "lds-wave": ("lds", {"lds_wave": True}),                # one wave: 8 proposals (T = 1) / 2 (T >= 2) per step
    "lds-pair": ("lds", {"lds_wave": True, "lds_pair": True}),   # one wave, two proposals per step
    "lds-single": ("lds", {"lds_single": True}),            # one wave, one proposal per step
    "cone": ("cone", None),
}
ap2 = os.environ.get("SA_VARIANTS")                      # e.g. "lds,lds-wg8": only these
if ap2:
    VARIANTS = {k: v for k, v in VARIANTS.items() if k in ap2.split(",")}
for pc in args.pc.split(";"):
    p, c = (int(x) for x in pc.split(","))
    for name, (layout, kern) in VARIANTS.items():
        if name == "cone" and args.no_cone:
            continue
        if name in ("lds-wg4", "lds-wg8", "lds-wg16", "lds-cu", "lds-cu16") and p + c - 1 < 2:
            continue
        K = 20000 if (layout == "lds" or p == 1) else 1000
        sa = mjx.SAReplicas(graphs, p, c, list(range(R)), layout=layout, kernel=kern)
        sa.steps(K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sa.steps(K)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"p={p} c={c} {name}: {1e6 * el / K:.3f} us/step, {R * K / el:.3g} proposals/s, "
              f"done {int((sa.done != 0).sum())}/{R}", flush=True)
