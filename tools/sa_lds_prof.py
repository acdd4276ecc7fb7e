"""Phase timers of k_sa_lds_fast (diagnostic build with -DMJX_SA_PROF): per-wave
s_memtime cycles per phase, per step, at SA_RRG.py's shapes (d=4, n=1e4, 64
replicas on distinct graphs, p=c=1 and p=3, c=1)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

mjx.load_library()
raw = ctypes.CDLL(mjx.lib_path())
# phases of k_sa_lds_multi (p+c-1 = 1): refill, level 1 + conflicts, resolution, -, -, dE + accept, apply
names = ["refill+proposal", "level 1", "level 2 / resolve", "level 3", "level 4", "dE+exp+accept", "apply+trace",
         "pair code"]
n, d, R = 10_000, 4, 64
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
for (p, c, kern) in ((1, 1, None), (1, 1, {"lds_pair": True}), (3, 1, None), (3, 1, {"lds_single": True})):
    sa = mjx.SAReplicas(graphs, p, c, list(range(R)), layout="lds", kernel=kern)
    K = 20000
    sa.steps(K)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    raw.mjx_sa_lds_prof_read(buf, 1)
    t0 = time.perf_counter()
    sa.steps(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    raw.mjx_sa_lds_prof_read(buf, 1)
    print(f"p={p} c={c} {kern or 'pair'}: {1e6 * el / K:.3f} us/step; cycles per step per wave: "
          + ", ".join(f"{nm} {buf[q] / R / K:.0f}" for q, nm in enumerate(names))
          + f"; total {sum(buf[:7]) / R / K:.0f}; pairs tried {(buf[7] % 1000000) / 1000 / R / K:.3f}, "
          f"second taken {(buf[7] // 1000000) / R / K:.3f} per step", flush=True)
    del sa
