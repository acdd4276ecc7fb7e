"""Phase timers of the whole-CU LDS SA kernel k_sa_lds_wg (a diagnostic build:
    python tools/ab_lib.py --build saprof -DMJX_SA_PROF mjx_sa_lds.hip      (CPU)
    python tools/ab_lib.py ab/libmjx_saprof.so tools/sa_wg_prof.py          (GPU)
): s_memtime cycles per round, averaged over the waves of every replica, at
SA_RRG.py's p=3, c=1 (d=4, n=1e4, 64 replicas on distinct graphs); every stamp
drains the wave's counters, so a phase's exposed latency is charged to it."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

lib = mjx._lib.load()
names = ["B0 (publish barrier)", "level 1", "level 2", "level 3", "dE+accept", "mark check+result+barrier",
         "resolve+apply"]
n, d, R = 10_000, 4, 64
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
for (p, c, kern, nw) in ((3, 1, None, 16), (3, 1, {"split": 8}, 8), (2, 1, None, 16)):
    sa = mjx.SAReplicas(graphs, p, c, list(range(R)), layout="lds", kernel=kern)
    K = 20000
    sa.steps(K)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    lib.mjx_sa_lds_prof_read(buf, 1)
    t0 = time.perf_counter()
    sa.steps(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    lib.mjx_sa_lds_prof_read(buf, 1)
    wave_rounds = buf[7]                       # rounds x waves, over all replicas
    rounds = wave_rounds / nw / R              # rounds per replica
    print(f"p={p} c={c} {kern or 'wg16'}: {1e6 * el / K:.3f} us/step, {K / rounds:.2f} proposals per round, "
          f"{1e6 * el / rounds:.3f} us per round; cycles per round per wave: "
          + ", ".join(f"{nm} {buf[q] / wave_rounds:.0f}" for q, nm in enumerate(names))
          + f"; total {sum(buf[:7]) / wave_rounds:.0f}; barrier-1 wait {buf[10] / wave_rounds:.0f}; "
          f"parse wave parsing {buf[9] / (wave_rounds / nw):.0f}", flush=True)
    print("  levels + test by wave: " + " ".join(f"{buf[16 + q] / (wave_rounds / nw):.0f}" for q in range(nw - 1)),
          flush=True)
    del sa
