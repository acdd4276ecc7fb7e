"""Phase timers of the level-synchronous whole-CU LDS SA kernel k_sa_lds_cu (a
diagnostic build:
    python tools/ab_lib.py --build saprof -DMJX_SA_PROF mjx_sa_lds.hip      (CPU)
    python tools/ab_lib.py ab/libmjx_saprof.so tools/sa_cu_prof.py          (GPU)
): s_memtime cycles per round, averaged over the item waves of every
replica but wave 0, wave 0's own and the parse wave's (SA_CU_WAVES=16: the 16-wave form), at SA_RRG.py's
shapes (d=4, n=1e4, 64 replicas on distinct graphs); every stamp drains the
wave's counters, so a phase's exposed latency is charged to it."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

lib = mjx._lib.load()
names = ["publish barrier", "level work", "level barriers", "accept test", "(unused)", "resolve+apply"]
n, d, R = 10_000, 4, 64
KERN = {"lds_cu": True, **({"split": 16} if os.environ.get("SA_CU_WAVES") == "16" else {})}
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
for (p, c) in ((3, 1), (2, 1), (2, 2)):
    sa = mjx.SAReplicas(graphs, p, c, list(range(R)), layout="lds", kernel=dict(KERN))
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
    wr = buf[6]                                 # rounds x item waves (wave 0 excluded), all replicas
    r0 = buf[16 + 6]                            # rounds, all replicas (wave 0)
    print(f"p={p} c={c}: {1e6 * el / K:.3f} us/step, {buf[16 + 7] / r0:.2f} proposals per round "
          f"({K * R / r0:.2f} by the clock), {1e6 * el * R / r0:.3f} us per round; "
          f"|C_1|,|C_2|,|C_3| per round {buf[16 + 8] / r0:.1f}, {buf[16 + 9] / r0:.1f}, {buf[16 + 10] / r0:.1f}",
          flush=True)
    print("  cycles per round, other waves: " + ", ".join(f"{nm} {buf[q] / wr:.0f}" for q, nm in enumerate(names))
          + f"; total {sum(buf[:6]) / wr:.0f}", flush=True)
    print("  cycles per round, wave 0:      " + ", ".join(f"{nm} {buf[16 + q] / r0:.0f}" for q, nm in enumerate(names))
          + f"; total {sum(buf[16:22]) / r0:.0f}", flush=True)
    print("  cycles per round, parse wave:  " + ", ".join(f"{nm} {buf[11 + q] / r0:.0f}" for q, nm in
                                                        enumerate(["publish barrier", "level work", "level barriers",
                                                                   "accept test", "resolve+apply"])), flush=True)
    del sa
