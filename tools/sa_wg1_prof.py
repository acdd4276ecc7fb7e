"""Phase timers of the whole-CU LDS SA kernel at p+c-1 = 1 (k_sa_lds_wg1, configs[0]:
d=4, n=1e4, 64 replicas on distinct graphs), from a diagnostic build:
    python tools/ab_lib.py --build saprof -DMJX_SA_PROF mjx_sa_lds.hip      (CPU)
    python tools/ab_lib.py ab/libmjx_saprof.so tools/sa_wg1_prof.py         (GPU)
s_memtime cycles per round averaged over the 4 waves (wave 0's parse is in
its own slot: every other wave waits for it at the publish barrier)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mjx  # noqa: E402

lib = mjx._lib.load()
names = ["publish barrier", "tag barrier", "-", "tags set (+ parse, parser wave)", "level 1+dE+result",
         "result barrier", "resolve+apply"]
n, d, R, nw = 10_000, 4, 64, 5
graphs = [mjx.random_regular_graph(d, n, seed=7000 + k) for k in range(R)]
sa = mjx.SAReplicas(graphs, 1, 1, list(range(R)), layout="lds")
K = 40000
sa.steps(K)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 32)()
lib.mjx_sa_lds_prof_read(buf, 1)
t0 = time.perf_counter()
sa.steps(K)
torch.cuda.synchronize()
el = time.perf_counter() - t0
lib.mjx_sa_lds_prof_read(buf, 1)
wr = buf[7]
rounds = wr / nw / R
print(f"p=c=1 wg1: {1e6 * el / K:.3f} us/step, {K / rounds:.2f} proposals per round, {1e6 * el / rounds:.3f} us per "
      "round; cycles per round per wave: " + ", ".join(f"{nm} {buf[q] / wr:.0f}" for q, nm in enumerate(names))
      + f"; total {sum(buf[:7]) / wr:.0f}", flush=True)
