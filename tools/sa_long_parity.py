"""Long-run parity of the default LDS SA kernel at SA_RRG.py's own shape (d=4,
n=1e4, p=3, c=1; k_sa_lds_cu): SA_LONG_K steps (default 60000, dozens of MT19937
twists, thousands of accepted flips) in ragged calls on SA_LONG_R replicas
(default 2), each on its own graph, against the C restatement of the
reference's loop (oracle/orc_majority.c) run in worker processes: conf, t and
the MT19937 stream must be equal.  A one-off check beyond the test suite's
3033 steps (the oracle needs ~1.4 ms a step on one core).

    python tools/sa_long_parity.py        (GPU box; SA_LONG_PC="p,c", SA_LONG_K, SA_LONG_R)
"""
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

D, N = 4, 10_000
P, C = (int(x) for x in os.environ.get("SA_LONG_PC", "3,1").split(","))   # e.g. "1,1": configs[0]'s kernel
K = int(os.environ.get("SA_LONG_K", 60000))
R = int(os.environ.get("SA_LONG_R", 2))


def _oracle(args):
    g, seed = args
    from oracle import fast
    st = np.random.RandomState(seed).get_state()
    t0 = time.perf_counter()
    o = fast.sa_loop(g, P, C, seed, max_steps=K, mt_state=(st[1], st[2]))
    return o, time.perf_counter() - t0


def main():
    import mjx
    graphs = [mjx.random_regular_graph(D, N, seed=4242 + k) for k in range(R)]
    seeds = [9000 + k for k in range(R)]
    pool = mp.get_context("spawn").Pool(R)
    fut = pool.map_async(_oracle, list(zip(graphs, seeds)))
    import torch
    sa = mjx.SAReplicas(graphs, P, C, seeds, layout="lds")
    chunks, left, k = [], K, 0
    while left > 0:
        c = min(left, [977, 4096, 13, 20011, 1][k % 5])
        chunks.append(c)
        left -= c
        k += 1
    t0 = time.perf_counter()
    for c in chunks:
        sa.steps(c)
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    mt, idx = sa.mt_state()
    w0 = time.perf_counter()
    while not fut.ready():                        # (a line a minute: the GPU box's hang detector)
        fut.wait(45)
        print(f"oracle running, {time.perf_counter() - w0:.0f} s", flush=True)
    res = fut.get()
    pool.close()
    ok = True
    for r in range(R):
        o, cpu_s = res[r]
        same = (o["num_steps"] == t[r] and np.array_equal(conf[r], o["conf"]) and
                np.array_equal(mt[r], o["mt_state"][0]) and idx[r] == o["mt_state"][1])
        ok &= bool(same)
        print(f"replica {r}: t {t[r]} (oracle {o['num_steps']}), conf equal {np.array_equal(conf[r], o['conf'])}, "
              f"MT19937 state equal {np.array_equal(mt[r], o['mt_state'][0]) and idx[r] == o['mt_state'][1]}, "
              f"m(s) {conf[r].mean():+.4f}; oracle {cpu_s:.1f} s on one core", flush=True)
    print(f"p={P} c={C}: {K} steps in {len(chunks)} calls, {R} replicas: GPU {gpu_s:.2f} s; {'EQUAL' if ok else 'DIFFERENT'}",
          flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
