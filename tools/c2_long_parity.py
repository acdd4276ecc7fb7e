"""configs[1] at full size against the C oracle for longer than the test suite
(whose full-size test checks 20 oracle steps): d=3 RRG N=1e6, p=2, c=1, 4096
replicas in the default light-cone layout (speculative batches, MT19937 tape on
the side stream), C2_LONG_K steps (default 2000) in ragged traced calls; the
replicas in C2_LONG_SAMPLE (default 0, 1, 2047, 4095) run through the reference
loop's C restatement (oracle/orc_majority.c, ~0.1 s a step on one core) in
worker processes: every step's proposal, accept, sum(s_end), the final conf
and t must be equal.

    python tools/c2_long_parity.py        (GPU box)
"""
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N, D, P, C, R = 1_000_000, 3, 2, 1, 4096
K = int(os.environ.get("C2_LONG_K", 2000))
SAMPLE = [int(x) for x in os.environ.get("C2_LONG_SAMPLE", "0,1,2047,4095").split(",")]


def _oracle(args):
    adj, seed = args
    from oracle import fast
    t0 = time.perf_counter()
    o = fast.sa_loop(adj, P, C, seed, max_steps=K, trace=True)
    return o, time.perf_counter() - t0


def main():
    import mjx
    adj = mjx.random_regular_graph(D, N, seed=1007)
    seeds = np.arange(R, dtype=np.int64)
    pool = mp.get_context("spawn").Pool(len(SAMPLE))
    fut = pool.map_async(_oracle, [(adj, int(seeds[r])) for r in SAMPLE])
    import torch
    sa = mjx.SAReplicas(adj, P, C, seeds)
    got = {k: [] for k in ("i", "accept", "sum_end")}
    left, j, t0 = K, 0, time.perf_counter()
    while left > 0:
        c = min(left, [131, 700, 9, 1024, 1][j % 5])
        tr = sa.steps(c, trace=True)
        for key in got:
            got[key].append(tr[key][:, SAMPLE].cpu().numpy())
        left -= c
        j += 1
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    got = {k: np.concatenate(v) for k, v in got.items()}
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    print(f"layout {sa.layout}, {K} traced steps in {j} calls on {R} replicas: GPU {gpu_s:.1f} s", flush=True)
    w0 = time.perf_counter()
    while not fut.ready():                        # (a line a minute: the GPU box's hang detector)
        fut.wait(45)
        print(f"oracle running, {time.perf_counter() - w0:.0f} s", flush=True)
    res = fut.get()
    pool.close()
    ok = True
    for s_, r in enumerate(SAMPLE):
        o, cpu_s = res[s_]
        L = len(o["trace"]["i"])
        same_tr = all(np.array_equal(got[k][:L, s_], o["trace"][k]) for k in got)
        same = same_tr and o["num_steps"] == t[r] and np.array_equal(conf[r], o["conf"])
        ok &= bool(same)
        print(f"replica {r}: t {t[r]} (oracle {o['num_steps']}), trace equal {same_tr}, conf equal "
              f"{np.array_equal(conf[r], o['conf'])}, accepts {int(got['accept'][:L, s_].sum())}; "
              f"oracle {cpu_s:.0f} s on one core", flush=True)
    print("EQUAL" if ok else "DIFFERENT", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
