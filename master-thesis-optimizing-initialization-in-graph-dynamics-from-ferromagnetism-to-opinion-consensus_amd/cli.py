"""Script-shaped fronts: ``python -m mjx sa|hpr|bdcm`` run the reference's three
experiments with its module constants as flags -- same names, same defaults --
and write its np.savez keys.

  sa    code/SA_RRG.py:44-52 (n, d, p, c, par_a, par_b, N_stat), loop :58-88,
        output :92 ("MCMC_p{p}_d{d}.npz": mag_reached, num_steps, conf, graphs)
  hpr   code/HPR_pytorch_RRG.py:224-237 (n, d, p, c, damppar, attr_value,
        lmbd_in, pie, gamma, TT) and :251 (n_rep), output :377
        ("hpr_d{d}_p{p}.npz": mag_reached, conf, num_steps, graphs, time)
  bdcm  code/ER_BDCM_entropy.ipynb raw lines 456-481 (n, deg, num_rep, p, c,
        eps, damppar, attr_value, epsilon, T_max, a, dl), output :515
        ("ER_p{p}.npz": m_init, ent1, ent, ... T_max, num_rep)

Added beside the reference's constants: ``--seed`` (the reference seeds
nothing), ``--graph-seed``, ``--replicas`` (N_stat / n_rep / num_rep by
another name), ``--gpus`` (replicas spread over that many devices of this
node: independent SA streams, HPR replicas), ``--out``.  Graphs are this
package's own random regular / Erdos-Renyi generators (the reference uses
networkx with seed=None: the dynamics depend only on the edge set).
"""
import argparse
import sys
import time

import numpy as np

# the reference's module constants (name -> default), cited line by line
SA_DEFAULTS = {            # code/SA_RRG.py
    "n": 10000,            # :44
    "d": 4,                # :45
    "p": 3,                # :46
    "c": 1,                # :47
    "par_a": 1.0005,       # :49
    "par_b": 1.0005,       # :50
    "N_stat": 5,           # :52
}
HPR_DEFAULTS = {           # code/HPR_pytorch_RRG.py
    "n": 10000,            # :224
    "d": 4,                # :225
    "p": 1,                # :226
    "c": 1,                # :227
    "damppar": 0.4,        # :229
    "attr_value": 1,       # :230
    "lmbd_in": None,       # :231  (25*n)
    "pie": 0.3,            # :235
    "gamma": 0.1,          # :236
    "TT": 10000,           # :237
    "n_rep": 1,            # :251
}
BDCM_DEFAULTS = {          # code/ER_BDCM_entropy.ipynb (raw JSON lines)
    "n": 1000,             # nb:456
    "deg": [1.0, 1.5, 2.0],  # nb:459 np.linspace(1,2,3)
    "num_rep": 3,          # nb:463
    "p": 1,                # nb:466
    "c": 1,                # nb:467
    "eps": 1e-6,           # nb:470
    "damppar": 0.1,        # nb:471
    "attr_value": 1,       # nb:472
    "epsilon": 0.0,        # nb:473
    "T_max": 1300,         # nb:478
    "a": 12,               # nb:480
    "dl": 0.1,             # nb:481
}


def _common(ap):
    ap.add_argument("--seed", type=int, default=0, help="numpy / torch seed (the reference seeds nothing)")
    ap.add_argument("--graph-seed", type=int, default=None, help="seed of the first replica's graph (+k for replica k)")
    ap.add_argument("--replicas", type=int, default=None, help="replica count (overrides N_stat / n_rep / num_rep)")
    ap.add_argument("--gpus", type=int, default=1, help="devices of this node to spread the replicas over")
    ap.add_argument("--out", default=None, help="output .npz (default: the reference's file name)")


def build_parser():
    ap = argparse.ArgumentParser(prog="python -m mjx", description=__doc__.split("\n\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    sa = sub.add_parser("sa", help="code/SA_RRG.py")
    for k, v in SA_DEFAULTS.items():
        sa.add_argument(f"--{k}", type=type(v), default=v)
    sa.add_argument("--stream", choices=("global", "independent"), default="global",
                    help="global: ONE numpy stream, replicas back to back (the script's own semantics); "
                         "independent: replica k seeded seed+k, all at once")
    sa.add_argument("--max-steps", type=int, default=None, help="proposal cap per replica (the script's is 2n^3)")
    sa.add_argument("--max-seconds", type=float, default=None)
    _common(sa)
    hp = sub.add_parser("hpr", help="code/HPR_pytorch_RRG.py")
    for k, v in HPR_DEFAULTS.items():
        hp.add_argument(f"--{k}", type=(int if k == "lmbd_in" else type(v)), default=v)
    hp.add_argument("--dtype", choices=("float32", "float64"), default="float32",
                    help="message precision (the reference's is float64, :11)")
    _common(hp)
    bd = sub.add_parser("bdcm", help="code/ER_BDCM_entropy.ipynb")
    for k, v in BDCM_DEFAULTS.items():
        if k == "deg":
            bd.add_argument("--deg", type=float, nargs="+", default=list(v))
        else:        # a (the lambda range's end) may be given as a float too
            bd.add_argument(f"--{k}", type=float if k == "a" else type(v), default=v)
    _common(bd)
    return ap


def _devices(k):
    import torch
    have = torch.cuda.device_count()
    if k < 1 or k > max(have, 0):
        raise SystemExit(f"--gpus {k}: this node has {have} device(s)")
    return list(range(k))


def run_sa(a):
    import torch
    from .graph import random_regular_graph
    from .npz import save_sa_npz
    from .sa import SAReplicas, sa_run
    R = a.replicas if a.replicas is not None else a.N_stat
    gs = a.graph_seed if a.graph_seed is not None else a.seed
    if a.stream == "global" and a.gpus > 1:
        # one numpy stream seeded once (code/SA_RRG.py:58-88): replica k+1's draws
        # start where replica k's end, so the replicas cannot run side by side
        raise SystemExit(f"--gpus {a.gpus} with --stream global: the global stream is serial and runs on one "
                         "device; use --stream independent to spread replicas over devices")
    t0 = time.time()
    if a.stream == "global" or a.gpus == 1:
        res = sa_run(a.d, a.n, a.p, a.c, par_a=a.par_a, par_b=a.par_b, N_stat=R, seed=a.seed, graph_seed=gs,
                     stream=a.stream, max_steps=a.max_steps, max_seconds=a.max_seconds)
    else:
        # independent streams over several devices: one SAReplicas per device,
        # stepped round-robin (launches are asynchronous, so the devices overlap)
        devs = _devices(a.gpus)
        graphs = [random_regular_graph(a.d, a.n, seed=gs + k) for k in range(R)]
        parts = [list(range(R))[j::len(devs)] for j in range(len(devs))]
        runs = []
        for dev, idx in zip(devs, parts):
            if not idx:
                continue
            with torch.cuda.device(dev):
                runs.append((dev, idx, SAReplicas([graphs[k] for k in idx], a.p, a.c, [a.seed + k for k in idx],
                                                  par_a=a.par_a, par_b=a.par_b)))
        chunk, taken = 256, 0
        while True:
            live = [(dev, sa) for dev, _, sa in runs if not sa.all_done()]
            if not live or (a.max_steps is not None and taken >= a.max_steps) or \
                    (a.max_seconds is not None and time.time() - t0 >= a.max_seconds):
                break
            k = chunk if a.max_steps is None else min(chunk, a.max_steps - taken)
            for dev, sa in live:
                with torch.cuda.device(dev):
                    sa.steps(k)
            taken += k
            chunk = min(2 * chunk, 16384)
        res = {"mag_reached": np.zeros(R), "num_steps": np.zeros(R), "conf": np.zeros((R, a.n)),
               "done": np.zeros(R, dtype=np.int32)}
        for dev, idx, sa in runs:
            with torch.cuda.device(dev):
                out = sa.results()
            for j, k in enumerate(idx):
                for key in res:
                    res[key][k] = out[key][j]
        res["graphs"] = np.stack([g.astype(int) for g in graphs])
    out = a.out or f"MCMC_p{a.p}_d{a.d}.npz"
    save_sa_npz(out, res)
    print(f"sa: {R} replicas, num_steps {res['num_steps'].astype(np.int64).tolist()}, "
          f"mag_reached {np.round(res['mag_reached'], 4).tolist()}, {time.time() - t0:.1f} s -> {out}", flush=True)
    return res


def run_hpr(a):
    import torch
    from .graph import random_regular_edges
    from .hpr import hpr_run
    from .npz import save_hpr_npz
    R = a.replicas if a.replicas is not None else a.n_rep
    gs = a.graph_seed if a.graph_seed is not None else a.seed
    devs = _devices(a.gpus)
    dtype = torch.float32 if a.dtype == "float32" else torch.float64
    res = {"mag_reached": np.zeros(R), "num_steps": np.zeros(R), "conf": np.zeros((R, a.n)),
           "graphs": np.zeros((R, a.n, a.d))}
    t0 = time.time()
    for k in range(R):                      # HPR_pytorch_RRG.py:259, one graph per replica
        with torch.cuda.device(devs[k % len(devs)]):
            edges = random_regular_edges(a.d, a.n, seed=gs + k)
            r = hpr_run(a.d, a.n, a.p, a.c, damppar=a.damppar, attr_value=a.attr_value, lmbd_in=a.lmbd_in,
                        pie=a.pie, gamma=a.gamma, TT=a.TT, edges=edges, seed=a.seed + k, dtype=dtype)
        for key in res:
            res[key][k] = r[key][0]
    out = a.out or f"hpr_d{a.d}_p{a.p}.npz"
    save_hpr_npz(out, res, time=time.time() - t0)
    print(f"hpr: {R} replicas, num_steps {res['num_steps'].astype(np.int64).tolist()}, "
          f"mag_reached {np.round(res['mag_reached'], 4).tolist()}, {time.time() - t0:.1f} s -> {out}", flush=True)
    return res


def run_bdcm(a):
    from .bdcm import bdcm_er_run
    from .npz import save_bdcm_npz
    R = a.replicas if a.replicas is not None else a.num_rep
    _devices(a.gpus)                        # notebook-sized graphs: replicas run on the current device
    t0 = time.time()
    res = bdcm_er_run(n=a.n, deg=tuple(a.deg), num_rep=R, p=a.p, c=a.c, eps=a.eps, damppar=a.damppar,
                      attr_value=a.attr_value, epsilon=a.epsilon, T_max=a.T_max, a=a.a, dl=a.dl, seed=a.seed)
    out = a.out or f"ER_p{a.p}.npz"
    save_bdcm_npz(out, res)
    print(f"bdcm: deg {list(a.deg)} x {R} replicas, {time.time() - t0:.1f} s -> {out}", flush=True)
    return res


def main(argv=None):
    a = build_parser().parse_args(argv)
    return {"sa": run_sa, "hpr": run_hpr, "bdcm": run_bdcm}[a.cmd](a)


if __name__ == "__main__":
    main(sys.argv[1:])
