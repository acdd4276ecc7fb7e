"""SA_RRG.py literally, at the script's own size (code/SA_RRG.py:44-92: n = 1e4,
d = 4, p = 3, c = 1, N_stat = 5): the replicas back to back on ONE numpy stream
seeded once, a fresh random 4-regular graph each, every replica run until
m(s_endstate(s)) = 1 (or the t > 2n^3 cap; --max-s bounds this call's wall time) -- what
mjx.sa_run(..., stream="global") does, stepped here with a progress line every
--every seconds.  Writes the script's np.savez keys (mag_reached, num_steps,
conf, graphs) to gpurun_out/MCMC_p3_d4.npz.  The replica running when
the call's wall cap is reached is checkpointed (SAReplicas.save_checkpoint: its configuration, the
stream, a, b, t) with the results so far to gpurun_out/sa_script_ckpt.npz;
--resume FILE continues the run from such a file (copied into the tree: the
GPU box sees only the tree), bit for bit as if it had never stopped.

    python tools/sa_script_run.py [--n 10000] [--nstat 5] [--seed 0] [--max-s 170] [--resume FILE]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mjx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000)
ap.add_argument("--nstat", type=int, default=5)
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--graph-seed", type=int, default=100)
ap.add_argument("--max-s", type=float, default=170.0, help="wall cap of this call (all replicas)")
ap.add_argument("--every", type=float, default=20.0)
ap.add_argument("--resume", default=None)
args = ap.parse_args()
d, p, c, n = 4, 3, 1, args.n
graphs = [mjx.random_regular_graph(d, n, seed=args.graph_seed + k) for k in range(args.nstat)]
res = {"mag_reached": np.zeros(args.nstat), "num_steps": np.zeros(args.nstat), "conf": np.zeros((args.nstat, n)),
       "wall_s": np.zeros(args.nstat)}
state, k0, ck = None, 0, None
if args.resume:
    with np.load(args.resume, allow_pickle=False) as z:
        z = {key: z[key] for key in z.files}
    k0 = int(z["replica"])
    for key in res:
        res[key] = z["res_" + key]
    ck = {key[3:]: z[key] for key in z if key.startswith("ck_")}
    print(f"resuming replica {k0} at t = {int(ck['t'][0])}", flush=True)
t_all = time.perf_counter()
for k, g in enumerate(graphs):
    if k < k0:
        continue
    if ck is not None and k == k0:
        sa = mjx.SAReplicas.resume(g, ck, layout="lds")
    else:
        sa = mjx.SAReplicas(g, p, c, [args.seed], tape=0, mt_state=state, layout="lds")
    torch.cuda.synchronize()
    steps0 = int(sa.t.item())            # > 0 for a resumed replica
    t0 = last = time.perf_counter()
    chunk = 1 << 16
    while not sa.all_done() and time.perf_counter() - t_all < args.max_s:
        sa.steps(chunk)
        chunk = min(2 * chunk, 1 << 22)
        if time.perf_counter() - last > args.every:
            last = time.perf_counter()
            print(f"  replica {k}: t = {int(sa.t.item())} after {last - t0:.0f} s", flush=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = sa.results()
    res["mag_reached"][k], res["num_steps"][k], res["conf"][k] = out["mag_reached"][0], out["num_steps"][0], out["conf"][0]
    res["wall_s"][k] += wall
    done = int(out["done"][0])
    print(f"replica {k}: done={done} num_steps={int(out['num_steps'][0])} mag_reached={out['mag_reached'][0]:.4f} "
          f"wall {wall:.1f} s ({1e6 * wall / max(out['num_steps'][0] - steps0, 1):.3f} us per proposal in this call)", flush=True)
    state = sa.mt_state()
    if done == 0:
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez("gpurun_out/sa_script_ckpt.npz", replica=np.array(k),
                 **{"res_" + key: v for key, v in res.items()},
                 **{"ck_" + key: v for key, v in sa.checkpoint().items()})
        print(f"stopped by the wall cap: replica {k} checkpointed to gpurun_out/sa_script_ckpt.npz "
              "(--resume continues it)", flush=True)
        break
    del sa
print(f"this call {time.perf_counter() - t_all:.1f} s; per replica wall s {np.round(res['wall_s'], 1).tolist()}, "
      f"num_steps {res['num_steps'].astype(np.int64).tolist()}, mag_reached {np.round(res['mag_reached'], 4).tolist()}",
      flush=True)
os.makedirs("gpurun_out", exist_ok=True)
res["graphs"] = np.stack([g.astype(int) for g in graphs])
mjx.save_sa_npz("gpurun_out/MCMC_p3_d4.npz", res)
