#!/usr/bin/env python3
"""Benchmark: majority-rule rollout throughput on MI355X (BASELINE.json metric).

Workload (one "step"): s_endstate + m for a batch of replicas — p+c-1 = 2
synchronous majority sweeps of R = 4096 bit-packed replicas on a d=4 random
regular graph with N = 1e6 nodes (configs[1]'s sizes, d=4 as the metric
names), with the per-replica +1 count fused into the last sweep.  Every step
starts from the same resident synthetic s0 (one SA-style scoring pass).
Inputs are resident in HBM before the timed region.

Multi-GPU (torch.distributed.run, one rank per GPU): each rank owns its own
graph instance and replicas (weak scaling, no data-path collective); the
timed region is bracketed by barrier + synchronize and the max over ranks is
reported.

Secondary line items in the same JSON object:
  * roofline of the dominant kernel (k_sweep_ell_rp) from HIP events,
  * cpu_baseline: the numpy restatement of the reference's onestep_majority
    (oracle/majority.py, same numpy ops as code/SA_RRG.py:18-20) on the same
    graph, one process per core, bounded sample, rank 0 at N=1 only,
  * sa: SA proposals/s and sweeps/s on configs[1] (d=3, N=1e6, p=2, c=1,
    4096 replicas; light-cone and full-rollout modes), timed after a warm-in
    of --sa-warmin proposals per replica,
  * sa_c1: configs[0] literally (SA_RRG.py's case: d=4, N=1e4, p=c=1, 64
    replicas) beside the numpy restatement of the reference's SA loop,
  * hpr / bdcm / er / giant legs, the HPR
    leg with the torch-CPU restatement on all host cores beside it.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--replicas", type=int, default=4096)
    ap.add_argument("--p", type=int, default=2)
    ap.add_argument("--c", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sa-steps", type=int, default=2000)
    ap.add_argument("--sa-rollout-steps", type=int, default=10)
    ap.add_argument("--sa-warmin", type=int, default=10000,
                    help="proposals every SA replica makes before the timed region (steady state, not t=0)")
    ap.add_argument("--c1-steps", type=int, default=10000)
    ap.add_argument("--c1-cpu-seconds", type=float, default=12.0)
    ap.add_argument("--consensus-replicas", type=int, default=64)
    ap.add_argument("--consensus-n", type=int, default=1000)
    ap.add_argument("--consensus-max-s", type=float, default=60.0,
                    help="wall-time cap of the run-to-consensus leg (reported, not hidden, if hit)")
    ap.add_argument("--consensus-script-s", type=float, default=20.0,
                    help="wall budget of the n=1e4 (SA_RRG.py's own size) leg")
    ap.add_argument("--no-consensus", action="store_true")
    ap.add_argument("--global-n", type=int, default=1000,
                    help="n of the sa_global leg (SA_RRG.py's own run: N_stat replicas back to back on one stream)")
    ap.add_argument("--global-nstat", type=int, default=5)
    ap.add_argument("--global-max-s", type=float, default=30.0, help="wall cap per replica of the sa_global leg")
    ap.add_argument("--no-global", action="store_true")
    ap.add_argument("--no-sa", action="store_true")
    ap.add_argument("--giant-n", type=int, default=1_000_000_000)
    ap.add_argument("--giant-d", type=int, default=6)
    ap.add_argument("--giant-sweeps", type=int, default=100,
                    help="timed sweeps of the C5 leg (SURVEY.md 8(d): 100 sweeps)")
    ap.add_argument("--giant-mode", default="binned", choices=["binned", "gather"])
    ap.add_argument("--giant-pieces", type=int, default=None,
                    help="node ranges per rank (exchange of piece g overlaps the sweep of g+1); "
                         "default 1 on one GPU, 2 otherwise")
    ap.add_argument("--no-giant", action="store_true")
    ap.add_argument("--er-n", type=int, default=10_000_000)
    ap.add_argument("--er-deg", type=float, default=5.0)
    ap.add_argument("--er-replicas", type=int, default=4096)
    ap.add_argument("--er-steps", type=int, default=5)
    ap.add_argument("--no-er", action="store_true")
    ap.add_argument("--hpr-n", type=int, default=100_000)
    ap.add_argument("--hpr-iters", type=int, default=10)
    ap.add_argument("--no-hpr", action="store_true")
    ap.add_argument("--bdcm-iters", type=int, default=100)
    ap.add_argument("--no-bdcm", action="store_true")
    ap.add_argument("--detail-out", default=None,
                    help="file for the full JSON object (every leg with its notes and per-replica arrays); the "
                         "printed line keeps each leg's numbers and ends with a compact `summary` (default "
                         "gpurun_out/bench_detail.json)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: the ranks join a gloo group, time an empty step and "
                         "rank 0 prints the merged JSON line (tests/test_bench_launch.py)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# Launcher: --gpus N > 1 without a torch.distributed.run environment
# ---------------------------------------------------------------------------
def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """Start one fresh rank process per GPU (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, rendezvous on 127.0.0.1) and wait for them.  This process
    never touches the GPU (device_count() does not initialise it) and never
    re-execs; it exits with the first failing rank's status, stopping the
    others, and fails when fewer than N devices are visible."""
    import subprocess
    n = args.gpus
    if not args.dry_run:
        import torch
        avail = torch.cuda.device_count()
        if avail < n:
            print(f"bench.py: --gpus {n} but only {avail} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with status {code}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def dry_run(args, rank, world):
    """The launch path without a GPU: gloo group, an empty timed step between
    barriers, max over ranks, one merged JSON line from rank 0."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    pids = [os.getpid()]
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        pids = [None] * world
        dist.all_gather_object(pids, os.getpid())
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "none", "n_gpus": world, "ranks": world,
                          "rank_pids": pids, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * el,
                          "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# CPU baseline (runs BEFORE the GPU is touched: forked workers, no exec)
# ---------------------------------------------------------------------------
def cpu_share():
    """Host cores this process may use: the CPUs in its affinity mask, capped by
    the cgroup CPU quota (cpu.max) when one is set -- the GPU box lists 256 CPUs
    in the mask but grants a 16-CPU share (cpu.max 1600000 100000)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(avail, quota) if quota else avail), avail, quota


def host_info():
    """CPU model, os.cpu_count(), the CPU share and library versions."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores, affinity, quota = cpu_share()
    info = {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "cpu_share": cores, "numpy": np.__version__}
    try:
        import torch
        info["torch"] = torch.__version__
    except ImportError:
        pass
    return info


def _cpu_worker(args):
    adj, steps_per_rollout, seconds, seed = args
    from oracle import majority as orc
    rng = np.random.default_rng(seed)
    n = adj.shape[0]
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        s = 2 * rng.integers(0, 2, n).astype(np.int64) - 1
        orc.s_endstate(adj, s, steps_per_rollout, 1)
        done += 1
    return done, time.perf_counter() - t0


def _single_thread_numpy():
    for k in ("OMP_NUM_THREADS", "MKL_NUM_THREADS", "OPENBLAS_NUM_THREADS"):
        os.environ[k] = "1"


def cpu_baseline(adj, T, seconds):
    """One process per core of the CPU share (cpu_share()), numpy single-threaded."""
    import multiprocessing as mp
    cores = cpu_share()[0]
    _single_thread_numpy()
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(adj, T, seconds, 1000 + i) for i in range(cores)])
    wall = time.perf_counter() - t0
    rollouts = sum(r[0] for r in res)
    n = adj.shape[0]
    value = rollouts * n * T / max(r[1] for r in res)
    return {
        "value": value, "unit": "node-updates/s", "cores": cores, "kind": "port", "host": host_info(),
        "sample": (f"oracle/majority.py s_endstate (numpy, same ops as code/SA_RRG.py:18-26) on the bench graph "
                   f"(d={adj.shape[1]}, N={n}), {T} sweeps per rollout, one replica per rollout, "
                   f"{rollouts} rollouts in ~{seconds:.0f}s per process x {cores} processes "
                   f"(wall {wall:.1f}s)"),
    }


# ---------------------------------------------------------------------------
def _timed(fn, dist, dev):
    """Run fn between barrier+synchronize brackets; max wall time over ranks."""
    import torch
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    return el


def bench_sa(args, rank, world, dist, dev):
    """configs[1]: SA on a d=3 RRG, N=1e6, p=2, c=1, 4096 bit-packed replicas per
    GPU (code/SA_RRG.py:63-88, bit-exact replay of numpy's seeded stream).
    Light-cone mode (default) and the full-rollout mode are both timed."""
    import torch
    import mjx
    sa_n, sa_d, sa_p, sa_c, sa_R = 1_000_000, 3, 2, 1, 4096
    sa_adj = mjx.random_regular_graph(sa_d, sa_n, seed=args.seed + 7 + 1000 * rank)
    seeds = np.arange(sa_R, dtype=np.int64) + rank * sa_R
    out = {"config": "configs[1]: d=3 RRG N=1e6 p=2 c=1, 4096 bit-packed SA replicas per GPU "
                     "(numpy MT19937 replay, bit-exact accept sequences)"}
    # "lightcone_philox": the same run on the non-parity Philox-4x32-10 proposal
    # stream (SAReplicas(rng="philox")) -- not the reference's
    # proposals; the parity line is "lightcone"
    for key, steps in (("lightcone", args.sa_steps), ("lightcone_philox", args.sa_steps),
                       ("rollout", args.sa_rollout_steps)):
        if steps <= 0:
            continue
        mode = "rollout" if key == "rollout" else "lightcone"
        torch.cuda.synchronize()
        t_init = time.perf_counter()
        sa = mjx.SAReplicas(sa_adj, sa_p, sa_c, seeds, mode=mode,
                            rng="philox" if key == "lightcone_philox" else "mt19937")
        sa.steps(2)
        torch.cuda.synchronize()
        t_init = time.perf_counter() - t_init
        sa.steps(args.sa_warmin)                      # steady state: past the all-accept start
        el = _timed(lambda: sa.steps(steps), dist, dev)
        props = world * sa_R * steps / el
        out[key] = {
            "proposals_per_s": props,
            "sweeps_per_s": props / sa_n,
            "ms_per_step": 1e3 * el / steps,
            "reference_equivalent_node_updates_per_s": props * 3 * (sa_p + sa_c - 1) * sa_n,
            "init_s": t_init,
            "warmin_proposals_per_replica": args.sa_warmin,
            "steps": steps,
        }
        del sa
    return out


def _sa_cpu_worker(args):
    """numpy restatement of the reference's SA loop (three rollouts per
    proposal, code/SA_RRG.py:63-88) on the replicas given, ~seconds in all:
    a short calibration run, then an equal proposal budget per replica."""
    graphs, p, c, seeds, seconds = args
    from oracle import majority as orc
    t0 = time.perf_counter()
    done = orc.sa_loop(graphs[0], p, c, seeds[0], max_steps=50)["num_steps"]
    per = (time.perf_counter() - t0) / max(1, done)
    budget = max(50, int((seconds - (time.perf_counter() - t0)) / per / len(graphs)))
    for g, sd in zip(graphs, seeds):
        done += orc.sa_loop(g, p, c, sd, max_steps=budget)["num_steps"]
    return done, time.perf_counter() - t0


def sa_cpu_baseline(graphs, p, c, seeds, seconds):
    """configs[0]'s CPU reference: the replicas spread over one process per
    core of the CPU share, each running the numpy SA loop."""
    import multiprocessing as mp
    cores = min(cpu_share()[0], len(seeds))
    _single_thread_numpy()
    parts = [([], []) for _ in range(cores)]
    for k, (g, sd) in enumerate(zip(graphs, seeds)):
        parts[k % cores][0].append(g)
        parts[k % cores][1].append(sd)
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(_sa_cpu_worker, [(gs, p, c, sds, seconds) for gs, sds in parts])
    props = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"proposals_per_s": props / wall, "cores": cores, "kind": "port", "host": host_info(),
            "sample": f"oracle/majority.py sa_loop (numpy, code/SA_RRG.py:63-88, three rollouts per proposal), "
                      f"{len(seeds)} replicas each on its own graph spread over {cores} processes, {props} "
                      f"proposals in {wall:.1f} s"}


def bench_sa_c1(args, rank, world, dist, dev, c1_cpu=None):
    """configs[0] literally: SA_RRG.py's own case, d=4 RRG, N=1e4, p=c=1, 64
    replicas, each on its OWN graph as the script draws them
    (code/SA_RRG.py:58-62), all 64 run together (graphs stacked in HBM),
    light-cone SA after a warm-in; the same replicas on one shared graph
    beside it; the numpy restatement of the reference's SA loop on the host
    cores (measured before the GPU was touched) as the CPU baseline."""
    import torch
    import mjx
    n, d, p, c, R = 10_000, 4, 1, 1, 64
    graphs = c1_graphs(args, rank)
    seeds = list(range(rank * R, (rank + 1) * R))
    K = args.c1_steps
    res = {"config": "configs[0]: SA_RRG.py case, d=4 RRG N=1e4, p=c=1, 64 replicas per GPU (numpy seeds), each on "
                     f"its own graph (code/SA_RRG.py:58-62), {K} proposals per replica after {args.sa_warmin} "
                     "warm-in proposals"}
    for tag, src in (("distinct_graphs", graphs), ("shared_graph", graphs[0])):
        sa = mjx.SAReplicas(src, p, c, seeds)
        sa.steps(args.sa_warmin)
        el = _timed(lambda: sa.steps(K), dist, dev)
        props = world * R * K / el
        res[tag] = {"mode": sa.mode, "layout": sa.layout, "proposals_per_s": props, "sweeps_per_s": props / n,
                    "ms_per_step": 1e3 * el / K}
        del sa
    res["proposals_per_s"] = res["distinct_graphs"]["proposals_per_s"]
    if c1_cpu is not None:
        res["cpu_baseline"] = c1_cpu
        res["speedup_vs_cpu"] = res["proposals_per_s"] / c1_cpu["proposals_per_s"]
    return res


def c1_graphs(args, rank):
    import mjx
    return [mjx.random_regular_graph(4, 10_000, seed=args.seed + 1000 + 64 * rank + k) for k in range(64)]


def _sa_until_done(mjx, graphs, p, c, seeds, cap_s):
    """Step every replica until m(s_endstate(s)) = 1 or t > 2n^3 (code/SA_RRG.py:
    72-85), or until the wall cap; the done flags are read once per chunk."""
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sa = mjx.SAReplicas(graphs, p, c, seeds)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    chunk, t0, taken = 4096, time.perf_counter(), 0
    while not sa.all_done() and time.perf_counter() - t0 < cap_s:
        sa.steps(chunk)
        taken += chunk
        chunk = min(2 * chunk, 65536)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = sa.results()
    steps, mag, done = out["num_steps"], out["mag_reached"], out["done"]
    fin = done != 0
    res = {"mode": sa.mode, "layout": sa.layout, "replicas": len(seeds), "init_s": init_s, "wall_s": wall,
           "all_done": bool(fin.all()), "replicas_done": int(fin.sum()), "wall_cap_s": cap_s,
           "proposals_launched_per_replica": taken,
           "num_steps": {"min": float(steps.min()), "median": float(np.median(steps)), "mean": float(steps.mean()),
                         "max": float(steps.max())},
           "mag_reached": {"min": float(mag.min()), "mean": float(mag.mean()), "max": float(mag.max())},
           "proposals_per_s": float(steps.sum()) / wall}
    if fin.any():
        res["done_num_steps"] = sorted(float(x) for x in steps[fin])
    del sa
    return res


def bench_sa_consensus(args, rank, world, dist, dev):
    """SA_RRG.py's own annealing problem (code/SA_RRG.py:44-52: d=4, p=3, c=1)
    run to the end, every replica on its own fresh graph, until m(s_endstate(s))
    = 1 or t > 2n^3 (code/SA_RRG.py:72-85), 64 replicas per GPU together:
      * to_consensus: n = --consensus-n (1000), where the runs end (1e5-1e7
        proposals per replica): wall time to consensus, the num_steps /
        mag_reached distributions (the script's np.savez keys);
      * script_size: the script's n = 1e4 for a fixed wall budget: there the
        runs need 4.4e7 to >5.8e8 proposals per replica (round 3, 1000 s on 64
        replicas: 50 done, profiles/r03_sa_consensus_n1e4_pair.log), so this
        reports the rate and how far the runs got."""
    import mjx
    d, p, c, R = 4, 3, 1, args.consensus_replicas
    out = {"config": f"SA_RRG.py's problem: d={d} RRG, p={p} c={c}, {R} replicas per GPU each on its own graph, "
                     "run until m_final = 1 or t > 2n^3"}
    for tag, n, cap in (("to_consensus", args.consensus_n, args.consensus_max_s),
                        ("script_size", 10_000, args.consensus_script_s)):
        if cap <= 0:
            continue
        graphs = [mjx.random_regular_graph(d, n, seed=args.seed + 5000 + R * rank + k) for k in range(R)]
        seeds = list(range(10_000 + rank * R, 10_000 + (rank + 1) * R))
        out[tag] = {"n": n, **_sa_until_done(mjx, graphs, p, c, seeds, cap)}
    return out


def bench_sa_global(args, rank, world, dist, dev):
    """The reference's own run, literally (code/SA_RRG.py:44-92): N_stat = 5
    replicas BACK TO BACK on ONE numpy stream seeded once, each on a fresh
    d=4 random regular graph, p=3, c=1, until m_final = 1 -- mjx.sa_run(...,
    stream="global"), replica k+1's draws continuing where replica k's last
    rand() left the stream.  One replica at a time is one workgroup: the
    whole-CU LDS kernel (k_sa_lds_cu).  Per replica: wall time to consensus,
    num_steps, mag_reached, us per proposal.  (Each rank runs its own seed.)"""
    import mjx
    n, d, p, c = args.global_n, 4, 3, 1
    seed, graph_seed = args.seed + 5 + 1000 * rank, args.seed + 70 + 1000 * rank
    res = mjx.sa_run(d, n, p, c, N_stat=args.global_nstat, seed=seed, graph_seed=graph_seed, stream="global",
                     max_seconds=args.global_max_s)
    reps = []
    for k in range(args.global_nstat):
        st, w = float(res["num_steps"][k]), float(res["wall_s"][k])
        if w == 0.0:
            break                                       # not run: an earlier replica hit the wall cap
        reps.append({"num_steps": st, "mag_reached": float(res["mag_reached"][k]), "done": int(res["done"][k]),
                     "wall_s": w, "us_per_step": 1e6 * w / max(st, 1.0)})
    return {"config": f"SA_RRG.py run: d={d} RRG n={n}, p={p} c={c}, N_stat={args.global_nstat} replicas back to "
                      f"back on one numpy stream (np.random.seed({seed})), fresh graph per replica "
                      f"(graph_seed {graph_seed}), until m_final = 1; wall cap {args.global_max_s} s per replica",
            "replicas": reps, "replicas_done": sum(r["done"] == 1 for r in reps),
            "wall_s_total": sum(r["wall_s"] for r in reps)}


def bench_er(args, rank, world, dist, dev):
    """configs[3]: Erdos-Renyi mean degree 5, N=1e7 (irregular CSR), replica
    parallel: every rank its own graph instance and R bit-packed replicas
    (weak scaling); p+c-1 = 2 sweeps + fused count per step."""
    import torch
    import mjx
    n, R, K = args.er_n, args.er_replicas, args.er_steps
    W = (R + 63) // 64
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = mjx.erdos_renyi_device(n, args.er_deg / (n - 1), seed=args.seed + 31 + 1000 * rank)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    g.class_ell()                    # degree-class ELL (nb:113-117's layout): setup, not timed
    torch.cuda.synchronize()
    layout_s = time.perf_counter() - t0
    gen = torch.Generator(device=dev).manual_seed(args.seed + 5 + rank)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device=dev, generator=gen)
    out, tmp = torch.empty_like(s0), torch.empty_like(s0)
    counts = torch.zeros(W * 64, dtype=torch.int64, device=dev)
    T = args.p + args.c - 1

    def step():
        counts.zero_()
        mjx.rollout(g, s0, T, words=W, out=out, tmp=tmp, counts=counts)

    # the random-row floor of the same step: T sweeps'
    # rows -- same class arrays, positions, unit mapping and resident grid, no
    # majority (mjx_gather_floor_class) -- in this process, on this box.  Step
    # and floor blocks alternate three times; each is reported as the median
    # (one block alone can catch a slow spell of the box)
    from mjx import _lib as L, _device as D
    order, cell, classes = g.class_ell()

    def floor_sweep():
        L.call("mjx_gather_floor_class", D.ptr(order), D.ptr(cell), classes.ctypes.data, classes.shape[0], n, W,
               D.ptr(s0), D.ptr(out), D.stream_handle())

    step()
    floor_sweep()
    els, floors = [], []
    for _ in range(3):
        els.append(_timed(lambda: [step() for _ in range(K)], dist, dev))
        floors.append(_timed(lambda: [floor_sweep() for _ in range(T * K)], dist, dev))
    el, el_floor = float(np.median(els)), float(np.median(floors))
    nnz = g.nnz
    # degree-class ELL sweep: int32 neighbours + int32 node order + state rows:
    # the deg neighbour rows, the row written, and the node's own row only
    # where a tie is possible (even degree, always-stay; nb:113-117) -- an
    # odd-degree class never reads it
    _, _, classes = g.class_ell()
    n_even = int(sum(int(cnt) for _, cnt, D, _ in classes.tolist() if D % 2 == 0))
    bytes_per_sweep = 4 * nnz + 4 * n + (W * 8) * (nnz + n + n_even)
    # sanity: an all-(+1) state is a fixed point of every node (isolated ones included)
    ones = torch.full_like(s0, -1)
    ck = torch.zeros_like(counts)
    assert torch.equal(mjx.rollout(g, ones, T, words=W, counts=ck), ones) and bool((ck == n).all())
    del s0, out, tmp, ones
    return {
        "config": f"configs[3]: ER mean degree {args.er_deg:g} N={n} (CSR generated on the device, own instance "
                  f"per GPU), {R} bit-packed "
                  f"replicas per GPU, {T} sweeps + fused count per step",
        "scaling": "weak", "ranks": world, "n": n, "nnz": nnz, "replicas_per_gpu": R, "steps": K,
        "device_graph_s": gen_s, "class_layout_s": layout_s,
        "layout": "degree-class ELL, one launch per degree class (nb:113-117)",
        "ms_per_step": 1e3 * el / K,
        # T floor sweeps (the step's rows, no majority, no count): the step over it
        "floor_ms": 1e3 * el_floor / K, "step_over_floor": el / el_floor,
        "step_ms_reps": [1e3 * x / K for x in els], "floor_ms_reps": [1e3 * x / K for x in floors],
        "floor_GBps": bytes_per_sweep * T * K / el_floor / 1e9,
        "node_updates_per_s": world * n * R * T * K / el,
        "algorithmic_bytes_per_sweep": bytes_per_sweep,
        "algorithmic_GBps_per_gpu": bytes_per_sweep * T * K / el / 1e9,
        "frac_of_hbm_peak": bytes_per_sweep * T * K / el / 1e9 / HBM_PEAK_GBS,
        # measured HBM bytes (rocprofv3 PMC FETCH/WRITE passes, same graph and replica count)
        "traffic": er_sweep_traffic(),
    }


def bench_bdcm(args, rank, world, dist, dev):
    """BDCM message passing at the notebook's regime (ER mean degree 5, n=1000,
    p=c=1, code/ER_BDCM_entropy.ipynb): BDCM_ER iterations/s with the
    convergence read-back the lambda loop does (nb:422-431), float64; the
    numpy restatement of one iteration timed beside it on one host core."""
    import torch
    import mjx
    from oracle import bdcm as orc
    n, deg, p, c = 1000, 5.0, 1, 1
    plan = mjx.bdcm_er_plan(n, deg / (n - 1), seed=args.seed + 77 + rank)
    rng = np.random.default_rng(args.seed + rank)
    chi0 = rng.random((2 * plan.E, 4 ** (p + c)))
    chi0 /= chi0.sum(axis=1, keepdims=True)
    chi = torch.from_numpy(chi0).to(dev)
    mjx.bdcm_leaf_reset(chi, plan, p, c, 1, 0.5)
    K = args.bdcm_iters
    dbits = plan._delta

    def run():
        for _ in range(K):
            dbits.zero_()
            mjx.BDCM_ER(chi, plan, p, c, 1, 0.5, 0.1, delta=dbits)
            float(dbits.view(torch.float64).item())

    run()
    el_host = _timed(run, dist, dev)
    # the device loop (procedure default): captured batches of 32 gated sweeps,
    # one host read per batch; eps = 0 never converges, T_max = Kd stops it
    Kd = 32 * max(1, K // 32)

    def run_dev(graph=False):
        mjx.bdcm_converge(chi, plan, p, c, 1, 0.5, 0.1, 0.0, Kd, batch=32, graph=graph)

    run_dev()
    el = _timed(run_dev, dist, dev)
    run_dev(True)                                             # capture once (kept on the plan)
    el_graph = _timed(lambda: run_dev(True), dist, dev)
    res = {"config": "ER mean degree 5, n=1000, p=c=1, lambda=0.5, damp 0.1 (the notebook's regime), float64",
           "iters_per_s": world * Kd / el_graph, "ms_per_iter": 1e3 * el_graph / Kd,
           "device_loop": f"{Kd} gated sweeps as a replayed hipGraph of 32 (the procedure's default: one capture "
                          f"per plan, lambda from device memory), device stop flag, one host read per batch",
           "eager_ms_per_iter": 1e3 * el / Kd,
           "host_loop_ms_per_iter": 1e3 * el_host / K, "classes": len(plan.edge_classes)}
    if rank == 0 and world == 1:
        hp = orc.Plan.from_csr(plan.edges_host, plan.row_ptr_host, plan.col_host, plan.n, plan.n_iso)
        x = chi.cpu().numpy()
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < 3.0:
            x = orc.BDCM_ER(x, hp, p, c, 1, 0.5, 0.1)
            reps += 1
        res["cpu_ms_per_iter"] = 1e3 * (time.perf_counter() - t0) / reps
        res["cpu_kind"] = "port (oracle/bdcm.py numpy restatement, 1 core)"
    return res


FP32_VECTOR_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: the FP32 vector (= FP32 matrix) peak


def hpr_dp_flops(d, p, c):
    """Algorithmic FLOPs of one HPr_dp message update (all valid x_a of the
    message, attr_value = +1), counted the way the kernel evaluates the DP
    (csrc/mjx_hpr_impl.h xa_messages; code/HPR_pytorch_RRG.py:183-218):
    bias x chi for the d-1 incoming rows, the count-table convolution of
    incoming neighbours 1..d-3 into neighbour 0's table (one multiply, then
    FMAs), the directional cumulative sums (one add per entry with a
    successor in each of the T dimensions), and the fold of the last incoming
    row (an FMA per non-empty corner, the weight and the row sum).  The
    corner rule restates corner() of the kernel."""
    T = p + c
    X, K = 1 << T, d - 2
    base = K + 1
    NS = base ** T

    def spin(x, t):
        return -1 if (x >> (T - 1 - t)) & 1 else 1

    def corner_ok(XA, x, XB):
        for t in range(T):
            s = spin(XA, t + 1) if t < T - 1 else spin(XA, p)
            prev = spin(XA, t) if t < T - 1 else spin(XA, T - 1)
            b, y = (1 if spin(x, t) > 0 else 0), spin(XB, t)
            if s > 0:
                lo = -((-(d - 1 - y + (0 if prev > 0 else 1))) // 2) - b
                if lo > K:
                    return False
            else:
                hi = (d - 1 - y + (0 if prev < 0 else -1)) // 2 - b
                if hi < 0:
                    return False
        return True

    def maxdigit(i):
        return max((i // base ** (T - 1 - t)) % base for t in range(T))

    total = 0
    for XA in range(0, X, 2):                      # x_a[T-1] = +1
        f = (d - 1) * X
        for j in range(1, K):
            f += sum(2 * X - 1 for i in range(NS) if maxdigit(i) <= j)
        f += T * (NS // base) * K
        f += sum(2 for x in range(X) for xb in range(X) if corner_ok(XA, x, xb)) + 2 * X
        total += f
    return total


def sq_counters(kernel_prefix):
    """wait / VALU-active fractions of a kernel from the newest committed SQ
    counter pass that holds it (profiles/rNN_sq_counters*.json, written by
    tools/pmc_sq_parse.py from the `sq` step of tools/gpu_check.sh), or None."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_sq_counters*.json")),
                   key=lambda p: (os.path.basename(p)[:3], os.path.basename(p)), reverse=True)
    for path in paths:
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if k.startswith("_") or kernel_prefix not in k:
                continue
            return {"kernel": k, "wait_frac": v.get("wait_frac"), "valu_active_frac": v.get("valu_active_frac"),
                    "source": "profiles/" + os.path.basename(path)}
    return None


def bench_hpr(args, rank, world, dist, dev):
    """configs[2]: HPR on a d=4 RRG with N=1e5, p=2, c=2, fp32 edge messages
    (code/HPR_pytorch_RRG.py:342-362): one iteration = HPr_dp (the message
    update, dominant) + marginals_comp, timed with HIP events; each rank its own
    graph (replicas only).  The numpy float64 restatement of HPr_dp
    (oracle/hpr.py, the reference's dtype) is timed beside it on a bounded
    sample of output rows of the same graph, one host core."""
    import torch
    import mjx
    n, d, p, c = args.hpr_n, 4, 2, 2
    edges = mjx.random_regular_edges(d, n, seed=args.seed + 31 + rank)
    plan = mjx.HPRPlan(edges, n, d)
    nc = plan.num_combs(p, c)
    gen = torch.Generator(device=dev).manual_seed(args.seed + rank)
    chi = torch.rand((2 * plan.E, nc), dtype=torch.float32, device=dev, generator=gen)
    chi /= chi.sum(1, keepdim=True)
    b = torch.rand((n, 2), dtype=torch.float32, device=dev, generator=gen)
    b /= b.sum(1, keepdim=True)
    out = torch.empty_like(chi)
    z = torch.empty(4 * plan.E, dtype=chi.dtype, device=dev)
    mg = torch.empty((n, 2), dtype=chi.dtype, device=dev)
    lmbd = 25 * n
    K = args.hpr_iters
    stream = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def run():
        e[0].record(stream)
        for _ in range(K):
            mjx.HPr_dp(chi, b, plan, p, c, 1, lmbd, 0.4, out=out)
        e[1].record(stream)
        for _ in range(K):
            mjx.marginals_comp(out, plan, p, c, zwork=z, out=mg)
        e[2].record(stream)

    run()
    el = _timed(run, dist, dev)
    upd_ms = e[0].elapsed_time(e[1]) / K
    marg_ms = e[1].elapsed_time(e[2]) / K
    msgs = 2 * plan.E
    # bytes k_hpr_update moves per message: its incoming row once (each row is
    # incoming to exactly one node's tile and staged there once), its own old
    # row (damping), the new row written, plus the in_row/out_row/nbr indices
    # and the source's two biases (HPR)
    bytes_per_iter = msgs * (3 * nc * 4 + 3 * 4 + 2 * 4)
    # marginals: every row read once (+ the Z pairs and the (n, 2) marginals written)
    marg_bytes = msgs * nc * 4 + msgs * 2 * 4 + n * 2 * 4
    res = {"config": f"configs[2]: HPR d={d} RRG N={n}, p={p} c={c} ({nc} columns), fp32 messages, "
                     "one iteration = HPr_dp + marginals_comp",
           "scaling": "weak", "ranks": world, "messages": msgs,
           "ms_per_iter": 1e3 * el / K, "iters_per_s": world * K / el,
           "hpr_dp_ms": upd_ms, "marginals_ms": marg_ms,
           "messages_per_s": world * msgs * K / el,
           "hpr_dp_algorithmic_GBps": bytes_per_iter / (upd_ms / 1e3) / 1e9,
           "hpr_dp_frac_of_hbm_peak": bytes_per_iter / (upd_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
           "hpr_dp_bytes_per_iter": bytes_per_iter,
           "marginals_algorithmic_GBps": marg_bytes / (marg_ms / 1e3) / 1e9,
           "marginals_bytes_per_iter": marg_bytes,
           "hpr_dp_traffic_bytes": rocprof_traffic("k_hpr_update_pipe"),
           "marginals_edge_z_traffic_bytes": rocprof_traffic("k_hpr_edge_z")}
    # the loop's own state layout (HPRState layout="q", the default of hpr_run
    # here): invalid-sender quadrants kept undecayed, read with the scale
    st = mjx.HPRState(plan, p, c, chi, b, dtype=torch.float32, layout="q")
    from mjx import _lib as L, _device as D
    code, sptr, sz = L.MJX_F32, st._sc.data_ptr(), st._sc.element_size()
    wp, wm = math.exp(-lmbd / n), math.exp(lmbd / n)
    bufs = (st.chi, st.chi_b)

    def run_q():
        s_ = D.stream_handle()
        e[0].record(stream)
        for k in range(K):
            L.call("mjx_hpr_update_q", code, bufs[k % 2].data_ptr(), bufs[1 - k % 2].data_ptr(), st.biases.data_ptr(),
                   plan.nbr.data_ptr(), plan.in_row.data_ptr(), plan.out_row.data_ptr(), n, d, p, c, 1, wp, wm, 0.4,
                   sptr, s_)
        e[1].record(stream)
        for k in range(K):
            L.call("mjx_hpr_marginals_q", code, bufs[k % 2].data_ptr(), plan.out_row.data_ptr(), n, d, p, c, 1e-15,
                   sptr + sz, st._ii.data_ptr(), st.zwork.data_ptr(), st.marg.data_ptr(), s_)
        e[2].record(stream)

    run_q()
    el_q = _timed(run_q, dist, dev)
    upd_q = e[0].elapsed_time(e[1]) / K
    marg_q = e[1].elapsed_time(e[2]) / K
    # per message: first half of its old row (damping) + the VV and IV quadrants
    # of its incoming row + first half written, indices and biases
    qbytes = msgs * (3 * (nc // 2) * 4 + 3 * 4 + 2 * 4)
    res["loop_state_q"] = {
        "layout": "decay-split (HPRState layout='q'): invalid-sender quadrants undecayed, read with (1-damp)^t",
        "ms_per_iter": 1e3 * el_q / K, "iters_per_s": world * K / el_q, "messages_per_s": world * msgs * K / el_q,
        "hpr_dp_ms": upd_q, "marginals_ms": marg_q, "hpr_dp_bytes_per_iter": qbytes,
        "hpr_dp_algorithmic_GBps": qbytes / (upd_q / 1e3) / 1e9,
        "hpr_dp_frac_of_hbm_peak": qbytes / (upd_q / 1e3) / 1e9 / HBM_PEAK_GBS,
        "hpr_dp_traffic_bytes": rocprof_traffic("k_hpr_update_q3"),
        "marginals_edge_z_traffic_bytes": rocprof_traffic("k_hpr_edge_z_q")}
    # the compute side of the same launch (the DP is a mixed contraction)
    fl = msgs * hpr_dp_flops(d, p, c)
    res["loop_state_q"]["hpr_dp_compute"] = {
        "flops_per_launch": fl, "achieved_tflops": fl / (upd_q / 1e3) / 1e12, "peak_tflops": FP32_VECTOR_PEAK_TFLOPS,
        "frac": fl / (upd_q / 1e3) / 1e12 / FP32_VECTOR_PEAK_TFLOPS, "sq": sq_counters("k_hpr_update_q3")}
    # the whole loop iteration of code/HPR_pytorch_RRG.py:344-356 (update,
    # marginals, bias refresh, trial configuration, majority check) in
    # hipGraph-replayed batches of 16 with one host read per batch
    gcpu = torch.Generator().manual_seed(args.seed + rank)
    st.steps_batched(16, gcpu)                      # eager batch
    st.steps_batched(16, gcpu)                      # capture + replay
    nb = max(1, K // 4)
    st.rng_attach(gcpu)
    drawn = [st.draw_batch_device(16)]

    def run_loop():
        # hpr_run's loop: the next batch's uniforms drawn (the CPU generator's
        # stream continued on the device, its own stream) while this batch
        # runs, one host read per batch
        for _ in range(nb):
            st.launch_batch(drawn[0])
            drawn[0] = st.draw_batch_device(16, st.t)
            st.collect_batch()

    el_loop = _timed(run_loop, dist, dev)
    res["loop_state_q"]["loop_ms_per_iter"] = 1e3 * el_loop / (16 * nb)
    res["loop_state_q"]["loop_note"] = ("hpr_run's loop in batches of 16: update + marginals + new_biases_i + "
                                        "pack + p+c-1 sweeps + count per iteration on the device; the reference's "
                                        "torch.rand(n) per iteration (CPU generator stream) continued on the device "
                                        "on a stream of its own beside the batch; one host read per batch")
    del st
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the reference runs HPr_dp as torch ops; on the host that is torch's CPU
        # backend with every core: oracle/hpr_torch.py, the same DP in torch ops
        from oracle import hpr as ohpr
        from oracle import hpr_torch
        inr, src = ohpr.incoming_rows(plan.edges, plan.nbrs_host)
        chi_h = chi.double().cpu()
        b_h = b.double().cpu()
        rows = np.random.default_rng(0).choice(msgs, size=2048, replace=False)
        cores = cpu_share()[0]
        old_threads = torch.get_num_threads()
        torch.set_num_threads(cores)
        hpr_torch.HPr_dp(chi_h, b_h, inr, src, n, d, p, c, 1, lmbd, 0.4, rows[:64])      # warm-up
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < 5.0:
            hpr_torch.HPr_dp(chi_h, b_h, inr, src, n, d, p, c, 1, lmbd, 0.4, rows)
            done += rows.size
        cpu_s = time.perf_counter() - t0
        torch.set_num_threads(old_threads)
        res["cpu_baseline"] = {"messages_per_s": done / cpu_s, "cores": cores, "kind": "port", "host": host_info(),
                               "sample": f"oracle/hpr_torch.py HPr_dp (torch CPU ops, float64, "
                                         f"code/HPR_pytorch_RRG.py:183-218) on {rows.size} sampled output rows of "
                                         f"the same graph, repeated for {cpu_s:.1f} s, torch threads = {cores}",
                               "ms_per_iter_equiv": 1e3 * msgs / (done / cpu_s)}
        res["speedup_vs_cpu"] = res["messages_per_s"] / res["cpu_baseline"]["messages_per_s"]
    return res


def bench_giant(args, rank, world, dist, dev):
    """configs[4]: ONE d=6 RRG with N=1e9 nodes, partitioned by node range over
    the ranks (strong scaling); each rank generates its own rows on its GPU and
    every sweep ends with an in-place RCCL all-gather of the packed state."""
    import torch
    import mjx
    n, d, K = args.giant_n, args.giant_d, args.giant_sweeps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sh = mjx.ShardedRRG(d, n, seed=args.seed + 12345, mode=args.giant_mode, pieces=args.giant_pieces)
    sh.drop_adjacency()
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    gen = torch.Generator(device=dev).manual_seed(args.seed + 99)     # same replicated state on every rank
    sh.buf[sh.cur].copy_(torch.randint(-2 ** 62, 2 ** 62, sh.buf[sh.cur].shape, dtype=torch.int64, device=dev,
                                       generator=gen))
    sh.rollout(2)                                                    # warm-up
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        ev0.record(stream)
        for _ in range(K):
            sh.sweep()
        ev1.record(stream)

    el = _timed(run, dist, dev)
    ev_ms = ev0.elapsed_time(ev1)
    per_update_bytes = 4 * d + (d + 2) / 8.0          # 4 d/R + (d+2)/8 at R = 1
    rows, npieces = sh.range.rows, sh.range.npieces
    del sh
    torch.cuda.empty_cache()
    return {
        "config": f"configs[4]: one d={d} RRG N={n} partitioned by node range over {world} GPU(s), "
                  "per-sweep in-place RCCL all-gather of the node-packed state; setup = device generation "
                  "(+ source-binned plan)",
        "scaling": "strong", "ranks": world, "n": n, "d": d, "sweeps": K, "mode": args.giant_mode,
        "setup_s": gen_s,
        # the C5 job as SURVEY.md 8(d) states it: setup (device generation + plan)
        # + K sweeps, the two barrier-bracketed regions summed (the state fill
        # and two warm-up sweeps between them excluded)
        "job_s": gen_s + el,
        "ms_per_sweep": 1e3 * el / K,
        "node_updates_per_s": n * K / el,
        "algorithmic_GBps": n * K * per_update_bytes / el / 1e9,
        "stream_ms_per_sweep": ev_ms / K,
        "rows_per_rank": rows, "pieces_per_rank": npieces,
    }


def rocprof_traffic(kernel_prefix="k_sweep_ell_rp"):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if any
    (profiles/pmc_traffic.json, written by tools/pmc_parse.py from
    rocprofv3 --pmc passes over tools/pmc_run.py)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_prefix, {}).get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def er_sweep_traffic():
    """Measured HBM bytes of one ER step (one plain + one counting degree-class
    sweep, every class launch summed) from profiles/pmc_traffic.json, whose
    ER pass (tools/pmc_run.py) runs the bench's own graph (N=1e7, mean degree
    5, seed 31) and replica count; None if absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    plain = sum(v["bytes_per_launch"] for k, v in d.items() if k.startswith("mjx::k_sweep_cls") and "false" in k)
    # the counting sweep: k_sweep_cls_all_rp (the D <= 8 classes in one launch) + the D > 8 tail
    count = sum(v["bytes_per_launch"] for k, v in d.items()
                if k.startswith("mjx::k_sweep_cls") and ("true" in k or k.startswith("mjx::k_sweep_cls_all_rp")))
    return {"plain_sweep_bytes": plain, "counting_sweep_bytes": count} if plain and count else None


LEG_KEYS = ("sa", "sa_c1", "sa_consensus", "sa_global", "er", "hpr", "bdcm", "giant")
# prose and per-replica arrays: kept in the detail file, not on the printed line
_DROP = {"config", "sample", "host", "note", "loop_note", "device_loop", "done_num_steps", "source",
         "replicas", "kind_note"}


def compact(v):
    """A leg's numbers for the printed line: prose, host descriptions and
    per-replica arrays dropped (they stay in the detail file), floats to 4
    significant digits."""
    if isinstance(v, dict):
        return {k: compact(x) for k, x in v.items() if k not in _DROP and not (isinstance(x, str) and len(x) > 40)}
    if isinstance(v, list):
        return [compact(x) for x in v[:8]]
    if isinstance(v, float):
        return float(f"{v:.4g}")
    return v


def _get(d, *path):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return float(f"{d:.4g}") if isinstance(d, float) else d


def summary(line):
    """One compact object per SURVEY.md 8 config, the last key of the line:
    the driver keeps only the tail of stdout, so every leg's headline number
    sits here."""
    sg = line.get("sa_global") or {}
    return {
        "headline_node_updates_per_s": _get(line, "value"), "headline_frac": _get(line, "roofline", "frac"),
        "c2_mt_props_per_s": _get(line, "sa", "lightcone", "proposals_per_s"),
        "c2_sa_sweeps_per_s": _get(line, "sa", "lightcone", "sweeps_per_s"),     # BASELINE.json: SA sweeps/s
        "c2_philox_props_per_s": _get(line, "sa", "lightcone_philox", "proposals_per_s"),
        "c2_rollout_props_per_s": _get(line, "sa", "rollout", "proposals_per_s"),
        "c1_props_per_s": _get(line, "sa_c1", "proposals_per_s"),
        "c1_cpu_props_per_s": _get(line, "sa_c1", "cpu_baseline", "proposals_per_s"),
        "sa_global_wall_s": _get(sg, "wall_s_total"), "sa_global_done": sg.get("replicas_done"),
        "script_size_done": _get(line, "sa_consensus", "script_size", "replicas_done"),
        "c4_ms_per_step": _get(line, "er", "ms_per_step"), "c4_frac": _get(line, "er", "frac_of_hbm_peak"),
        "c4_floor_ms": _get(line, "er", "floor_ms"),
        "c3_hpr_dp_ms": _get(line, "hpr", "loop_state_q", "hpr_dp_ms"),
        "c3_loop_ms_per_iter": _get(line, "hpr", "loop_state_q", "loop_ms_per_iter"),
        "c5_ms_per_sweep": _get(line, "giant", "ms_per_sweep"), "c5_setup_s": _get(line, "giant", "setup_s"),
        "c5_job_s": _get(line, "giant", "job_s"), "c5_sweeps": _get(line, "giant", "sweeps"),
    }


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        dry_run(args, rank, world)
        return
    n, d, R = args.n, args.d, args.replicas
    T = args.p + args.c - 1
    W = (R + 63) // 64

    import mjx
    adj = mjx.random_regular_graph(d, n, seed=args.seed + 1000 * rank)

    cpu = c1_cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(adj, T, args.cpu_seconds)
        if not args.no_sa and args.c1_steps > 0:
            c1_cpu = sa_cpu_baseline(c1_graphs(args, 0), 1, 1, list(range(64)), args.c1_cpu_seconds)

    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    g = mjx.Graph.ell(adj)
    gen = torch.Generator(device=dev).manual_seed(args.seed + rank)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device=dev, generator=gen)
    out = torch.empty_like(s0)
    tmp = torch.empty_like(s0)
    counts = torch.zeros(W * 64, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        counts.zero_()
        mjx.rollout(g, s0, T, words=W, out=out, tmp=tmp, counts=counts)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    updates = world * n * R * T * args.steps
    value = updates / elapsed

    # roofline of the sweep kernel: algorithmic bytes per launch / avg duration.
    # The events bracket only this stream's work: K steps x T sweeps plus one
    # tiny memset of the counts per step.
    bytes_per_sweep = 4 * d * n + (R // 8) * n * (d + 2)
    sweep_s = (ev_ms / 1e3) / (args.steps * T)
    achieved = bytes_per_sweep / sweep_s / 1e9
    traffic = rocprof_traffic()

    # sanity: the rollout of a constant state is the same constant state
    chk = torch.full_like(s0, -1)
    ck = torch.zeros_like(counts)
    o2 = mjx.rollout(g, chk, T, words=W, counts=ck)
    assert torch.equal(o2, chk) and bool((ck == n).all()), "fixed-point check failed"

    sa_res = None
    if not args.no_sa and args.sa_steps > 0:
        sa_res = bench_sa(args, rank, world, dist, dev)
    c1 = None
    if not args.no_sa and args.c1_steps > 0:
        c1 = bench_sa_c1(args, rank, world, dist, dev, c1_cpu)
    cons = None
    if not args.no_sa and not args.no_consensus and args.consensus_replicas > 0:
        cons = bench_sa_consensus(args, rank, world, dist, dev)
    sglob = None
    if not args.no_sa and not args.no_global and args.global_nstat > 0:
        sglob = bench_sa_global(args, rank, world, dist, dev)

    del s0, out, tmp, counts, chk, o2
    torch.cuda.empty_cache()
    er = None
    if not args.no_er and args.er_n > 0:
        er = bench_er(args, rank, world, dist, dev)
        torch.cuda.empty_cache()
    hpr = None
    if not args.no_hpr and args.hpr_iters > 0:
        hpr = bench_hpr(args, rank, world, dist, dev)
        torch.cuda.empty_cache()
    bdcm = None
    if not args.no_bdcm and args.bdcm_iters > 0:
        bdcm = bench_bdcm(args, rank, world, dist, dev)
    giant = None
    if not args.no_giant and args.giant_n > 0:
        giant = bench_giant(args, rank, world, dist, dev)

    for leg in (sa_res, c1, cons, sglob, er, hpr, bdcm, giant):
        if leg is not None:
            leg["n_gpus"] = world
            leg["ranks"] = world
    if rank == 0:
        line = {
            "metric": "node-updates/s, d=4 RRG majority rollout (s_endstate + m of bit-packed replicas)",
            "value": value,
            "unit": "node-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64 bit-packed spins (int32 indices)",
            "data": "synthetic: own random d-regular graph per rank, random +-1 spins",
            "config": {
                "workload": f"d={d} RRG N={n}, R={R} replicas/GPU, p={args.p} c={args.c} "
                            f"({T} sweeps per step) + fused per-replica +1 count",
                "n": n, "d": d, "replicas_per_gpu": R, "sweeps_per_step": T,
                "parallelism": f"replica/instance sharding x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_sweep_ell_rp<4,2,*>",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "bytes_per_launch": bytes_per_sweep,
                "avg_launch_us": sweep_s * 1e6,
            },
            "cpu_baseline": cpu,
            "sa": sa_res,
            "sa_c1": c1,
            "sa_consensus": cons,
            "sa_global": sglob,
            "er": er,
            "hpr": hpr,
            "bdcm": bdcm,
            "giant": giant,
        }
        detail = args.detail_out or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(line, f, indent=1)
        except OSError as e:
            print(f"bench.py: could not write {detail}: {e}", file=sys.stderr, flush=True)
        out = {k: (compact(v) if k in LEG_KEYS else v) for k, v in line.items()}
        out["detail_file"] = os.path.relpath(detail, ROOT) if detail.startswith(ROOT) else detail
        out["summary"] = summary(line)                  # the LAST key: inside any tail of the line
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
