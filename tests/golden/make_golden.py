"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where the reference is mounted read-only at
/root/reference.  The reference scripts execute their experiments at import,
so they are not imported: their ``def``/``import`` statements are
AST-extracted and exec'd with the module globals they read injected
(SURVEY.md 8c recipe).  Full-script runs use text substitution of the
parameter constants.  Only data (inputs and the reference's outputs) is
written; no reference source is copied.

Usage:  python tests/golden/make_golden.py [dyn] [er] [sa] [sa_full] [hpr] [hpr_full] [bdcm]
"""
import ast
import json
import os
import random
import sys
import time

import numpy as np

REF = os.environ.get("MJX_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
SA_PATH = os.path.join(REF, "code", "SA_RRG.py")
HPR_PATH = os.path.join(REF, "code", "HPR_pytorch_RRG.py")
NB_PATH = os.path.join(REF, "code", "ER_BDCM_entropy.ipynb")

PC_CASES = [(1, 1), (2, 1), (2, 2), (3, 1)]


def _defs_only(src, filename):
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.Import, ast.ImportFrom))]
    return compile(ast.Module(body=keep, type_ignores=[]), filename, "exec")


def load_ref(path, **inject):
    """Exec only the function definitions and imports of a reference file."""
    with open(path) as f:
        src = f.read()
    g = {"__name__": "ref_" + os.path.basename(path).split(".")[0]}
    g.update(inject)
    exec(_defs_only(src, path), g)
    return g


def notebook_source():
    with open(NB_PATH) as f:
        nb = json.load(f)
    cells = [c for c in nb["cells"] if c["cell_type"] == "code"]
    return "".join(cells[0]["source"])


def load_nb(**inject):
    g = {"__name__": "ref_nb"}
    g.update(inject)
    exec(_defs_only(notebook_source(), NB_PATH), g)
    return g


# ---------------------------------------------------------------------------
def gen_dyn():
    """RRG majority rollouts: reference neighbours() + s_endstate() (numpy,
    code/SA_RRG.py) and the torch twins of code/HPR_pytorch_RRG.py."""
    import networkx as nx
    import torch
    out = {}
    for d in (3, 4, 6):
        for n in (64, 1000):
            ref = load_ref(SA_PATH, n=n, d=d)
            random.seed(1000 * d + n)
            G = nx.random_regular_graph(d, n)
            N = ref["neighbours"](G)
            rng = np.random.default_rng(7 * d + n)
            S0 = 2 * rng.integers(0, 2, size=(3, n)).astype(np.int64) - 1
            key = f"d{d}_n{n}"
            out[f"{key}_N"] = N.astype(np.int32)
            out[f"{key}_s0"] = S0
            for (p, c) in PC_CASES:
                out[f"{key}_p{p}c{c}"] = np.stack([ref["s_endstate"](N, s0, p, c) for s0 in S0])
            out[f"{key}_m"] = np.array([ref["m"](s0) for s0 in S0])
            # torch twin (code/HPR_pytorch_RRG.py:169-180), int32 spins as there
            refh = load_ref(HPR_PATH, n=n, d=d, device=torch.device("cpu"))
            Nt = torch.tensor(N, dtype=torch.int32)
            for (p, c) in PC_CASES:
                st = torch.stack([refh["s_endstate"](Nt, torch.tensor(s0, dtype=torch.int32), p, c) for s0 in S0])
                assert np.array_equal(st.numpy(), out[f"{key}_p{p}c{c}"]), "numpy/torch reference disagree"
    np.savez_compressed(os.path.join(OUT, "rrg_dyn.npz"), **out)
    print("rrg_dyn.npz", len(out), "arrays")


def gen_er():
    """ER majority rollouts with the notebook's own graph builder and its
    degree-class onestep_majority (nb:113-123, 278-369)."""
    nb = load_nb()
    out = {}
    for (n, deg, gseed) in ((2000, 5.0, 11), (500, 1.0, 12), (1000, 2.0, 13)):
        T = 2
        random.seed(gseed)
        res = nb["GENERAL_ERgraph_and_auxialiaryarrays_generation"](n, deg / (n - 1), 1, 1, T, 1)
        (avg_deg, n_core, n_iso, num_edg, adj_matrix, degrees_all, degrees_nodes, N_nodes, A, Ai,
         N_edges_pos_dm1, N_edges_pos_full, N_edges_pos_full_marginals, N_nodes_pos, edges_with_d_positions,
         nodes_with_d_positions, degrees_edges, edges) = res
        row_ptr = np.zeros(n_core + 1, np.int64)
        cols = []
        for i in range(n_core):
            row_ptr[i + 1] = row_ptr[i] + len(N_nodes[i])
            cols.extend(N_nodes[i])
        rng = np.random.default_rng(gseed)
        S0 = 2 * rng.integers(0, 2, size=(3, n_core)).astype(np.int64) - 1
        key = f"er_n{n}_deg{deg:g}"
        out[f"{key}_row_ptr"] = row_ptr
        out[f"{key}_col"] = np.asarray(cols, np.int32)
        out[f"{key}_s0"] = S0
        out[f"{key}_iso"] = np.array(n_iso)
        for (p, c) in PC_CASES:
            out[f"{key}_p{p}c{c}"] = np.stack([
                nb["s_endstate"](nodes_with_d_positions, degrees_nodes, N_nodes_pos, s0, p, c) for s0 in S0])
    np.savez_compressed(os.path.join(OUT, "er_dyn.npz"), **out)
    print("er_dyn.npz", len(out), "arrays")


# ---------------------------------------------------------------------------
def sa_harness(ref, N, n, p, c, seed, max_steps, par_a=1.0005, par_b=1.0005):
    """The loop of code/SA_RRG.py:63-88 around the reference's own E_delta,
    s_endstate and m, on numpy's global stream, recording every step."""
    np.random.seed(seed)
    s = 2 * np.random.binomial(n=1, p=0.5, size=[n]) - 1
    s0 = s.copy()
    a = 0.015 * n
    b = 0.01 * n
    t = 0
    m_final = ref["m"](ref["s_endstate"](N, s, p, c))
    tr_i, tr_acc, tr_sum, tr_dE = [], [], [], []
    while m_final < 1:
        if t >= max_steps:
            break
        i = np.random.randint(low=0, high=n)
        delta_H = ref["E_delta"](N, s, a, b, p, c, i)
        prob_accept = min([1, np.exp(-delta_H)])
        acc = np.random.rand() < prob_accept
        if acc:
            s[i] = -s[i]
        if a < 4.5 * n:
            a = par_a * a
        if b < 5 * n:
            b = par_b * b
        t += 1
        if t > (2 * n ** 3):
            m_final = 2
        else:
            m_final = ref["m"](ref["s_endstate"](N, s, p, c))
        tr_i.append(i)
        tr_acc.append(int(acc))
        tr_sum.append(int(round(m_final * n)) if m_final != 2 else 0)
        tr_dE.append(delta_H)
    return {"s0": s0, "conf": s, "num_steps": t, "mag_reached": ref["m"](s), "converged": int(m_final >= 1),
            "i": np.asarray(tr_i, np.int32), "accept": np.asarray(tr_acc, np.int8),
            "sum_end": np.asarray(tr_sum, np.int32), "dE": np.asarray(tr_dE, np.float64)}


SA_CASES = [
    # (name, d, n, p, c, graph seed, numpy seeds, max steps recorded)
    ("sa_d4_n200_p3c1", 4, 200, 3, 1, 1, (0, 1, 2, 3), 10 ** 6),
    ("sa_d3_n300_p2c1", 3, 300, 2, 1, 2, (5, 6), 10 ** 6),
    ("sa_d4_n200_p1c1", 4, 200, 1, 1, 3, (1,), 20000),
    ("sa_d4_n1000_p2c2", 4, 1000, 2, 2, 4, (9,), 3000),
]


def gen_sa():
    import networkx as nx
    for (name, d, n, p, c, gseed, seeds, max_steps) in SA_CASES:
        ref = load_ref(SA_PATH, n=n, d=d)
        random.seed(gseed)
        G = nx.random_regular_graph(d, n)
        N = ref["neighbours"](G)
        out = {"N": N.astype(np.int32), "p": np.array(p), "c": np.array(c), "seeds": np.array(seeds)}
        for sd in seeds:
            t0 = time.time()
            r = sa_harness(ref, N, n, p, c, sd, max_steps)
            print(f"{name} seed {sd}: {r['num_steps']} steps converged={r['converged']} ({time.time() - t0:.1f}s)")
            for k, v in r.items():
                out[f"seed{sd}_{k}"] = np.asarray(v)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)


def gen_sa_full():
    """Whole-script runs of code/SA_RRG.py (constants substituted, np.savez
    re-enabled into a temp file) that pin the harness above: same graph seed
    and numpy seed must give the same conf / num_steps / mag_reached."""
    import tempfile
    with open(SA_PATH) as f:
        src = f.read()
    runs = {}
    # (n, d, p, graph seed, numpy seed, N_stat): N_stat = 2 pins the back-to-back
    # use of ONE numpy stream by consecutive replicas, each on its own graph
    for (n, d, p, gseed, nseed, nstat) in ((200, 4, 3, 1, 0, 1), (300, 3, 2, 2, 5, 1), (200, 4, 3, 3, 11, 2)):
        tmp = tempfile.mktemp(suffix=".npz")
        s = src
        # c stays the script's c=1 in every run
        for old, new in (("n=10000", f"n={n}"), ("d=4", f"d={d}"), ("p=3", f"p={p}"), ("N_stat=5", f"N_stat={nstat}")):
            assert old in s, old
            s = s.replace(old, new, 1)
        s = s.replace('#np.savez("MCMC_p3_d4.npz"', f'np.savez("{tmp}"')
        s = s.replace("for k in range(N_stat):", f"random.seed({gseed}); np.random.seed({nseed})\nfor k in range(N_stat):")
        s = "import random\n" + s
        g = {"__name__": "ref_sa_full"}
        exec(compile(s, SA_PATH, "exec"), g)
        z = np.load(tmp)
        runs[f"n{n}_d{d}_p{p}" + (f"_nstat{nstat}" if nstat > 1 else "")] = {k: z[k] for k in z.files}
        os.unlink(tmp)
        print("full script", n, d, p, "steps", z["num_steps"])
    out = {}
    for key, r in runs.items():
        for k, v in r.items():
            out[f"{key}_{k}"] = v
    np.savez_compressed(os.path.join(OUT, "sa_fullscript.npz"), **out)


# ---------------------------------------------------------------------------
# HPR (code/HPR_pytorch_RRG.py): one HPr_dp step, marginals_comp, new_biases_i,
# a short chain of full loop iterations, and a whole-script run.
# ---------------------------------------------------------------------------
HPR_CASES = [
    # (name, d, n, p, c, graph seed, torch seed, chain iterations)
    ("hpr_d4_n64_p1c1", 4, 64, 1, 1, 21, 1, 4),
    ("hpr_d4_n64_p2c2", 4, 64, 2, 2, 22, 2, 2),
    ("hpr_d3_n50_p2c1", 3, 50, 2, 1, 23, 3, 3),
    ("hpr_d4_n40_p1c2", 4, 40, 1, 2, 24, 4, 2),
    ("hpr_d5_n40_p1c1", 5, 40, 1, 1, 25, 5, 2),
    ("hpr_d3_n40_p3c1", 3, 40, 3, 1, 26, 6, 2),
]


def hpr_env(G, n, d, p, c):
    """Globals the reference's HPR functions read (code/HPR_pytorch_RRG.py:224-304)."""
    import itertools
    import torch
    T = p + c
    num_edg = int(n * d / 2)
    num_combs = 2 ** (2 * (p + c))
    x = torch.tensor([1, 0], dtype=torch.int)
    xi_comb = torch.cartesian_prod(*x.repeat(T, 1))
    edge_dict = {}
    N_nodes_order = np.zeros(2 * num_edg)
    for idx, edge in enumerate(G.edges):
        edge_dict[edge] = idx * num_combs
        edge_dict[edge[::-1]] = (idx + num_edg) * num_combs
        N_nodes_order[idx] = edge[0]
        N_nodes_order[idx + num_edg] = edge[1]
    env = dict(n=n, d=d, T=T, num_edg=num_edg, num_combs=num_combs, xi_comb=xi_comb,
               device=torch.device("cpu"), edge_dict=edge_dict)
    ref = load_ref(HPR_PATH, **env)
    xi_comb_cpu = np.array(list(itertools.product([1, -1], repeat=p + c)))
    pairs = np.zeros(num_combs)
    pji = np.zeros(num_combs)
    pls = mns = 0
    for idx, xixj in enumerate(itertools.product(xi_comb_cpu, repeat=2)):
        pairs[idx] = ref["order"](xixj[1], xixj[0], p, c)
        if xixj[1][0] == 1:
            pji[pls] = idx
            pls += 1
        else:
            pji[mns + int(num_combs / 2)] = idx
            mns += 1
    N_edg_pos_chi_mat = ref["neib_edg_pos_chi_mat"](G)
    N_edges_pos, N_nodes = ref["neighb_edges_pos_AND_nodes"](G)
    pos_biases = ref["positions_biases"](N_nodes_order, n, p, c, num_edg)
    rho = torch.zeros((2 ** T, T)).int()
    for idx, xi in enumerate(xi_comb):
        rho[idx] = xi
    aux = dict(pairs=torch.tensor(pairs).int(), pji=torch.tensor(pji).int(),
               N_edg_pos_chi_mat=torch.tensor(N_edg_pos_chi_mat).int(), N_edges_pos=torch.tensor(N_edges_pos).int(),
               N_nodes=torch.tensor(N_nodes).int(), pos_biases=torch.tensor(pos_biases).int(), rho_D11=rho)
    return ref, env, aux


def gen_hpr():
    import networkx as nx
    import torch
    torch.set_default_dtype(torch.float64)     # code/HPR_pytorch_RRG.py:11
    damppar, attr_value, pie, gamma = 0.4, 1, 0.3, 0.1
    for (name, d, n, p, c, gseed, tseed, chain) in HPR_CASES:
        t0 = time.time()
        lmbd_in = 25 * n
        random.seed(gseed)
        G = nx.random_regular_graph(d, n)
        ref, env, aux = hpr_env(G, n, d, p, c)
        torch.manual_seed(tseed)
        chi_mat = ref["mes_init_mat"](env["num_edg"], p, c)
        chi_col = chi_mat.reshape(-1)
        biases_i = torch.rand((n, 2))
        biases_i = biases_i / torch.sum(biases_i, axis=1, keepdims=True)
        out = {"edges": np.array(list(G.edges), dtype=np.int64), "n": np.array(n), "d": np.array(d),
               "p": np.array(p), "c": np.array(c), "damppar": np.array(damppar), "attr_value": np.array(attr_value),
               "lmbd_in": np.array(lmbd_in), "pie": np.array(pie), "gamma": np.array(gamma),
               "N_nodes": aux["N_nodes"].numpy(), "N_edges_pos": aux["N_edges_pos"].numpy(),
               "N_edg_pos_chi_mat": aux["N_edg_pos_chi_mat"].numpy(),
               "chi0": chi_mat.numpy().copy(), "biases0": biases_i.numpy().copy()}
        for k in range(chain):
            biases_chi = ref["new_biases_chi"](biases_i, aux["pos_biases"])
            rho_D1 = aux["rho_D11"].detach().clone()
            chi_col, chi_mat = ref["HPr_dp"](chi_mat, chi_col, biases_chi, rho_D1, aux["N_edg_pos_chi_mat"], d, p, c,
                                              attr_value, lmbd_in, damppar)
            marg = ref["marginals_comp"](chi_mat, aux["pairs"], aux["pji"], aux["N_edges_pos"],
                                         epsilon=torch.tensor(1e-15))
            st = torch.get_rng_state()
            u = torch.rand(n)
            torch.set_rng_state(st)
            biases_i, s = ref["new_biases_i"](biases_i, pie, gamma, marg, k)
            s_end = ref["s_endstate"](aux["N_nodes"], s, p, c)
            out[f"it{k}_chi"] = chi_mat.numpy().copy()
            out[f"it{k}_marg"] = marg.numpy().copy()
            out[f"it{k}_u"] = u.numpy().copy()
            out[f"it{k}_biases"] = biases_i.numpy().copy()
            out[f"it{k}_s"] = s.numpy().copy()
            out[f"it{k}_m_end"] = np.array(float(ref["m"](s_end)))
        out["chain"] = np.array(chain)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print(f"{name}: {chain} iterations ({time.time() - t0:.1f}s)")


def gen_hpr_full():
    """Whole-script runs of code/HPR_pytorch_RRG.py on the CPU (constants
    substituted, device forced to the CPU, seeds fixed, np.savez redirected)."""
    import tempfile
    with open(HPR_PATH) as f:
        src = f.read()
    out = {}
    # p+c = 4 cases: the decay-split fp32 loop state (hpr_run's fp32 default) applies there
    for (n, d, p, c, TT, gseed, tseed) in ((40, 4, 1, 1, 300, 31, 7), (30, 3, 2, 1, 300, 32, 8),
                                           (40, 4, 2, 2, 300, 33, 9), (40, 3, 3, 1, 300, 34, 10),
                                           (60, 4, 3, 1, 120, 35, 11)):
        key = f"n{n}_d{d}_p{p}c{c}"
        only = os.environ.get("HPR_FULL_ONLY")
        if only and key not in only.split(","):
            continue
        tmp = tempfile.mktemp(suffix=".npz")
        s = src
        # whole-line anchors: "p=1 c=1" also occurs in a comment above the
        # parameter block (code/HPR_pytorch_RRG.py:65, 224-237)
        for old, new in (("\nn=10000\n", f"\nn={n}\n"), ("\nd=4\n", f"\nd={d}\n"), ("\np=1\n", f"\np={p}\n"),
                         ("\nc=1\n", f"\nc={c}\n"), ("\nTT=10000", f"\nTT={TT}"),
                         ("device = torch.device('cuda' if torch.cuda.is_available() else 'cpu')",
                          "device = torch.device('cpu')"),
                         (".to(device='cuda')", ".to(device=device)"),
                         ('np.savez("hpr_d4_p1.npz"', f'np.savez("{tmp}"'),
                         ("for kkk in range(n_rep):", f"random.seed({gseed}); torch.manual_seed({tseed})\nfor kkk in range(n_rep):")):
            assert old in s, old
            s = s.replace(old, new, 1)
        g = {"__name__": "ref_hpr_full"}
        t0 = time.time()
        exec(compile(s, HPR_PATH, "exec"), g)
        z = np.load(tmp)
        for k in z.files:
            if k != "time":
                out[f"{key}_{k}"] = z[k]
        import networkx as nx
        random.seed(gseed)
        G = nx.random_regular_graph(d, n)
        out[f"{key}_edges"] = np.array(list(G.edges), dtype=np.int64)
        out[f"{key}_params"] = np.array([n, d, p, c, TT, tseed])
        os.unlink(tmp)
        print("hpr full script", key, "steps", z["num_steps"], "m", z["mag_reached"], f"({time.time() - t0:.1f}s)")
    path = os.path.join(OUT, "hpr_fullscript.npz")
    if os.environ.get("HPR_FULL_ONLY") and os.path.exists(path):
        with np.load(path) as old:                  # keep the other cases
            out = {**{k: old[k] for k in old.files}, **out}
    np.savez_compressed(path, **out)


# ---------------------------------------------------------------------------
# BDCM on Erdos-Renyi graphs (code/ER_BDCM_entropy.ipynb): the notebook's own
# graph builder, one BDCM_ER sweep with its observables, and the whole
# lambda procedure (iteration counts parsed from its printed output).
# ---------------------------------------------------------------------------
BDCM_CASES = [
    # (name, n, mean degree, p, c, graph seed, numpy seed, lambdas)
    ("bdcm_er_n300_deg2_p1c1", 300, 2.0, 1, 1, 41, 1, (0.0, 0.5, 1.0)),
    ("bdcm_er_n300_deg5_p1c1", 300, 5.0, 1, 1, 42, 2, (0.0, 0.5)),
    ("bdcm_er_n150_deg3_p2c1", 150, 3.0, 2, 1, 43, 3, (0.0, 0.4)),
    ("bdcm_er_n120_deg3_p1c2", 120, 3.0, 1, 2, 44, 4, (0.3,)),
]


def gen_bdcm():
    import contextlib
    import io
    import itertools
    import re
    attr_value, damppar, eps, epsilon, T_max = 1, 0.1, 1e-6, 0, 1300
    for (name, n, deg, p, c, gseed, nseed, lambdas) in BDCM_CASES:
        t0 = time.time()
        T = p + c
        nb = load_nb(T=T, p=p, c=c, n=n, attr_value=attr_value, eps=eps, damppar=damppar, epsilon=epsilon)
        random.seed(gseed)
        res = nb["GENERAL_ERgraph_and_auxialiaryarrays_generation"](n, deg / (n - 1), p, c, T, attr_value)
        (avg_deg, n_core, n_iso, num_edg, adj_matrix, degrees_all, degrees_nodes, N_nodes, A, Ai,
         N_edges_pos_dm1, N_edges_pos_full, N_edges_pos_full_marginals, N_nodes_pos, edges_with_d_positions,
         nodes_with_d_positions, degrees_edges, edges) = res
        nb.update(num_edg=num_edg, degrees_all=degrees_all, degrees_nodes=degrees_nodes, A=A, Ai=Ai,
                  N_edges_pos_dm1=N_edges_pos_dm1, N_edges_pos_full=N_edges_pos_full,
                  edges_with_d_positions=edges_with_d_positions, nodes_with_d_positions=nodes_with_d_positions,
                  degrees_edges=degrees_edges, edges=edges, N_G_without_isolated=n_core, number_iso=n_iso)
        row_ptr = np.zeros(n_core + 1, np.int64)
        cols = []
        for i in range(n_core):
            row_ptr[i + 1] = row_ptr[i] + len(N_nodes[i])
            cols.extend(N_nodes[i])
        np.random.seed(nseed)
        chi = np.random.random([2 * num_edg] + [2] * T + [2] * T)
        chi = nb["normalize"](chi)
        flat = lambda x: np.asarray(x).reshape(2 * num_edg, -1).copy()
        out = {"edges": np.asarray(edges[:num_edg], np.int64), "row_ptr": row_ptr, "col": np.asarray(cols, np.int64),
               "n": np.array(n), "n_iso": np.array(n_iso), "p": np.array(p), "c": np.array(c),
               "attr_value": np.array(attr_value), "damppar": np.array(damppar), "eps": np.array(eps),
               "epsilon": np.array(float(epsilon)), "T_max": np.array(T_max), "lambdas": np.array(lambdas, float),
               "chi0": flat(chi)}
        # one sweep at the last lambda: leaf reset exactly as nb:404-417, then BDCM_ER (nb:425)
        lm = float(lambdas[-1])
        ch = chi.copy()
        if degrees_edges[0] == 0:
            aux = np.zeros_like(ch[edges_with_d_positions[0]])
            zero_sum = np.zeros(T)
            for xi in itertools.product([1, 0], repeat=T):
                if xi[-1] == attr_value:
                    for xj in itertools.product([1, 0], repeat=T):
                        aux[tuple([slice(None)] + list(xi) + list(xj))] = nb["A_i_sums"](
                            2 * np.array(xi) - 1, 2 * np.array(xj) - 1, zero_sum, p, c, attr_value, lm)
            ch[edges_with_d_positions[0]] = nb["normalize"](aux)
        out["sweep_lmbd"] = np.array(lm)
        out["sweep_leaf"] = flat(ch)
        ch = nb["BDCM_ER"](ch, degrees_edges, edges_with_d_positions, N_edges_pos_dm1, A, p, c, attr_value, lm,
                           damppar, epsilon)
        out["sweep_chi"] = flat(ch)
        out["sweep_zi"] = nb["Zi_ER"](ch, degrees_nodes, nodes_with_d_positions, N_edges_pos_full, Ai, p, c, n_core,
                                      attr_value, lm)
        out["sweep_zij"] = nb["Zij"](ch, num_edg, epsilon)
        out["sweep_phi"] = np.array(nb["phi_BP_GENERAL_ER"](ch, num_edg, degrees_nodes, nodes_with_d_positions,
                                                            N_edges_pos_full, Ai, n_core, n, p, c, attr_value, lm,
                                                            epsilon, n_iso))
        out["sweep_m_init"] = np.array(nb["avg_m_init_GENERAL_ER"](ch, num_edg, degrees_all, edges, n, epsilon, n_iso))
        # the whole procedure (mutates its chi argument in place: it ends holding the last fixed point)
        run = chi.copy()
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            m_init, ent1, ent, counts = nb["BDCM_entropy_procedure_GENERAL_ER"](run, np.array(lambdas, float), T_max,
                                                                               0, 1e9, time.time())
        iters = [int(x) for x in re.findall(r"t=\s*(\d+)", buf.getvalue())]
        out.update(m_init=np.asarray(m_init), ent1=np.asarray(ent1), ent=np.asarray(ent), counts=np.array(counts),
                   iters=np.array(iters, np.int64), chi_final=flat(run))
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        print(f"{name}: n_core={n_core} iso={n_iso} E={num_edg} classes={list(degrees_edges)} iters={iters} "
              f"m_init={np.round(m_init, 5)} ent1={np.round(ent1, 5)} ({time.time() - t0:.1f}s)")


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit(f"reference not found at {REF}: fixtures can only be generated in the build container")
    what = sys.argv[1:] or ["dyn", "er", "sa", "sa_full"]
    for w in what:
        {"dyn": gen_dyn, "er": gen_er, "sa": gen_sa, "sa_full": gen_sa_full, "hpr": gen_hpr,
         "hpr_full": gen_hpr_full, "bdcm": gen_bdcm}[w]()
