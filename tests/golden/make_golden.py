"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where the reference is mounted read-only at
/root/reference.  The reference scripts execute their experiments at import,
so they are not imported: their ``def``/``import`` statements are
AST-extracted and exec'd with the module globals they read injected
(SURVEY.md 8c recipe).  Full-script runs use text substitution of the
parameter constants.  Only data (inputs and the reference's outputs) is
written; no reference source is copied.

Usage:  python tests/golden/make_golden.py [dyn] [er] [sa] [sa_full]
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
    for (n, d, p, gseed, nseed) in ((200, 4, 3, 1, 0), (300, 3, 2, 2, 5)):
        tmp = tempfile.mktemp(suffix=".npz")
        s = src
        for old, new in (("n=10000", f"n={n}"), ("d=4", f"d={d}"), ("p=3", f"p={p}"), ("c=1 ", "c=1 "),
                         ("N_stat=5", "N_stat=1")):
            assert old in s, old
            s = s.replace(old, new, 1)
        if p == 2:
            pass
        s = s.replace('#np.savez("MCMC_p3_d4.npz"', f'np.savez("{tmp}"')
        s = s.replace("for k in range(N_stat):", f"random.seed({gseed}); np.random.seed({nseed})\nfor k in range(N_stat):")
        s = "import random\n" + s
        if d == 3:
            # p+c for d=3 case: c stays 1 (p=2, c=1)
            pass
        g = {"__name__": "ref_sa_full"}
        exec(compile(s, SA_PATH, "exec"), g)
        z = np.load(tmp)
        runs[f"n{n}_d{d}_p{p}"] = {k: z[k] for k in z.files}
        os.unlink(tmp)
        print("full script", n, d, p, "steps", z["num_steps"])
    out = {}
    for key, r in runs.items():
        for k, v in r.items():
            out[f"{key}_{k}"] = v
    np.savez_compressed(os.path.join(OUT, "sa_fullscript.npz"), **out)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit(f"reference not found at {REF}: fixtures can only be generated in the build container")
    what = sys.argv[1:] or ["dyn", "er", "sa", "sa_full"]
    for w in what:
        {"dyn": gen_dyn, "er": gen_er, "sa": gen_sa, "sa_full": gen_sa_full}[w]()
