"""ORACLE (test infrastructure only): numpy float64 restatement of the BDCM
(backtracking dynamical cavity method) message update and observables of the
Erdos-Renyi notebook, code/ER_BDCM_entropy.ipynb ("nb:L" = raw JSON line L).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use it.

Follows:
  A_i_sums / atr_condition / traj_condition / attr_fix    nb:66-111
  normalize                                               nb:128-130
  BDCM_ER (per degree class, Gauss-Seidel across classes)  nb:133-198
  Zij                                                     nb:200-209
  Zi_ER                                                   nb:211-276
  GENERAL_ERgraph_and_auxialiaryarrays_generation         nb:278-369 (index arrays only)
  phi_BP_GENERAL_ER, avg_m_init_GENERAL_ER                nb:372-392
  BDCM_entropy_procedure_GENERAL_ER (leaf reset, loop)    nb:394-452

Layout (the reference's): chi[2E, 2^T (x_i), 2^T (x_j)] flattened to (2E, 4^T);
a trajectory index bit = 1 means spin +1, time 0 is the most significant bit
(the ndarray axes [2]*T are indexed by the values of itertools.product([1, 0]),
nb:150-154, so flat position 2^T - 1 is the all-(+1) trajectory).  Row r < E is list(G.edges)[r]
= (i, j) as the message i -> j, row r + E is j -> i (nb:303-314).
"""
import itertools

import numpy as np


def traj01(T):
    """(2^T, T) 0/1 index values (1 = spin +1) of the trajectory stored at flat
    position k: the bits of k, time 0 most significant (the notebook's
    ndarray axes [2]*T indexed by these values, nb:150-154)."""
    return np.array(list(itertools.product([0, 1], repeat=T)), dtype=np.int64)


def _sgn(x):
    return int(x > 0) - int(x < 0)


def allowed(xi, y, rho2, p, c):
    """atr_condition * traj_condition (nb:66-83) for a +-1 trajectory xi, the
    receiver's +-1 trajectory y (zeros for the node factor, nb:85-98) and the
    neighbour field 2*rho - D per time step."""
    T = p + c
    for t in range(T - 1):
        f = rho2[t] + y[t]
        if xi[t + 1] == _sgn(f):
            continue
        if f == 0 and xi[t + 1] == xi[t]:
            continue
        return 0
    f = rho2[T - 1] + y[T - 1]
    if xi[p] == _sgn(f):
        return 1
    if f == 0 and xi[p] == xi[T - 1]:
        return 1
    return 0


def _allowed_vec(xi, Y, rho2, p, c):
    """allowed() for one trajectory xi, every receiver row of Y (B, T) and every
    field row of rho2 (Q, T) at once: (B, Q) 0/1 (the same conditions, nb:66-83)."""
    T = p + c
    F = rho2[None, :, :] + Y[:, None, :]                      # (B, Q, T) field per time
    ok = np.ones(F.shape[:2], dtype=bool)
    for t in range(T - 1):
        f = F[:, :, t]
        ok &= (xi[t + 1] == np.sign(f)) | ((f == 0) & (xi[t + 1] == xi[t]))
    f = F[:, :, T - 1]
    ok &= (xi[p] == np.sign(f)) | ((f == 0) & (xi[p] == xi[T - 1]))
    return ok.astype(np.float64)


def factor_A(D, p, c, attr_value):
    """A[xi, xj, rho] for D incoming messages (nb:330-336, lambda = 0), 0/1."""
    T = p + c
    X = 2 ** T
    tr = 2 * traj01(T) - 1
    rhos = np.array(list(itertools.product(range(D + 1), repeat=T)), dtype=np.int64)
    A = np.zeros((X, X, rhos.shape[0]))
    for a in range(X):
        if tr[a][T - 1] != attr_value:                       # attr_fix (nb:103-105)
            continue
        A[a] = _allowed_vec(tr[a], tr, 2 * rhos - D, p, c)
    return A


def factor_Ai(D, p, c, attr_value):
    """Ai[xi, rho] of the node factor (nb:362-366), 0/1."""
    T = p + c
    X = 2 ** T
    tr = 2 * traj01(T) - 1
    rhos = np.array(list(itertools.product(range(D + 1), repeat=T)), dtype=np.int64)
    A = np.zeros((X, rhos.shape[0]))
    zero = np.zeros((1, T), dtype=np.int64)
    for a in range(X):
        if tr[a][T - 1] != attr_value:
            continue
        A[a] = _allowed_vec(tr[a], zero, 2 * rhos - D, p, c)[0]
    return A


class Plan:
    """Index arrays of GENERAL_ERgraph_and_auxialiaryarrays_generation (nb:278-369)
    for a core graph given by its edge list (list(G.edges)) and neighbour lists
    (G.neighbors order); n_total and n_iso include the removed isolated nodes."""

    def __init__(self, edges, nbrs, n_total, n_iso):
        self.edges = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
        self.nbrs = [list(map(int, x)) for x in nbrs]
        self.n_core = len(self.nbrs)
        self.n = int(n_total)
        self.n_iso = int(n_iso)
        E = self.E = self.edges.shape[0]
        row = {}
        for r, (u, v) in enumerate(self.edges.tolist()):
            row[(u, v)] = r
            row[(v, u)] = r + E
        self.deg = np.array([len(x) for x in self.nbrs], dtype=np.int64)
        full = np.concatenate([self.edges, self.edges[:, ::-1]])
        self.edge_class = self.deg[full[:, 0]] - 1           # edges_degree (nb:312-313)
        self.classes = sorted(set(self.edge_class.tolist()))
        self.class_rows, self.class_inc = {}, {}
        for D in self.classes:
            rows = np.flatnonzero(self.edge_class == D)
            self.class_rows[D] = rows
            self.class_inc[D] = np.array([[row[(k, i)] for k in self.nbrs[i] if k != j]
                                          for i, j in full[rows].tolist()], dtype=np.int64).reshape(rows.size, D)
        self.node_classes = sorted(set(self.deg.tolist()))
        self.node_rows, self.node_inc = {}, {}
        for D in self.node_classes:
            nodes = np.flatnonzero(self.deg == D)
            self.node_rows[D] = nodes
            self.node_inc[D] = np.array([[row[(k, i)] for k in self.nbrs[i]] for i in nodes.tolist()],
                                        dtype=np.int64).reshape(nodes.size, D)

    @classmethod
    def from_csr(cls, edges, row_ptr, col, n_total, n_iso):
        rp = np.asarray(row_ptr, dtype=np.int64)
        col = np.asarray(col, dtype=np.int64)
        return cls(edges, [col[rp[i]:rp[i + 1]] for i in range(rp.size - 1)], n_total, n_iso)


def normalize(chi):
    """nb:128-130: divide every row by its sum (no epsilon)."""
    return chi / np.sum(chi, axis=1, keepdims=True)


def _dp(chi3, inc, ok, D, T):
    """LL[e, xa, rho] = sum over neighbour trajectories ending in the attractor of
    prod_m chi^{k_m -> a}(x_km, xa), rho_t = number of +1 among them at time t
    (nb:150-184); zero for xa not ending in the attractor."""
    X = 2 ** T
    b = traj01(T)
    pw = (D + 1) ** np.arange(T - 1, -1, -1)
    off = b @ pw
    S = (D + 1) ** T
    m = inc.shape[0]
    LL = np.zeros((m, X, S))
    if D == 0:
        LL[:, :, 0] = 1.0
    else:
        M = chi3[inc]                                      # (m, D, X(xk), X(xa))
        for k in range(X):
            if ok[k]:
                LL[:, :, off[k]] = M[:, 0, k, :]
        digits = np.array(list(itertools.product(range(D + 1), repeat=T)), dtype=np.int64)
        for Dm in range(1, D):
            L = np.zeros_like(LL)
            for k in range(X):
                if not ok[k]:
                    continue
                src = np.nonzero(np.all(digits + b[k] <= D, axis=1))[0]
                L[:, :, src + off[k]] += LL[:, :, src] * M[:, Dm, k, :][:, :, None]
            LL = L
    LL[:, ~ok, :] = 0.0
    return LL


def weights(T, lmbd_in):
    """exp(-lmbd*(2 x[0] - 1)) per trajectory (nb:191, no 1/n)."""
    return np.exp(-lmbd_in * (2 * traj01(T)[:, 0] - 1))


def bdcm_update_class(chi, plan, D, p, c, attr_value, lmbd_in, damppar, epsilon=0.0):
    """New rows of edge class D: damp*normalize(max(chi2, eps)) + (1-damp)*chi (nb:186-196)."""
    T = p + c
    X = 2 ** T
    ok = (2 * traj01(T) - 1)[:, T - 1] == attr_value
    rows = plan.class_rows[D]
    LL = _dp(chi.reshape(-1, X, X), plan.class_inc[D], ok, D, T)
    chi2 = np.einsum("eaq,abq->eab", LL, factor_A(D, p, c, attr_value)) * weights(T, lmbd_in)[None, :, None]
    chi2 = np.maximum(chi2.reshape(rows.size, X * X), epsilon)
    return damppar * normalize(chi2) + (1 - damppar) * chi[rows]


def BDCM_ER(chi, plan, p, c, attr_value, lmbd_in, damppar, epsilon=0.0):
    """One sweep over the edge classes d' > 0 in ascending order; each class
    reads chi as already overwritten by the earlier classes (nb:133-198)."""
    chi = np.array(chi, dtype=np.float64, copy=True)
    for D in plan.classes:
        if D > 0:
            chi[plan.class_rows[D]] = bdcm_update_class(chi, plan, D, p, c, attr_value, lmbd_in, damppar, epsilon)
    return chi


def leaf_message(p, c, attr_value, lmbd_in):
    """normalize(exp(-lmbd x_i[0]) A(x_i, x_j, rho = 0)) of a leaf edge (nb:404-417), shape (4^T,)."""
    T = p + c
    X = 2 ** T
    tr = 2 * traj01(T) - 1
    row = np.zeros((X, X))
    zero = np.zeros(T, dtype=np.int64)
    for a in range(X):
        if tr[a][T - 1] != attr_value:
            continue
        for b in range(X):
            row[a, b] = np.exp(-lmbd_in * tr[a][0]) * allowed(tr[a], tr[b], zero, p, c)
    row = row.reshape(-1)
    return row / row.sum()


def _pair_products(chi, plan, p, c, attr_value):
    T = p + c
    X = 2 ** T
    E = plan.E
    ok = (2 * traj01(T) - 1)[:, T - 1] == attr_value
    f = chi[:E].reshape(E, X, X)
    bk = chi[E:].reshape(E, X, X).transpose(0, 2, 1)     # chi^{j->i}(x_j, x_i) at [x_i, x_j]
    prod = f * bk
    prod[:, ~ok, :] = 0.0
    prod[:, :, ~ok] = 0.0
    return prod


def Zij(chi, plan, p, c, attr_value, epsilon=0.0):
    """nb:200-209."""
    return np.maximum(_pair_products(chi, plan, p, c, attr_value).sum(axis=(1, 2)), epsilon)


def Zi_ER(chi, plan, p, c, attr_value, lmbd_in, epsilon=0.0):
    """Node partition functions of the core graph (nb:211-276)."""
    T = p + c
    X = 2 ** T
    ok = (2 * traj01(T) - 1)[:, T - 1] == attr_value
    out = np.zeros(plan.n_core)
    w = weights(T, lmbd_in)
    for D in plan.node_classes:
        if D == 0:
            continue
        LL = _dp(chi.reshape(-1, X, X), plan.node_inc[D], ok, D, T)
        out[plan.node_rows[D]] = np.einsum("eaq,aq->e", LL, factor_Ai(D, p, c, attr_value) * w[:, None])
    return np.maximum(out, epsilon)


def phi_BP(chi, plan, p, c, attr_value, lmbd_in, epsilon=0.0):
    """(sum log Zi - sum log Zij - lmbd*n_iso)/n (nb:372-376)."""
    zi = Zi_ER(chi, plan, p, c, attr_value, lmbd_in, epsilon)
    zij = Zij(chi, plan, p, c, attr_value, epsilon)
    with np.errstate(divide="ignore"):
        return (np.sum(np.log(zi)) - np.sum(np.log(zij)) - lmbd_in * plan.n_iso) / plan.n


def avg_m_init(chi, plan, p, c, attr_value, epsilon=0.0):
    """nb:379-392."""
    T = p + c
    s0 = (2 * traj01(T) - 1)[:, 0].astype(np.float64)
    prod = _pair_products(chi, plan, p, c, attr_value)
    du = plan.deg[plan.edges[:, 0]].astype(np.float64)
    dv = plan.deg[plan.edges[:, 1]].astype(np.float64)
    wgt = s0[None, :, None] / du[:, None, None] + s0[None, None, :] / dv[:, None, None]
    m = (wgt * prod).sum(axis=(1, 2))
    z = np.maximum(prod.sum(axis=(1, 2)), epsilon)
    return (np.sum(m / z) + plan.n_iso) / plan.n


def entropy_procedure(chi, plan, p, c, attr_value, lambdas, damppar, eps=1e-6, T_max=1300, epsilon=0.0,
                      stop_ent=-0.05):
    """BDCM_entropy_procedure_GENERAL_ER (nb:394-452) on a copy of chi.  Returns
    (m_init, ent1, ent, counts, iters, chi) with arrays of len(lambdas) (zeros
    past an early stop)."""
    chi = np.array(chi, dtype=np.float64, copy=True)
    L = len(lambdas)
    ent, m_init, ent1 = np.zeros(L), np.zeros(L), np.zeros(L)
    iters = np.zeros(L, dtype=np.int64)
    counts = 0
    for k, lmbd in enumerate(lambdas):
        if 0 in plan.class_rows:
            chi[plan.class_rows[0]] = leaf_message(p, c, attr_value, lmbd)[None, :]
        delta, t = 1.0, 0
        while delta > eps:
            old = chi
            chi = BDCM_ER(chi, plan, p, c, attr_value, lmbd, damppar, epsilon)
            delta = np.abs(chi - old).max()
            t += 1
            if t >= T_max:
                delta = 0
                counts = lmbd
        iters[k] = t
        ent[k] = phi_BP(chi, plan, p, c, attr_value, lmbd, epsilon)
        m_init[k] = avg_m_init(chi, plan, p, c, attr_value, epsilon)
        ent1[k] = ent[k] + lmbd * m_init[k]
        if ent1[k] < stop_ent or counts > 0:
            break
    return m_init, ent1, ent, counts, iters, chi
