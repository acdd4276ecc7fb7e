"""ORACLE (test infrastructure only): numpy float64 restatement of the HPR
edge-message update and its companions in code/HPR_pytorch_RRG.py.

Follows (paths relative to the reference repository):
  trajectory factor A        code/HPR_pytorch_RRG.py:14-39 (atr_condition, traj_condition,
                             attr_fix, A_i_sums)
  column order               code/HPR_pytorch_RRG.py:46-74 (order_gpu / order): column of
                             (x_a, x_b) = sum_k [z_k = -1] 2^(2T-1-k), z = (x_a, x_b)
  row layout                 code/HPR_pytorch_RRG.py:277-285 (row r < E: G.edges[r] = (u, v),
                             message u->v; row r+E: v->u)
  incoming rows              code/HPR_pytorch_RRG.py:81-97 (neib_edg_pos_chi_mat)
  reinforced message         code/HPR_pytorch_RRG.py:120-133 (positions_biases, new_biases_chi)
  HPr_dp                     code/HPR_pytorch_RRG.py:183-218
  marginals_comp             code/HPR_pytorch_RRG.py:147-167
  new_biases_i               code/HPR_pytorch_RRG.py:137-145
  HPr_dp_er, er_classes,     the same update on an Erdos-Renyi graph with the degree taken
  marginals_comp_csr         per message (the "general (ER)" HPR of code/README.md:1, which
                             the repository does not ship): pinned by equality with HPr_dp on
                             d-regular graphs (tests/test_hpr_oracle.py)
The DP is the reference's: per (edge, x_a), a table over count vectors rho
(number of +1 among the incoming neighbours at each time) built one neighbour
at a time, then contracted with A.  Vectorised over edges.
"""
import itertools

import numpy as np


def traj_table(T):
    """(2^T, T) +-1 trajectories in the reference's xi_comb order (index 0 = all +1)."""
    return np.array(list(itertools.product([1, -1], repeat=T)), dtype=np.int64)


def incoming_rows(edges, nbrs):
    """(2E, d-1) row indices of the messages k->a feeding row a->b, and the
    source node of every row (code/HPR_pytorch_RRG.py:81-97, 277-285).
    ``edges`` is list(G.edges) as an (E, 2) array, ``nbrs`` the (n, d)
    neighbour array in G.neighbors order (the reference's N_nodes)."""
    edges = np.asarray(edges, dtype=np.int64)
    nbrs = np.asarray(nbrs, dtype=np.int64)
    E = edges.shape[0]
    d = nbrs.shape[1]
    row = {}
    for r, (u, v) in enumerate(edges.tolist()):
        row[(u, v)] = r
        row[(v, u)] = r + E
    out = np.zeros((2 * E, d - 1), dtype=np.int64)
    src = np.zeros(2 * E, dtype=np.int64)
    for r, (u, v) in enumerate(edges.tolist()):
        for (a, b, rr) in ((u, v, r), (v, u, r + E)):
            src[rr] = a
            out[rr] = [row[(k, a)] for k in nbrs[a].tolist() if k != b]
    return out, src


def edges_pos(edges, nbrs):
    """(n, d) row of i->k_m (the reference's N_edges_pos, code/HPR_pytorch_RRG.py:110-118)."""
    edges = np.asarray(edges, dtype=np.int64)
    E = edges.shape[0]
    row = {}
    for r, (u, v) in enumerate(edges.tolist()):
        row[(u, v)] = r
        row[(v, u)] = r + E
    nbrs = np.asarray(nbrs, dtype=np.int64)
    return np.array([[row[(i, k)] for k in nbrs[i].tolist()] for i in range(nbrs.shape[0])], dtype=np.int64)


def A_factor(T, p, c, d, attr_value):
    """A[xa, xb, rho] (0/1, without the exp weight), rho = count vector of +1
    among the d-1 incoming neighbours, flattened base-d (code/HPR_pytorch_RRG.py:14-39)."""
    X = 2 ** T
    tr = traj_table(T)
    rhos = np.array(list(itertools.product(range(d), repeat=T)), dtype=np.int64)   # base-d, rho[0] most significant
    A = np.zeros((X, X, rhos.shape[0]), dtype=np.float64)
    for ia in range(X):
        xi = tr[ia]
        if xi[p + c - 1] != attr_value:                      # attr_fix (:34-36)
            continue
        sig = (2 * rhos - d + 1)[None, :, :] + tr[:, None, :]   # (xb, rho, t): rho passed as 2*rho-d+1 (:212)
        ok = np.ones(sig.shape[:2], dtype=bool)
        for t in range(p + c - 1):                           # traj_condition (:19-29)
            f = sig[:, :, t]
            ok &= (xi[t + 1] == np.sign(f)) | ((f == 0) & (xi[t + 1] == xi[t]))
        f = sig[:, :, p + c - 1]                             # atr_condition (:14-17)
        ok &= (xi[p] == np.sign(f)) | ((f == 0) & (xi[p] == xi[p + c - 1]))
        A[ia] = ok
    return A


def _chi_new(chi, biases, inr, src, n, d, p, c, attr_value, lmbd_in):
    """Unnormalised chi_new of the rows whose incoming rows are inr (R, d-1):
    the DP over count vectors and the contraction with A (:186-212)."""
    T = p + c
    X = 2 ** T
    R = inr.shape[0]
    tr = traj_table(T)
    plus0 = tr[:, 0] == 1
    # M[e, m, xk, xa] = bias_{k}(xk[0]) * chi[k->a][xk*X + xa]
    cm = chi.reshape(-1, X, X)
    M = cm[inr]                                                # (R, d-1, X(xk), X(xa))
    bs = np.where(plus0[None, :], biases[src][:, 0:1], biases[src][:, 1:2])     # (2E, X)
    M = M * bs[inr][..., None]
    nb = d ** T
    digits = np.array(list(itertools.product(range(d), repeat=T)), dtype=np.int64)
    pw = d ** np.arange(T - 1, -1, -1)
    x01 = (tr == 1).astype(np.int64)                           # +1 -> 1
    LL = np.zeros((R, X, nb), dtype=np.float64)
    if d == 1:                                                 # no incoming message: rho = 0
        LL[:, :, 0] = 1.0
    else:
        for ik in range(X):
            LL[:, :, int(x01[ik] @ pw)] += M[:, 0, ik, :]
    for m in range(1, d - 1):
        L = np.zeros_like(LL)
        for ik in range(X):
            off = int(x01[ik] @ pw)
            # only source states whose digits stay < d after the shift
            valid = np.all(digits + x01[ik] < d, axis=1)
            srcs = np.nonzero(valid)[0]
            L[:, :, srcs + off] += LL[:, :, srcs] * M[:, m, ik, :][:, :, None]
        LL = L
    A = A_factor(T, p, c, d, attr_value)
    w = np.exp(-lmbd_in * tr[:, 0] / n)                        # exp(-lmbd*xi[0]/n)
    new = np.einsum("raq,abq->rab", LL, A) * w[None, :, None]
    return new.reshape(R, X * X)


def HPr_dp(chi, biases, in_rows, src, n, d, p, c, attr_value, lmbd_in, damppar, rows=None):
    """One HPR message update (code/HPR_pytorch_RRG.py:183-218), float64.

    chi (2E, 4^T); biases (n, 2) with column 0 = bias of +1; in_rows (2E, d-1)
    incoming row indices; src (2E,) source node of each row.  ``rows``: compute
    only these output rows (returns len(rows) rows)."""
    chi = np.asarray(chi, dtype=np.float64)
    biases = np.asarray(biases, dtype=np.float64)
    rows = np.arange(chi.shape[0]) if rows is None else np.asarray(rows)
    new = _chi_new(chi, biases, np.asarray(in_rows)[rows], src, n, d, p, c, attr_value, lmbd_in)
    return damppar * new / np.sum(new, axis=1, keepdims=True) + (1 - damppar) * chi[rows]


# ---- the ER ("general") HPR: the same update with a per-message degree --------
def er_classes(edges, row_ptr, col):
    """Messages of an ER graph (no isolated nodes) grouped by D = deg(a) - 1
    for a -> b: list of (D, rows (m,), inc (m, D) rows of k -> a, k != b), the
    source node of every row (2E,), and the CSR out-rows (row of i -> col[j]).
    Row layout of code/HPR_pytorch_RRG.py:277-285."""
    edges = np.asarray(edges, dtype=np.int64)
    rp = np.asarray(row_ptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    E = edges.shape[0]
    row = {}
    for r, (u, v) in enumerate(edges.tolist()):
        row[(u, v)] = r
        row[(v, u)] = r + E
    src = np.concatenate([edges[:, 0], edges[:, 1]])
    dst = np.concatenate([edges[:, 1], edges[:, 0]])
    deg = np.diff(rp)
    D_of = deg[src] - 1
    classes = []
    for D in sorted(set(D_of.tolist())):
        rows = np.flatnonzero(D_of == D)
        inc = np.array([[row[(k, a)] for k in col[rp[a]:rp[a + 1]].tolist() if k != b]
                        for a, b in zip(src[rows].tolist(), dst[rows].tolist())], dtype=np.int64).reshape(rows.size, D)
        classes.append((int(D), rows, inc))
    n = rp.size - 1
    out_rows = np.array([row[(i, k)] for i in range(n) for k in col[rp[i]:rp[i + 1]].tolist()], dtype=np.int64)
    return classes, src, out_rows


def HPr_dp_er(chi, biases, classes, src, n, p, c, attr_value, lmbd_in, damppar):
    """HPr_dp on an ER graph: every degree class D with the factor of d-1 = D
    incoming messages, all from the old chi (Jacobi), float64."""
    chi = np.asarray(chi, dtype=np.float64)
    biases = np.asarray(biases, dtype=np.float64)
    out = np.empty_like(chi)
    for D, rows, inc in classes:
        new = _chi_new(chi, biases, inc, src, n, D + 1, p, c, attr_value, lmbd_in)
        out[rows] = damppar * new / np.sum(new, axis=1, keepdims=True) + (1 - damppar) * chi[rows]
    return out


def marginals_comp_csr(chi, row_ptr, out_rows, p, c, epsilon=1e-15):
    """marginals_comp (code/HPR_pytorch_RRG.py:147-167) with a per-node degree:
    products over the CSR out-rows of every node."""
    T = p + c
    X = 2 ** T
    chi = np.asarray(chi, dtype=np.float64)
    E = chi.shape[0] // 2
    fw = chi[:E].reshape(E, X, X)
    bw = chi[E:].reshape(E, X, X).transpose(0, 2, 1)
    ZZ = fw * bw
    half = X // 2
    zp = np.concatenate([ZZ[:, :half, :].sum(axis=(1, 2)), ZZ[:, :, :half].sum(axis=(1, 2))])
    zm = np.concatenate([ZZ[:, half:, :].sum(axis=(1, 2)), ZZ[:, :, half:].sum(axis=(1, 2))])
    zp = np.maximum(zp, epsilon)
    zm = np.maximum(zm, epsilon)
    s = zp + zm
    zp, zm = zp / s, zm / s
    rp = np.asarray(row_ptr, dtype=np.int64)
    n = rp.size - 1
    mp = np.array([np.prod(zp[out_rows[rp[i]:rp[i + 1]]]) for i in range(n)])
    mm = np.array([np.prod(zm[out_rows[rp[i]:rp[i + 1]]]) for i in range(n)])
    marg = np.stack([mp, mm], axis=1)
    return marg / (marg[:, 0] + marg[:, 1])[:, None]


def marginals_comp(chi, edges_pos, p, c, epsilon=1e-15):
    """Node marginals (code/HPR_pytorch_RRG.py:147-167).  edges_pos (n, d) =
    row of i->k_m (the reference's N_edges_pos)."""
    T = p + c
    X = 2 ** T
    chi = np.asarray(chi, dtype=np.float64)
    E = chi.shape[0] // 2
    fw = chi[:E].reshape(E, X, X)
    bw = chi[E:].reshape(E, X, X).transpose(0, 2, 1)           # chi^{v->u}(x_v, x_u) at [x_u, x_v]
    ZZ = fw * bw
    half = X // 2
    zp = np.concatenate([ZZ[:, :half, :].sum(axis=(1, 2)), ZZ[:, :, :half].sum(axis=(1, 2))])
    zm = np.concatenate([ZZ[:, half:, :].sum(axis=(1, 2)), ZZ[:, :, half:].sum(axis=(1, 2))])
    zp = np.maximum(zp, epsilon)
    zm = np.maximum(zm, epsilon)
    s = zp + zm
    zp, zm = zp / s, zm / s
    marg = np.stack([np.prod(zp[edges_pos], axis=1), np.prod(zm[edges_pos], axis=1)], axis=1)
    return marg / (marg[:, 0] + marg[:, 1])[:, None]


def new_biases_i(biases, pie, gamma, marginals, t, u):
    """Bias refresh with the uniforms ``u`` the reference draws with torch.rand(n)
    (code/HPR_pytorch_RRG.py:137-145).  Returns (biases', s int32)."""
    biases = np.array(biases, dtype=np.float64, copy=True)
    Tm = marginals[:, 1] >= marginals[:, 0]
    nbias = np.where(Tm[:, None], np.array([pie, 1 - pie]), np.array([1 - pie, pie]))
    prob = u < 1 - (1 + t) ** (-gamma)
    biases[prob] = nbias[prob]
    s = biases[:, 0] > biases[:, 1]
    return biases, (2 * s.astype(np.int32) - 1)
