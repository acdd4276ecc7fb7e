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
        for ib in range(X):
            xj = tr[ib]
            for q, rho in enumerate(rhos):
                sig = (2 * rho - d + 1) + xj                  # rho passed as 2*rho-d+1 (:212)
                ok = True
                for t in range(p + c - 1):                    # traj_condition (:19-29)
                    if xi[t + 1] == np.sign(sig[t]):
                        continue
                    if sig[t] == 0 and xi[t + 1] == xi[t]:
                        continue
                    ok = False
                    break
                if ok:                                        # atr_condition (:14-17)
                    s = sig[p + c - 1]
                    ok = (xi[p] == np.sign(s)) or (s == 0 and xi[p] == xi[p + c - 1])
                A[ia, ib, q] = 1.0 if ok else 0.0
    return A


def HPr_dp(chi, biases, in_rows, src, n, d, p, c, attr_value, lmbd_in, damppar, rows=None):
    """One HPR message update (code/HPR_pytorch_RRG.py:183-218), float64.

    chi (2E, 4^T); biases (n, 2) with column 0 = bias of +1; in_rows (2E, d-1)
    incoming row indices; src (2E,) source node of each row.  ``rows``: compute
    only these output rows (returns len(rows) rows)."""
    T = p + c
    X = 2 ** T
    chi = np.asarray(chi, dtype=np.float64)
    biases = np.asarray(biases, dtype=np.float64)
    rows = np.arange(chi.shape[0]) if rows is None else np.asarray(rows)
    R = rows.size
    tr = traj_table(T)
    plus0 = tr[:, 0] == 1
    # M[e, m, xk, xa] = bias_{k}(xk[0]) * chi[k->a][xk*X + xa]
    cm = chi.reshape(-1, X, X)
    inr = np.asarray(in_rows)[rows]
    M = cm[inr]                                                # (R, d-1, X(xk), X(xa))
    bs = np.where(plus0[None, :], biases[src][:, 0:1], biases[src][:, 1:2])     # (2E, X)
    M = M * bs[inr][..., None]
    nb = d ** T
    digits = np.array(list(itertools.product(range(d), repeat=T)), dtype=np.int64)
    pw = d ** np.arange(T - 1, -1, -1)
    x01 = (tr == 1).astype(np.int64)                           # +1 -> 1
    LL = np.zeros((R, X, nb), dtype=np.float64)
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
    new = new.reshape(R, X * X)
    return damppar * new / np.sum(new, axis=1, keepdims=True) + (1 - damppar) * chi[rows]


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
