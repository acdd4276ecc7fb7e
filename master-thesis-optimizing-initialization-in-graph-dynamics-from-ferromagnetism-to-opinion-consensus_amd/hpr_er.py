"""History-passing reinforcement on Erdos-Renyi graphs — the "general (ER)"
HPR that code/README.md:1 announces (the repository ships only the RRG one).

It is code/HPR_pytorch_RRG.py with the degree taken per message: the message
a -> b carries the trajectory factor of deg(a) - 1 incoming messages
(A_i_sums with d - 1 = deg(a) - 1, :14-39), the reinforced incoming messages
(new_biases_chi, :128-133), normalisation and damping (:215), all messages
from the old chi (Jacobi, like HPr_dp); node marginals multiply over each
node's own edges (:147-167); the trial configuration is checked with the ER
majority dynamics (nb:113-123).  On a d-regular graph every call equals its
RRG counterpart (tests pin this).

  HPRERPlan(edges, row_ptr, col)            index plan (no isolated nodes)
  HPr_dp_er(chi, biases, plan, p, c, ...)   -> mjx_hpr_er_update_class per degree class
  marginals_comp_er(chi, plan, p, c)        -> mjx_hpr_edge_z + mjx_hpr_node_marg_csr
  hpr_er_run(n, prob, p, c, ...)            the experiment loop on a G(n, prob) core graph
"""
import math

import numpy as np
import torch

from . import _device, _lib
from .dynamics import pack, rollout
from .graph import Graph, csr_from_edges, erdos_renyi_edges, remove_isolated
from .hpr import _code, new_biases_i


def _i32(a, dev):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32).reshape(-1))).to(dev)


class HPRERPlan:
    """Device index plan of an ER graph with no isolated nodes.

    edges: (E, 2) list(G.edges) — row r = edges[r] as u -> v, row r + E =
    v -> u (code/HPR_pytorch_RRG.py:277-285).  row_ptr/col: neighbour lists.
    Per degree class D (messages a -> b with deg(a) = D + 1): rows, the D
    incoming rows k -> a (k != b) of each, and their senders k."""

    def __init__(self, edges, row_ptr, col):
        e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
        rp = np.asarray(row_ptr, dtype=np.int64)
        cl = np.asarray(col, dtype=np.int64)
        n = rp.size - 1
        E = e.shape[0]
        if n < 1 or cl.size != 2 * E or rp[0] != 0 or rp[-1] != cl.size:
            raise ValueError("CSR must hold both directions of every edge of the edge list")
        deg = np.diff(rp)
        if deg.min() < 1:
            raise ValueError("remove isolated nodes first (their spins are free of the messages)")
        keys = np.concatenate([e[:, 0] * n + e[:, 1], e[:, 1] * n + e[:, 0]])
        order = np.argsort(keys, kind="stable")
        sk = keys[order]
        if sk.size > 1 and np.any(sk[1:] == sk[:-1]):
            raise ValueError("multi-edge in the edge list")

        def row_of(x, y):
            k = (np.asarray(x) * n + np.asarray(y)).reshape(-1)
            pos = np.minimum(np.searchsorted(sk, k), sk.size - 1)
            if k.size and np.any(sk[pos] != k):
                raise ValueError("neighbour lists inconsistent with the edge list")
            return order[pos]

        full = np.concatenate([e, e[:, ::-1]])
        cls = deg[full[:, 0]] - 1
        dev = _device.require_gpu()
        self.device, self.n, self.E = dev, int(n), int(E)
        self.edges, self.deg_host = e, deg
        self.row_ptr_host, self.col_host = rp, cl
        self.classes = []
        for D in np.unique(cls).tolist():
            rows = np.flatnonzero(cls == D)
            a, b = full[rows, 0], full[rows, 1]
            nb = cl[rp[a][:, None] + np.arange(D + 1)[None, :]]
            keep = nb != b[:, None]
            if not np.all(keep.sum(axis=1) == D):
                raise ValueError("graph is not simple")
            kn = nb[keep].reshape(rows.size, D)
            inc = row_of(kn, np.broadcast_to(a[:, None], kn.shape)) if D else np.zeros(0, np.int64)
            self.classes.append((int(D), _i32(rows, dev), _i32(inc, dev), _i32(kn, dev), int(rows.size)))
        self.out_rows_host = row_of(np.repeat(np.arange(n), deg), cl)
        self.out_ptr = torch.from_numpy(rp).to(dev)
        self.out_rows = _i32(self.out_rows_host, dev)
        self._graph = None

    @classmethod
    def from_csr(cls, row_ptr, col):
        rp = np.asarray(row_ptr, dtype=np.int64)
        cl = np.asarray(col, dtype=np.int64)
        src = np.repeat(np.arange(rp.size - 1), np.diff(rp))
        up = src < cl
        return cls(np.stack([src[up], cl[up]], axis=1), rp, cl)

    @property
    def graph(self):
        """CSR graph for the ER majority-dynamics check (nb:113-123)."""
        if self._graph is None:
            self._graph = Graph.csr(self.row_ptr_host, self.col_host)
        return self._graph

    SCRATCH_CAP = 256 << 20          # bytes of count tables in flight for the high-degree classes

    def scratch(self, dtype, p, c):
        """Global slab for the count tables of classes beyond the LDS budget
        (None if every class fits); raises if a class is unsupported."""
        lib = _lib.load()
        need = 0
        for D, *_, m in self.classes:
            b = lib.mjx_hpr_er_scratch_bytes(_code(dtype), D, int(p), int(c))
            if b < 0:
                raise _lib.MjxError(f"ER-HPR class D={D} at p+c={p + c} is unsupported")
            need = max(need, min(b * m, max(b, self.SCRATCH_CAP)))
        key = (dtype, int(p), int(c))
        if need and getattr(self, "_scratch_key", None) != key:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
            self._scratch_key = key
        return self._scratch if need else None

    def check_sizes(self, dtype, p, c):
        self.scratch(dtype, p, c)


def HPr_dp_er(chi_mat, biases_i, plan, p, c, attr_value, lmbd_in, damppar, out=None):
    """One ER-HPR message update; returns the new (2E, 4^T) message matrix."""
    chi = _device.to_device(chi_mat)
    dt = chi.dtype
    nc = 4 ** (int(p) + int(c))
    if chi.shape != (2 * plan.E, nc):
        raise ValueError(f"chi_mat must be ({2 * plan.E}, {nc}), got {tuple(chi.shape)}")
    b = _device.to_device(biases_i, dtype=dt)
    out = torch.empty_like(chi) if out is None else out
    wp, wm = math.exp(-lmbd_in * 1 / plan.n), math.exp(-lmbd_in * -1 / plan.n)   # exp(-lmbd*xi[0]/n) (:39)
    st = _device.stream_handle()
    sc = plan.scratch(dt, p, c)
    for D, rows, inc, src, m in plan.classes:
        _lib.call("mjx_hpr_er_update_class", _code(dt), _device.ptr(chi), _device.ptr(out), _device.ptr(b),
                  _device.ptr(rows), _device.ptr(inc) if D else None, _device.ptr(src) if D else None, m, D,
                  int(p), int(c), int(attr_value), wp, wm, float(damppar), _device.ptr(sc) if sc is not None else None,
                  sc.numel() if sc is not None else 0, st)
    return out


def marginals_comp_er(chi_mat, plan, p, c, epsilon=1e-15, zwork=None, out=None):
    """(n, 2) node marginals, column 0 = spin +1 (:147-167, per-node degree)."""
    chi = _device.to_device(chi_mat)
    dt = chi.dtype
    zwork = torch.empty(4 * plan.E, dtype=dt, device=chi.device) if zwork is None else zwork
    out = torch.empty((plan.n, 2), dtype=dt, device=chi.device) if out is None else out
    st = _device.stream_handle()
    _lib.call("mjx_hpr_edge_z", _code(dt), _device.ptr(chi), plan.E, int(p), int(c), float(epsilon),
              _device.ptr(zwork), st)
    _lib.call("mjx_hpr_node_marg_csr", _code(dt), _device.ptr(zwork), plan.E, _device.ptr(plan.out_ptr),
              _device.ptr(plan.out_rows), plan.n, _device.ptr(out), st)
    return out


def hpr_er_plan(n, prob, seed=None):
    """G(n, prob) with isolated nodes removed and relabelled (as the notebook
    builds its ER graphs, nb:280-291) as an HPRERPlan; also the number of
    isolated nodes removed."""
    u, v = erdos_renyi_edges(int(n), float(prob), seed)
    n2, u2, v2, iso = remove_isolated(int(n), u, v)
    rp, col = csr_from_edges(n2, u2, v2)
    return HPRERPlan(np.stack([u2, v2], axis=1), rp, col), iso


def hpr_er_run(n=None, prob=None, p=1, c=1, damppar=0.4, attr_value=1, lmbd_in=None, pie=0.3, gamma=0.1, TT=10000,
               plan=None, seed=0, dtype=torch.float32, chi0=None, biases0=None, generator=None):
    """The HPR experiment (code/HPR_pytorch_RRG.py:224-377) on an ER core graph:
    random normalised messages and biases from the torch CPU generator,
    then new_biases_chi -> HPr_dp_er -> marginals_comp_er -> new_biases_i
    until the ER majority dynamics of the trial configuration reach consensus
    (m = 1, nb:113-126) or t > TT.  Returns the np.savez keys of :377 over the
    core graph's nodes (mag_reached, conf, num_steps) plus its CSR."""
    if plan is None:
        plan, _ = hpr_er_plan(n, prob, seed=seed)
    plan.check_sizes(dtype, p, c)
    nn = plan.n
    if generator is None:
        generator = torch.Generator().manual_seed(int(seed))
    nc = 4 ** (p + c)
    if chi0 is None:
        chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, generator=generator)
        chi0 = chi0 / torch.sum(chi0, axis=1, keepdims=True)
    if biases0 is None:
        biases0 = torch.rand((nn, 2), dtype=torch.float64, generator=generator)
        biases0 = biases0 / torch.sum(biases0, axis=1, keepdims=True)
    lmbd = 25 * nn if lmbd_in is None else lmbd_in
    chi = _device.to_device(chi0, dtype=dtype)
    chi_b = torch.empty_like(chi)
    biases = _device.to_device(biases0, dtype=dtype).clone()
    dev = chi.device
    zwork = torch.empty(4 * plan.E, dtype=dtype, device=dev)
    marg = torch.empty((nn, 2), dtype=dtype, device=dev)
    s = torch.empty(nn, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    T = p + c - 1

    def sum_end():
        cnt.zero_()
        bits = pack(s)
        if T:
            rollout(plan.graph, bits, T, counts=cnt)
        else:
            _lib.call("mjx_popcount_np", _device.ptr(bits), nn, _device.ptr(cnt), _device.stream_handle())
        return 2 * int(cnt.item()) - nn

    # s from the initial biases: s_i = +1 iff b_i(+1) > b_i(-1) (:337-338)
    s.copy_(torch.where(biases[:, 0] > biases[:, 1], 1, -1).to(torch.int32))
    m_final = sum_end() / nn
    t = 0
    while m_final < 1:                                          # :344-356
        HPr_dp_er(chi, biases, plan, p, c, attr_value, lmbd, damppar, out=chi_b)
        chi, chi_b = chi_b, chi
        marginals_comp_er(chi, plan, p, c, zwork=zwork, out=marg)
        new_biases_i(biases, pie, gamma, marg, t, generator=generator, s_out=s)
        t += 1
        if t > TT:
            m_final = 2
        else:
            m_final = sum_end() / nn
    sh = s.cpu().numpy()
    return {"mag_reached": np.array([np.sum(sh) / nn]), "num_steps": np.array([float(t)]),
            "conf": sh[None, :].astype(np.float64), "row_ptr": plan.row_ptr_host, "col": plan.col_host}
