"""BDCM (backtracking dynamical cavity method) entropy of majority-dynamics
attractors on Erdos-Renyi graphs, backed by HIP kernels
(code/ER_BDCM_entropy.ipynb; "nb:L" = raw JSON line L of the notebook).

Reference-shaped entry points, with the notebook's module globals turned into
explicit arguments:

  BDCMPlan / bdcm_er_plan(n, prob)   GENERAL_ERgraph_and_auxialiaryarrays_generation (nb:278-369)
  BDCM_ER(chi, plan, p, c, attr_value, lmbd_in, damppar, epsilon)     nb:133-198 (in place)
  bdcm_leaf_reset(chi, plan, p, c, attr_value, lmbd_in)              nb:404-417
  Zij(chi, plan, p, c, attr_value, epsilon)                          nb:200-209
  Zi_ER(chi, plan, p, c, attr_value, lmbd_in, epsilon)               nb:211-276
  phi_BP_GENERAL_ER(chi, plan, p, c, attr_value, lmbd_in, epsilon)   nb:372-376
  avg_m_init_GENERAL_ER(chi, plan, p, c, attr_value, epsilon)        nb:379-392
  BDCM_entropy_procedure_GENERAL_ER(chi, plan, lambdas, ...)         nb:394-452
  bdcm_er_run(n, deg, ...)                                           the notebook cell's main loop (nb:455-515)

``chi`` is the notebook's message array in float64, shape (2E, 4^T) or
(2E,) + (2,)*2T, resident on the device and updated in place like the
reference's.  Every update and observable is a libmjx kernel.  The convergence loop
(the reference's ``while(delta>eps)``, nb:422-431) runs on the device: a
batch of sweeps is captured once per lambda as a hipGraph, each sweep gated by
a device stop flag that the sweep's end sets (mjx_bdcm_iter_end), and the host
reads the control block once per batch.
"""

import numpy as np
import torch

from . import _device, _lib
from .graph import csr_from_edges, erdos_renyi_edges, remove_isolated


def _i32(a, dev):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32).reshape(-1))).to(dev)


class BDCMPlan:
    """Device-resident index arrays of an ER core graph (isolated nodes removed,
    nb:283-291) for the BDCM kernels.

    edges: (E, 2) list(G.edges) — fixes the message row order (row r: u -> v,
    row r + E: v -> u).  row_ptr/col: neighbour lists in G.neighbors order
    (any order gives the same messages up to floating-point summation order).
    n_total / n_iso: node count before isolated-node removal and the number
    removed (they enter phi and m_init, nb:376, 392)."""

    def __init__(self, edges, row_ptr, col, n_total=None, n_iso=0):
        e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
        rp = np.asarray(row_ptr, dtype=np.int64)
        cl = np.asarray(col, dtype=np.int64)
        n = rp.size - 1
        E = e.shape[0]
        if n < 1 or cl.size != 2 * E or rp[0] != 0 or rp[-1] != cl.size:
            raise ValueError("CSR must hold both directions of every edge of the edge list")
        deg = np.diff(rp)
        if deg.min() < 1:
            raise ValueError("remove isolated nodes first (nb:283-291) and pass their number as n_iso")
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
        cls = deg[full[:, 0]] - 1                               # edges_degree (nb:312-313)
        dev = _device.require_gpu()
        self.device = dev
        self.n_core, self.E = int(n), int(E)
        self.n_iso = int(n_iso)
        self.n = int(n_total) if n_total is not None else self.n_core + self.n_iso
        self.edges_host, self.deg_host = e, deg
        self.row_ptr_host, self.col_host = rp, cl
        self.edge_classes = []                                  # ascending D: Gauss-Seidel order (nb:138)
        for D in np.unique(cls).tolist():
            rows = np.flatnonzero(cls == D)
            a, b = full[rows, 0], full[rows, 1]
            nb = cl[rp[a][:, None] + np.arange(D + 1)[None, :]]
            keep = nb != b[:, None]
            if not np.all(keep.sum(axis=1) == D):
                raise ValueError("graph is not simple")
            kn = nb[keep].reshape(rows.size, D)
            inc = row_of(kn, np.broadcast_to(a[:, None], kn.shape)) if D else np.zeros(0, np.int64)
            self.edge_classes.append((int(D), _i32(rows, dev), _i32(inc, dev), int(rows.size)))
        self.node_classes = []
        for D in np.unique(deg).tolist():
            nodes = np.flatnonzero(deg == D)
            nb = cl[rp[nodes][:, None] + np.arange(D)[None, :]]
            inc = row_of(nb, np.broadcast_to(nodes[:, None], nb.shape))
            self.node_classes.append((int(D), _i32(nodes, dev), _i32(inc, dev), int(nodes.size)))
        self.edges = _i32(e, dev)
        self.deg = _i32(deg, dev)
        self._work = torch.empty(256, dtype=torch.float64, device=dev)
        self._sums = torch.zeros(4, dtype=torch.float64, device=dev)
        self._delta = torch.zeros(1, dtype=torch.int64, device=dev)
        self._ctl = torch.zeros(4, dtype=torch.int64, device=dev)     # device loop control (mjx_bdcm_iter_*)
        self._w = torch.zeros(2, dtype=torch.float64, device=dev)      # lambda weights of a captured loop
        self._upd = None

    @property
    def classes(self):
        return [D for D, _, _, _ in self.edge_classes]

    SCRATCH_CAP = 256 << 20          # bytes of count tables in flight for the high-degree classes

    def scratch(self, p, c):
        """Global slab for the count tables of the classes beyond the LDS budget
        (None if every class fits); raises MjxError if a class is unsupported."""
        lib = _lib.load()
        need = 0
        for D, _, _, m in list(self.edge_classes) + list(self.node_classes):
            b = lib.mjx_bdcm_scratch_bytes(D, int(p), int(c))
            if b < 0:
                raise _lib.MjxError(f"BDCM class D={D} at p+c={p + c} is unsupported")
            need = max(need, min(b * m, max(b, self.SCRATCH_CAP)))
        key = (int(p), int(c))
        if need and getattr(self, "_scratch_key", None) != key:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
            self._scratch_key = key
            self._drop_graphs()            # a captured loop holds the old slab's address
        return self._scratch if need else None

    def check_sizes(self, p, c):
        """Raise MjxError if some class is unsupported (tables beyond the LDS
        budget run from a global scratch slab)."""
        self.scratch(p, c)

    def upd(self, nc):
        need = max((m for _, _, _, m in self.edge_classes), default=0) * nc
        if self._upd is None or self._upd.numel() < need:
            self._upd = torch.empty(max(need, 1), dtype=torch.float64, device=self.device)
            self._drop_graphs()            # a captured loop holds the old buffer's address
        return self._upd

    def _drop_graphs(self):
        if getattr(self, "_graphs", None):
            self._graphs.clear()

    @classmethod
    def from_networkx(cls, G, n_total=None, n_iso=0):
        """From a networkx graph already relabelled 0..n-1 without isolated nodes."""
        n = G.number_of_nodes()
        rp = np.zeros(n + 1, dtype=np.int64)
        cols = []
        for i in range(n):
            nb = list(G.neighbors(i))
            rp[i + 1] = rp[i] + len(nb)
            cols.extend(nb)
        return cls(np.array(list(G.edges), dtype=np.int64).reshape(-1, 2), rp, np.asarray(cols), n_total, n_iso)


def bdcm_er_plan(n, prob, seed=None):
    """G(n, prob) with isolated nodes removed and relabelled (nb:280-291) as a
    BDCMPlan.  The graph comes from this package's own sampler (geometric
    skipping); its parity with networkx.fast_gnp_random_graph is distributional."""
    u, v = erdos_renyi_edges(int(n), float(prob), seed)
    n2, u2, v2, iso = remove_isolated(int(n), u, v)
    rp, col = csr_from_edges(n2, u2, v2)
    return BDCMPlan(np.stack([u2, v2], axis=1), rp, col, n_total=int(n), n_iso=iso)


def _chi2d(chi, plan, p, c):
    if not (isinstance(chi, torch.Tensor) and chi.is_cuda and chi.dtype == torch.float64 and chi.is_contiguous()):
        raise _lib.MjxError("chi must be a contiguous float64 device tensor (it is updated in place, nb:196-198)")
    nc = 4 ** (int(p) + int(c))
    if chi.numel() != 2 * plan.E * nc:
        raise ValueError(f"chi must hold (2E, 4^T) = ({2 * plan.E}, {nc}) messages, got {tuple(chi.shape)}")
    return chi.view(2 * plan.E, nc)


def _scratch_args(plan, p, c):
    sc = plan.scratch(p, c)
    return (_device.ptr(sc), sc.numel()) if sc is not None else (None, 0)


def _update(ch, plan, D, rows, inc, m, p, c, attr_value, lmbd, damp, eps, delta, gate=None, w_dev=None):
    _lib.call("mjx_bdcm_update_class", _device.ptr(ch), _device.ptr(rows), _device.ptr(inc) if D else None, m, D,
              int(p), int(c), int(attr_value), float(lmbd), float(damp), float(eps),
              _device.ptr(plan.upd(ch.shape[1])), _device.ptr(delta) if delta is not None else None,
              _device.ptr(gate) if gate is not None else None, _device.ptr(w_dev) if w_dev is not None else None,
              *_scratch_args(plan, p, c), _device.stream_handle())


def BDCM_ER(chi, plan, p, c, attr_value, lmbd_in, damppar, epsilon=0.0, delta=None, gate=None, w_dev=None):
    """One BDCM sweep over the edge classes D > 0 in ascending order, each class
    reading chi as already overwritten by the earlier ones (nb:133-198).
    Updates chi in place and returns it.  ``delta`` (int64 device tensor of 1,
    optional): receives max |chi_new - chi_old| as float64 bits (atomic max).
    ``gate`` (int64 device tensor, optional): the sweep does nothing while
    gate[0] != 0 (the stop flag of a captured loop).  ``w_dev`` (float64
    device tensor of 2, optional): {exp(-lmbd), exp(lmbd)} read on the device
    instead of ``lmbd_in``."""
    ch = _chi2d(chi, plan, p, c)
    for (D, rows, inc, m) in plan.edge_classes:
        if D > 0:
            _update(ch, plan, D, rows, inc, m, p, c, attr_value, lmbd_in, damppar, epsilon, delta, gate, w_dev)
    return chi


def _sweep_gated(ch, plan, p, c, attr_value, lmbd, damppar, epsilon, eps, T_max, w_dev=None):
    """One iteration of the device loop: begin, the gated sweep, end."""
    st = _device.stream_handle()
    ctl = plan._ctl
    _lib.call("mjx_bdcm_iter_begin", _device.ptr(ctl), st)
    BDCM_ER(ch, plan, p, c, attr_value, lmbd, damppar, epsilon, delta=ctl[0:1], gate=ctl[1:2], w_dev=w_dev)
    _lib.call("mjx_bdcm_iter_end", _device.ptr(ctl), float(eps), int(T_max), st)


def converge(chi, plan, p, c, attr_value, lmbd_in, damppar, eps, T_max, epsilon=0.0, batch=32, graph=True):
    """BDCM_ER until max|delta chi| <= eps or T_max sweeps (nb:422-431) with the
    loop test on the device: batches of ``batch`` gated sweeps, one host read
    per batch.  ``graph``: the batch is captured once as a hipGraph (kept on the
    plan for the same chi and arguments; lambda is read from device memory, so
    one capture serves the whole lambda sweep) and replayed; else the sweeps
    are launched eagerly.  Returns (t, delta of the last sweep) like the
    reference's loop; chi ends in the state after sweep t exactly (the sweeps
    past the stop are no-ops)."""
    ch = _chi2d(chi, plan, p, c)
    sc = plan.scratch(p, c)
    upd = plan.upd(ch.shape[1])              # every buffer exists before a capture
    ctl = plan._ctl
    ctl.zero_()
    g = None
    w_dev = None
    if graph:
        import math
        w_dev = plan._w
        w_dev.copy_(torch.tensor([math.exp(-lmbd_in), math.exp(lmbd_in)], dtype=torch.float64))
        # every address the capture bakes in is part of the key
        key = (ch.data_ptr(), upd.data_ptr(), sc.data_ptr() if sc is not None else None, int(p), int(c),
               int(attr_value), float(damppar), float(eps), int(T_max), float(epsilon), int(batch))
        cache = getattr(plan, "_graphs", None)
        if cache is None:
            cache = plan._graphs = {}
        g = cache.get(key)
        if g is None:
            # capture on a side stream (torch's rule); replayed on the current one
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(batch):
                    _sweep_gated(ch, plan, p, c, attr_value, lmbd_in, damppar, epsilon, eps, T_max, w_dev)
            cache.clear()                    # one live graph per plan
            cache[key] = g
    while True:
        if graph:
            g.replay()
        else:
            for _ in range(batch):
                _sweep_gated(ch, plan, p, c, attr_value, lmbd_in, damppar, epsilon, eps, T_max)
        h = ctl.cpu()
        if int(h[1]):
            return int(h[2]), float(h[3:4].view(torch.float64)[0])


def bdcm_leaf_reset(chi, plan, p, c, attr_value, lmbd_in):
    """Messages out of leaves (edge class 0) set to normalize(exp(-lmbd x_i[0]) A(x_i, x_j, 0))
    (nb:404-417), undamped."""
    ch = _chi2d(chi, plan, p, c)
    for (D, rows, inc, m) in plan.edge_classes:
        if D == 0:
            _update(ch, plan, 0, rows, inc, m, p, c, attr_value, lmbd_in, 1.0, 0.0, None)
    return chi


def Zij(chi, plan, p, c, attr_value, epsilon=0.0, m_term=None):
    """(E,) edge partition functions max(sum chi^ij chi^ji, eps) (nb:200-209)."""
    ch = _chi2d(chi, plan, p, c)
    z = torch.empty(plan.E, dtype=torch.float64, device=ch.device)
    _lib.call("mjx_bdcm_edge_obs", _device.ptr(ch), _device.ptr(plan.edges), _device.ptr(plan.deg), plan.E,
              int(p), int(c), int(attr_value), float(epsilon), _device.ptr(z),
              _device.ptr(m_term) if m_term is not None else None, _device.stream_handle())
    return z


def Zi_ER(chi, plan, p, c, attr_value, lmbd_in, epsilon=0.0):
    """(n_core,) node partition functions max(Zi, eps) (nb:211-276)."""
    ch = _chi2d(chi, plan, p, c)
    zi = torch.empty(plan.n_core, dtype=torch.float64, device=ch.device)
    for (D, nodes, inc, m) in plan.node_classes:
        _lib.call("mjx_bdcm_node_z", _device.ptr(ch), _device.ptr(nodes), _device.ptr(inc), m, D, int(p), int(c),
                  int(attr_value), float(lmbd_in), float(epsilon), _device.ptr(zi), *_scratch_args(plan, p, c),
                  _device.stream_handle())
    return zi


def _sum(plan, x, take_log, slot):
    _lib.call("mjx_sum_f64", _device.ptr(x), x.numel(), int(take_log), _device.ptr(plan._work),
              _device.ptr(plan._sums[slot:slot + 1]), _device.stream_handle())


def observables(chi, plan, p, c, attr_value, lmbd_in, epsilon=0.0):
    """(phi, m_init) of nb:372-392 with one device->host read."""
    ch = _chi2d(chi, plan, p, c)
    zi = Zi_ER(ch, plan, p, c, attr_value, lmbd_in, epsilon)
    mt = torch.empty(plan.E, dtype=torch.float64, device=ch.device)
    zij = Zij(ch, plan, p, c, attr_value, epsilon, m_term=mt)
    _sum(plan, zi, 1, 0)
    _sum(plan, zij, 1, 1)
    _sum(plan, mt, 0, 2)
    s = plan._sums.cpu().numpy()
    phi = (s[0] - s[1] - lmbd_in * plan.n_iso) / plan.n
    m_init = (s[2] + plan.n_iso) / plan.n
    return float(phi), float(m_init)


def phi_BP_GENERAL_ER(chi, plan, p, c, attr_value, lmbd_in, epsilon=0.0):
    """Free-entropy density (sum log Zi - sum log Zij - lmbd*n_iso)/n (nb:372-376)."""
    return observables(chi, plan, p, c, attr_value, lmbd_in, epsilon)[0]


def avg_m_init_GENERAL_ER(chi, plan, p, c, attr_value, epsilon=0.0):
    """Mean initial magnetisation (nb:379-392)."""
    return observables(chi, plan, p, c, attr_value, 0.0, epsilon)[1]


def BDCM_entropy_procedure_GENERAL_ER(chi, plan, lambdas, T_max=1300, p=1, c=1, attr_value=1, eps=1e-6,
                                      damppar=0.1, epsilon=0.0, stop_ent=-0.05, verbose=False, device_loop=True,
                                      batch=32):
    """The lambda sweep of nb:394-452: per lambda, leaf reset, BDCM_ER until
    max|delta chi| <= eps or T_max iterations (warm start from the previous
    lambda), then phi, m_init and ent1 = phi + lambda*m_init; stops after
    ent1 < stop_ent or a non-converged lambda (the reference's ``counts``).
    ``device_loop``: the convergence loop runs as captured batches with a
    device stop flag (``converge``); False: one host read per sweep.
    Returns dict(m_init, ent1, ent, counts, iters) (zeros past an early stop)."""
    ch = _chi2d(chi, plan, p, c)
    plan.check_sizes(p, c)
    lambdas = np.asarray(lambdas, dtype=np.float64)
    L = lambdas.size
    ent, m_init, ent1 = np.zeros(L), np.zeros(L), np.zeros(L)
    iters = np.zeros(L, dtype=np.int64)
    counts = 0
    dbits = plan._delta
    dval = dbits.view(torch.float64)
    for k, lm in enumerate(lambdas.tolist()):
        bdcm_leaf_reset(ch, plan, p, c, attr_value, lm)
        if device_loop:
            t, _ = converge(ch, plan, p, c, attr_value, lm, damppar, eps, T_max, epsilon, batch=batch)
            if t >= T_max:
                counts = lm
        else:
            delta, t = 1.0, 0
            while delta > eps:
                dbits.zero_()
                BDCM_ER(ch, plan, p, c, attr_value, lm, damppar, epsilon, delta=dbits)
                delta = float(dval.item())
                t += 1
                if t >= T_max:
                    delta = 0
                    counts = lm
        iters[k] = t
        ent[k], m_init[k] = observables(ch, plan, p, c, attr_value, lm, epsilon)
        ent1[k] = ent[k] + lm * m_init[k]
        if verbose:
            print(f"lambda= {lm}  t= {t}  m_init: {m_init[k]} ent: {ent1[k]}", flush=True)
        if ent1[k] < stop_ent:
            break
        if counts > 0:
            break
    return {"m_init": m_init, "ent1": ent1, "ent": ent, "counts": counts, "iters": iters}


def bdcm_er_run(n=1000, deg=(1.0, 1.5, 2.0), num_rep=3, p=1, c=1, eps=1e-6, damppar=0.1, attr_value=1,
                epsilon=0.0, T_max=1300, a=12, dl=0.1, seed=0, verbose=False):
    """The notebook's experiment (nb:455-515) on this package's own ER graphs:
    for every mean degree and replica a fresh G(n, deg/(n-1)) core graph,
    uniform random normalised messages, and the lambda sweep
    linspace(0, a, a/dl + 1).  Returns the arrays of the (commented) np.savez
    of nb:515 with the same keys."""
    deg = np.atleast_1d(np.asarray(deg, dtype=np.float64))
    prob = deg / (n - 1)
    lambdas = np.linspace(0, a, int(a / dl + 1))
    shape = (deg.size, num_rep, lambdas.size)
    out = {k: np.zeros(shape) for k in ("m_init", "ent1", "ent")}
    for k in ("nodes_numbers", "mean_degrees", "max_degrees", "nodes_isolated", "mean_degrees_total"):
        out[k] = np.zeros((deg.size, num_rep))
    rng = np.random.default_rng(seed)
    T = p + c
    for i in range(deg.size):
        for r in range(num_rep):
            plan = bdcm_er_plan(n, prob[i], seed=int(rng.integers(2 ** 63)))
            out["nodes_isolated"][i, r] = plan.n_iso
            out["mean_degrees"][i, r] = plan.deg_host.mean()
            out["mean_degrees_total"][i, r] = 2 * plan.E / n
            out["max_degrees"][i, r] = plan.deg_host.max()
            chi = rng.random((2 * plan.E, 4 ** T))
            chi = torch.from_numpy(chi / chi.sum(axis=1, keepdims=True)).to(plan.device)
            res = BDCM_entropy_procedure_GENERAL_ER(chi, plan, lambdas, T_max=T_max, p=p, c=c, attr_value=attr_value,
                                                    eps=eps, damppar=damppar, epsilon=epsilon, verbose=verbose)
            for k in ("m_init", "ent1", "ent"):
                out[k][i, r] = res[k]
    out.update(deg=deg, prob=prob, T_max=np.array(T_max), num_rep=np.array(num_rep))
    return out
