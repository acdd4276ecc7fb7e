"""Graphs for the majority dynamics: host builders and the device-resident form.

Reference counterparts:
  * ``neighbours(G)`` (code/SA_RRG.py:9-16) and ``N_nodes`` of
    ``neighb_edges_pos_AND_nodes`` (code/HPR_pytorch_RRG.py:110-118): the (n, d)
    adjacency ("ELL") of a random regular graph, row i = ``G.neighbors(i)``.
  * ``GENERAL_ERgraph_and_auxialiaryarrays_generation`` (nb:278-369): an
    Erdos-Renyi graph with isolated nodes removed and relabelled; the dynamics
    use ``N_nodes_pos`` per degree class (nb:359-361), i.e. the neighbour lists.
    Here the same neighbour lists are stored as CSR (row_ptr int64, col int32).

Dynamics depend only on the edge set (the +-1 sum is order free), so any
neighbour order gives bit-identical trajectories.

Graph *generation* in the reference is networkx (third party, seeded through
Python's ``random``).  ``from_networkx`` reproduces the reference's arrays
exactly when networkx is importable; ``random_regular_graph`` and
``erdos_renyi`` are this package's own samplers (configuration model with
double-edge-swap repair; Batagelj-Brandes geometric skipping), whose parity
with networkx is distributional, not bit-exact.
"""
import math

import numpy as np
import torch

from . import _device


# ---------------------------------------------------------------------------
# host builders
# ---------------------------------------------------------------------------
def neighbours(G, n=None, d=None):
    """(n, d) int32 adjacency in ``G.neighbors(i)`` order (code/SA_RRG.py:9-16)."""
    n = G.number_of_nodes() if n is None else n
    if d is None:
        d = max((deg for _, deg in G.degree()), default=0)
    N = np.ones((n, d), dtype=np.int64)  # reference pre-fills with ones
    for i in range(n):
        for count, k in enumerate(G.neighbors(i)):
            N[i, count] = k
    return N.astype(np.int32)


def csr_from_networkx(G):
    """CSR (row_ptr int64, col int32) with row i = list(G.neighbors(i))."""
    n = G.number_of_nodes()
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    cols = []
    for i in range(n):
        nb = list(G.neighbors(i))
        row_ptr[i + 1] = row_ptr[i] + len(nb)
        cols.extend(nb)
    return row_ptr, np.asarray(cols, dtype=np.int32)


def _edge_keys(u, v, n):
    lo = np.minimum(u, v).astype(np.int64)
    hi = np.maximum(u, v).astype(np.int64)
    return lo * n + hi


def random_regular_edges(d, n, seed=None):
    """Simple d-regular graph on n nodes as an (n*d/2, 2) int64 edge array.

    Configuration model (uniform stub pairing) followed by random double-edge
    swaps that remove self-loops and multi-edges while preserving degrees.
    """
    if (n * d) % 2:
        raise ValueError("n * d must be even")  # networkx raises NetworkXError here
    if not 0 <= d < n:
        raise ValueError("the 0 <= d < n inequality must be satisfied")
    rng = np.random.default_rng(seed)
    if d == 0:
        return np.zeros((0, 2), dtype=np.int64)
    stubs = np.repeat(np.arange(n, dtype=np.int64), d)
    rng.shuffle(stubs)
    e = stubs.reshape(-1, 2)
    m = e.shape[0]
    for _ in range(1000):
        keys = _edge_keys(e[:, 0], e[:, 1], n)
        loops = e[:, 0] == e[:, 1]
        order = np.argsort(keys, kind="stable")
        sk = keys[order]
        dup_sorted = np.zeros(m, dtype=bool)
        dup_sorted[1:] = sk[1:] == sk[:-1]
        dup = np.zeros(m, dtype=bool)
        dup[order] = dup_sorted
        bad = np.flatnonzero(loops | dup)
        if bad.size == 0:
            return e
        keyset = set(keys.tolist())
        for idx in bad.tolist():
            u, v = int(e[idx, 0]), int(e[idx, 1])
            for _attempt in range(10000):
                j = int(rng.integers(m))
                if j == idx:
                    continue
                x, y = int(e[j, 0]), int(e[j, 1])
                if rng.random() < 0.5:
                    x, y = y, x
                # (u,v),(x,y) -> (u,x),(v,y)
                if u == x or v == y:
                    continue
                k1 = min(u, x) * n + max(u, x)
                k2 = min(v, y) * n + max(v, y)
                if k1 == k2 or k1 in keyset or k2 in keyset:
                    continue
                keyset.discard(min(u, v) * n + max(u, v))
                keyset.discard(min(x, y) * n + max(x, y))
                keyset.add(k1)
                keyset.add(k2)
                e[idx] = (u, x)
                e[j] = (v, y)
                break
    raise RuntimeError("random_regular_edges: repair did not converge")


def ell_from_edges(n, d, e):
    """(n, d) int32 adjacency of a d-regular edge list."""
    src = np.concatenate([e[:, 0], e[:, 1]])
    dst = np.concatenate([e[:, 1], e[:, 0]])
    order = np.argsort(src, kind="stable")
    adj = dst[order].astype(np.int32).reshape(n, d)
    return adj


def random_regular_graph(d, n, seed=None):
    """(n, d) int32 ELL adjacency of a random simple d-regular graph."""
    return ell_from_edges(n, d, random_regular_edges(d, n, seed))


def csr_from_edges(n, u, v):
    """Undirected edge list -> CSR (row_ptr int64, col int32), rows sorted by neighbour."""
    src = np.concatenate([u, v]).astype(np.int64)
    dst = np.concatenate([v, u]).astype(np.int64)
    keys = src * int(n) + dst
    keys.sort()                      # one int64 sort (radix-friendly) instead of a lexsort
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(keys // n, minlength=n), out=row_ptr[1:])
    return row_ptr, (keys % n).astype(np.int32)


def erdos_renyi_edges(n, p, seed=None, chunk=1 << 22):
    """G(n, p) edges by geometric skipping over the n(n-1)/2 pair index."""
    rng = np.random.default_rng(seed)
    total = n * (n - 1) // 2
    if p <= 0 or n < 2:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    if p >= 1:
        idx = np.arange(total, dtype=np.int64)
    else:
        lp = np.log1p(-p)
        parts = []
        pos = -1
        while True:
            gaps = np.floor(np.log(1.0 - rng.random(chunk)) / lp).astype(np.int64) + 1
            cs = pos + np.cumsum(gaps)
            keep = cs[cs < total]
            parts.append(keep)
            if keep.size < cs.size:
                break
            pos = int(cs[-1])
        idx = np.concatenate(parts)
    # pair index -> (v, w), v > w:  idx = v(v-1)/2 + w
    v = np.floor((1.0 + np.sqrt(1.0 + 8.0 * idx.astype(np.float64))) / 2.0).astype(np.int64)
    v[v * (v - 1) // 2 > idx] -= 1
    v[(v + 1) * v // 2 <= idx] += 1
    w = idx - v * (v - 1) // 2
    return v, w


def remove_isolated(n, u, v):
    """Drop degree-0 nodes and relabel in increasing order (nb:283-291).

    Returns (n_kept, u', v', number_iso)."""
    deg = np.bincount(np.concatenate([u, v]), minlength=n)
    keep = deg > 0
    new_id = np.cumsum(keep) - 1
    return int(keep.sum()), new_id[u], new_id[v], int(n - keep.sum())


def erdos_renyi(n, p, seed=None, drop_isolated=False):
    """CSR of G(n, p).  With ``drop_isolated`` the notebook's relabelled core
    graph is returned together with the isolated-node count."""
    u, v = erdos_renyi_edges(n, p, seed)
    if drop_isolated:
        n2, u2, v2, iso = remove_isolated(n, u, v)
        rp, col = csr_from_edges(n2, u2, v2)
        return rp, col, iso
    return csr_from_edges(n, u, v)


# ---------------------------------------------------------------------------
# device generation (libmjx, mjx_rrg_generate)
# ---------------------------------------------------------------------------
_RRG_WORK_WORDS = 1 + 2 * 65536


def random_regular_rows_device(d, n, seed=0, row_lo=0, row_hi=None):
    """ELL rows [row_lo, row_hi) of a random simple d-regular graph generated on
    the device (int32 tensor of shape (row_hi-row_lo, d)).  Every call with the
    same (d, n, seed) describes the same graph, so ranks of a node-range
    partition each generate only their own rows."""
    from . import _lib
    import ctypes
    if (n * d) % 2:
        raise ValueError("n * d must be even")  # networkx raises NetworkXError here
    if not 0 < d < n:
        raise ValueError("the 0 < d < n inequality must be satisfied")
    row_hi = n if row_hi is None else int(row_hi)
    dev = _device.require_gpu()
    adj = torch.empty((row_hi - row_lo, d), dtype=torch.int32, device=dev)
    work = torch.empty(_RRG_WORK_WORDS, dtype=torch.int64, device=dev)
    nsw = ctypes.c_int64(0)
    _lib.call("mjx_rrg_generate", int(n), int(d), int(seed) & 0xFFFFFFFFFFFFFFFF, int(row_lo), row_hi,
              _device.ptr(adj) if adj.numel() else None, _device.ptr(work), work.numel(), ctypes.byref(nsw),
              _device.stream_handle())
    return adj


def erdos_renyi_device(n, p, seed=0, drop_isolated=False):
    """G(n, p) generated on the device into CSR (mjx_er_generate): the
    notebook's ER graph (code/ER_BDCM_entropy.ipynb nb:278-291) at sizes its
    dense adjacency cannot reach (config C4: n = 1e7, p = 5/(n-1)).
    Distributional parity with networkx; deterministic in (n, p, seed).
    Returns a device ``Graph``; with ``drop_isolated`` also the number of
    isolated nodes removed (the survivors are relabelled in increasing order)."""
    from . import _lib
    import ctypes
    n, p = int(n), float(p)
    if n < 1 or not 0.0 <= p < 1.0:
        raise ValueError("need n >= 1 and 0 <= p < 1")
    dev = _device.require_gpu()
    row_ptr = torch.empty(n + 1, dtype=torch.int64, device=dev)
    work = torch.empty(int(_lib.load().mjx_er_work_bytes(n)), dtype=torch.uint8, device=dev)
    mean = n * (n - 1) * p                       # E[2 * edges]
    cap = int(mean + 12 * math.sqrt(2 * mean + 1) + 64)
    n_out, nnz = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = 0
    for attempt in range(2):
        col = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        rc = _lib.load().mjx_er_generate(n, p, int(seed) & 0xFFFFFFFFFFFFFFFF, int(bool(drop_isolated)),
                                         _device.ptr(row_ptr), _device.ptr(col), cap, ctypes.byref(n_out),
                                         ctypes.byref(nnz), _device.ptr(work), work.numel(), _device.stream_handle())
        if rc == _lib.MJX_ERANGE and nnz.value > cap and attempt == 0:
            cap = int(nnz.value)                 # a (very) unlikely edge count: retry once at its size
            continue
        break
    _lib.check(rc, "mjx_er_generate")            # never build a Graph from a failed generate
    del work
    g = Graph.csr_device(row_ptr[:n_out.value + 1], col[:nnz.value])
    return (g, n - n_out.value) if drop_isolated else g


def random_regular_graph_device(d, n, seed=0):
    """Device-resident ELL ``Graph`` of a random simple d-regular graph (for
    sizes networkx cannot reach, e.g. N = 1e9 at d = 6: 24 GB of int32)."""
    return Graph.ell(random_regular_rows_device(d, n, seed))


def check_ell(graph):
    """(self-loops, repeated entries, asymmetric entries) of a device ELL graph."""
    from . import _lib
    counts = torch.zeros(3, dtype=torch.int64, device=graph.adj.device)
    _lib.call("mjx_graph_check_ell", _device.ptr(graph.adj), graph.n, graph.d, _device.ptr(counts),
              _device.stream_handle())
    return tuple(int(x) for x in counts.cpu())


# ---------------------------------------------------------------------------
# device-resident graph
# ---------------------------------------------------------------------------
class Graph:
    """Adjacency resident in HBM.

    kind == "ell": ``adj`` int32 (n, d) — random regular graphs.
    kind == "csr": ``row_ptr`` int64 (n+1,), ``col`` int32 (nnz,) — any graph.
    """

    def __init__(self, kind, n, d=None, adj=None, row_ptr=None, col=None, order=None):
        self.kind, self.n, self.d = kind, int(n), d
        self.adj, self.row_ptr, self.col = adj, row_ptr, col
        self.order = order          # CSR: nodes sorted by degree (visiting order of the rp sweep)
        # CSR replica-packed sweeps: "class" = degree-class ELL (class_ell), "csr" = row_ptr/col
        self.rp_layout = "class"
        self._class_ell = None

    def class_ell(self):
        """Degree-class ELL of a CSR graph, the notebook's ER layout
        (``nodes_with_d_positions[d]`` / ``N_nodes_pos[d]``, nb:359-361, used by
        ``onestep_majority`` nb:113-117): ``(order, cell, classes)`` where
        ``order`` (device int32) lists the nodes by degree, ``classes`` (host
        int64, rows ``i0, count, D, base``) the runs of one degree, and
        ``cell`` (device int32) row k of a class at ``base + k*D``.  Built once
        (mjx_class_ell_fill), cached."""
        if self._class_ell is None:
            from . import _lib
            if self.kind != "csr":
                raise ValueError("class_ell needs a CSR graph")
            deg = self.row_ptr[1:] - self.row_ptr[:-1]
            degs, cnts = torch.unique_consecutive(deg[self.order.long()], return_counts=True)
            degs, cnts = degs.cpu().numpy().astype(np.int64), cnts.cpu().numpy().astype(np.int64)
            rows, i0, base = [], 0, 0
            for D, c in zip(degs, cnts):
                rows.append((i0, c, D, base))
                i0 += c
                base += -(-(c * D) // 4) * 4          # next class at a multiple of 4 (int4 row loads)
            classes = np.ascontiguousarray(np.array(rows, dtype=np.int64).reshape(-1, 4))
            cell = torch.empty(max(base, 1), dtype=torch.int32, device=self.row_ptr.device)
            _lib.call("mjx_class_ell_fill", _device.ptr(self.row_ptr), _device.ptr(self.col) if self.nnz else None,
                      _device.ptr(self.order), classes.ctypes.data, classes.shape[0], self.n, _device.ptr(cell),
                      _device.stream_handle())
            self._class_ell = (self.order, cell, classes)
        return self._class_ell

    @classmethod
    def ell(cls, adj):
        if isinstance(adj, torch.Tensor) and adj.is_cuda and adj.dtype == torch.int32 and adj.is_contiguous():
            t = adj
        else:
            a = adj.cpu().numpy() if isinstance(adj, torch.Tensor) else np.asarray(adj)
            if a.ndim != 2:
                raise ValueError("ELL adjacency must be (n, d)")
            n = a.shape[0]
            if a.size and (a.min() < 0 or a.max() >= n):
                raise ValueError("adjacency index out of range")
            t = _device.to_device(a.astype(np.int32, copy=False))
        return cls("ell", t.shape[0], d=int(t.shape[1]), adj=t)

    @classmethod
    def csr(cls, row_ptr, col):
        rp = np.asarray(row_ptr.cpu() if isinstance(row_ptr, torch.Tensor) else row_ptr, dtype=np.int64)
        cl = np.asarray(col.cpu() if isinstance(col, torch.Tensor) else col, dtype=np.int32)
        n = rp.shape[0] - 1
        if n < 0 or rp[0] != 0 or rp[-1] != cl.shape[0] or np.any(np.diff(rp) < 0):
            raise ValueError("malformed CSR")
        if cl.size and (cl.min() < 0 or cl.max() >= n):
            raise ValueError("CSR column index out of range")
        if n and int(np.diff(rp).max()) > 255:
            raise ValueError("CSR rows longer than 255 are not supported by the bit-sliced counter")
        order = np.argsort(np.diff(rp), kind="stable").astype(np.int32)
        return cls("csr", n, row_ptr=_device.to_device(rp), col=_device.to_device(cl), order=_device.to_device(order))

    @classmethod
    def csr_device(cls, row_ptr, col):
        """CSR graph from device tensors (no host round trip of the arrays):
        row_ptr int64 (n+1,), col int32 (nnz,)."""
        rp = row_ptr.to(torch.int64).contiguous()
        cl = col.to(torch.int32).contiguous()
        n = rp.shape[0] - 1
        if n < 0:
            raise ValueError("malformed CSR")
        deg = rp[1:] - rp[:-1]
        if n and int(deg.max().item()) > 255:
            raise ValueError("CSR rows longer than 255 are not supported by the bit-sliced counter")
        order = torch.sort(deg, stable=True).indices.to(torch.int32)
        return cls("csr", n, row_ptr=rp, col=cl, order=order)

    @property
    def nnz(self):
        return self.n * self.d if self.kind == "ell" else int(self.col.shape[0])
