"""Drop-ins with the reference's exact signatures for code/HPR_pytorch_RRG.py.

``mjx.HPr_dp`` / ``mjx.marginals_comp`` take an ``HPRPlan`` (one object for
the reference's seven auxiliary index arrays).  The functions here take the
reference's own arguments instead, so its script runs unchanged after

    from mjx.drop_in import HPr_dp, marginals_comp, new_biases_i, new_biases_chi

  HPr_dp(chi_mat, chi_col, biases_chi, rho_D1, N_edg_pos_chi_mat, d, p, c,
         attr_value, lmbd_in, damppar) -> (chi_col, chi_mat)
                                          code/HPR_pytorch_RRG.py:183-218
  marginals_comp(chi_mat, pairs, pji, N_edges_pos, epsilon)
                                          code/HPR_pytorch_RRG.py:147-167
  new_biases_i(biases_i, pie, gamma, marginals, t) -> (biases_i, s)
                                          code/HPR_pytorch_RRG.py:137-145
  new_biases_chi(biases_i, pos_biases)    code/HPR_pytorch_RRG.py:128-133
  onestep_majority, s_endstate, m         code/HPR_pytorch_RRG.py:169-180

The module globals the reference's functions read (n, num_edg, T, xi_comb)
follow from the argument shapes: 2E = chi_mat.shape[0], 4^T =
chi_mat.shape[1], n = 2E/d.  ``rho_D1`` (the D = 1 count vectors) and
``pairs``/``pji`` (column permutations) are fixed functions of T and are not
read.  Every call runs the HIP kernels of ``mjx.hpr``; the index plan is built
once per ``N_edg_pos_chi_mat`` / ``N_edges_pos`` array and reused while the
same, unmodified array is passed again.
"""
import math
import weakref

import numpy as np
import torch

from . import _device, _lib
from .dynamics import m, onestep_majority, s_endstate  # noqa: F401  (same signatures as :169-180)
from .hpr import HPRPlan, _code, _weights
from .hpr import new_biases_i as _new_biases_i

__all__ = ["HPr_dp", "marginals_comp", "new_biases_i", "new_biases_chi", "ChiBiases", "onestep_majority",
           "s_endstate", "m", "plan_arrays_from_positions"]


# ---------------------------------------------------------------------------
# index plan from the reference's own arrays
# ---------------------------------------------------------------------------
def plan_arrays_from_positions(N_edg_pos_chi_mat, num_combs):
    """Recover the graph of a message system from the reference's
    N_edg_pos_chi_mat (code/HPR_pytorch_RRG.py:81-97): row r (< E) is the
    message u->v of G.edges[r], row r+E is v->u, and N_edg_pos_chi_mat[r] holds
    num_combs * (row of k->u) for the d-1 neighbours k != v of u.

    The rows leaving u are r itself and the reverses of u's incoming rows, so
    each node is named by the smallest row leaving it.  Returns
    (edges (E, 2), n, d, rep_row (n,)): node ids 0..n-1 in the order of their
    smallest outgoing row, ``rep_row[v]`` = that row.  Raises ValueError when
    the array is not the message system of a d-regular simple graph."""
    P = np.asarray(N_edg_pos_chi_mat, dtype=np.int64)
    if P.ndim != 2 or P.shape[0] % 2 or P.shape[0] == 0:
        raise ValueError(f"N_edg_pos_chi_mat must be (2E, d-1), got {P.shape}")
    nc = int(num_combs)
    if np.any(P % nc) or np.any(P < 0) or np.any(P >= P.shape[0] * nc):
        raise ValueError("N_edg_pos_chi_mat entries must be row * num_combs of rows in [0, 2E)")
    rows_in = P // nc
    E2 = P.shape[0]
    E, d = E2 // 2, P.shape[1] + 1
    r = np.arange(E2, dtype=np.int64)
    rev = np.where(r < E, r + E, r - E)
    out_set = np.concatenate([r[:, None], rev[rows_in]], axis=1)     # the d rows leaving source(r)
    key = out_set.min(axis=1)
    if not np.array_equal(key[out_set], np.repeat(key[:, None], d, axis=1)):
        raise ValueError("N_edg_pos_chi_mat is not the message system of a d-regular graph")
    rep_row, node = np.unique(key, return_inverse=True)
    n = rep_row.size
    if n * d != E2:
        raise ValueError(f"{E} edges and degree {d} do not give a d-regular graph ({n} nodes)")
    edges = np.stack([node[:E], node[E:]], axis=1)
    return edges, n, d, rep_row


class _Cache:
    """Objects derived from an index array, kept while the same unmodified
    array is passed again (numpy: identity + a CRC-32 of all its bytes;
    tensors: identity, storage pointer and version counter)."""

    def __init__(self):
        self._d = {}

    @staticmethod
    def _sig(a):
        if isinstance(a, torch.Tensor):
            return ("t", a.data_ptr(), tuple(a.shape), a._version)
        import zlib
        arr = np.ascontiguousarray(np.asarray(a))
        # every byte: an in-place edit anywhere gives a new plan
        return ("n", tuple(arr.shape), arr.dtype.str, zlib.crc32(memoryview(arr).cast("B")))

    def get(self, a, extra, make):
        k = (id(a), extra)
        sig = self._sig(a)
        hit = self._d.get(k)
        if hit is not None and hit[0]() is a and hit[1] == sig:
            return hit[2]
        val = make()
        try:
            ref = weakref.ref(a, lambda _, kk=k: self._d.pop(kk, None))
        except TypeError:
            return val
        self._d[k] = (ref, sig, val)
        return val


_PLANS = _Cache()
_ROWS = _Cache()
_POSB = _Cache()


def _host(a):
    return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)


class _RefPlan:
    def __init__(self, N_edg_pos_chi_mat, nc):
        edges, n, d, rep_row = plan_arrays_from_positions(_host(N_edg_pos_chi_mat), nc)
        self.plan = HPRPlan(edges, n, d)
        self.rep_row_host = rep_row
        self.rep_row = torch.from_numpy(rep_row).to(self.plan.nbr.device)


# ---------------------------------------------------------------------------
# biases
# ---------------------------------------------------------------------------
class ChiBiases:
    """What new_biases_chi returns here: biases_i and pos_biases, not the
    (2E * 4^T) gathered vector (code/HPR_pytorch_RRG.py:128-133), which
    HPr_dp would only read back per source node.  ``materialize()`` builds the
    reference's vector for a caller that needs it."""

    def __init__(self, biases_i, pos_biases):
        self.biases_i = biases_i
        self.pos_biases = pos_biases

    def materialize(self):
        b = self.biases_i
        flat = torch.vstack((b[:, 0], b[:, 1])).reshape(-1)
        return flat[torch.as_tensor(self.pos_biases, device=b.device).long()]


def new_biases_chi(biases_i, pos_biases):
    """code/HPR_pytorch_RRG.py:128-133 (deferred, see ChiBiases)."""
    return ChiBiases(biases_i, pos_biases)


def _node_biases(biases_chi, rp, nc, dtype):
    """(n, 2) bias pairs in the plan's node numbering (mjx_hpr_node_biases)."""
    plan = rp.plan
    out = torch.empty((plan.n, 2), dtype=dtype, device=plan.nbr.device)
    if isinstance(biases_chi, ChiBiases):
        # node v of the plan is the source of row rep_row[v]; its id in the
        # reference's numbering is pos_biases[rep_row[v] * num_combs] (:120-125)
        def ids():
            pos = _host(biases_chi.pos_biases).reshape(-1)
            if pos.size != 2 * plan.E * nc:
                raise ValueError(f"pos_biases must have {2 * plan.E * nc} entries, got {pos.size}")
            return torch.from_numpy(pos[rp.rep_row_host * nc].astype(np.int64)).to(plan.nbr.device)
        idx = _POSB.get(biases_chi.pos_biases, (id(rp), nc), ids)
        src = _device.to_device(biases_chi.biases_i, dtype=dtype)
        stride, half = 2, 1
    else:
        src = _device.to_device(biases_chi, dtype=dtype).reshape(-1)
        if src.numel() != 2 * plan.E * nc:
            raise ValueError(f"biases_chi must have {2 * plan.E * nc} entries, got {src.numel()}")
        idx, stride, half = rp.rep_row, nc, nc // 2
    _lib.call("mjx_hpr_node_biases", _code(dtype), _device.ptr(src), _device.ptr(idx), stride, half, plan.n,
              _device.ptr(out), _device.stream_handle())
    return out


# ---------------------------------------------------------------------------
# the reference's functions
# ---------------------------------------------------------------------------
def HPr_dp(chi_mat, chi_col, biases_chi, rho_D1, N_edg_pos_chi_mat, d, p, c, attr_value, lmbd_in, damppar):
    """code/HPR_pytorch_RRG.py:183-218 with its arguments; returns
    (chi_col, chi_mat) of the new messages (a new device tensor and its flat
    view, like the reference).  ``chi_col`` and ``rho_D1`` are not read."""
    chi = _device.to_device(chi_mat)
    if chi.dim() != 2:
        raise ValueError("chi_mat must be (2E, 4^(p+c))")
    nc = chi.shape[1]
    if nc != 4 ** (int(p) + int(c)):
        raise ValueError(f"chi_mat has {nc} columns, p={p}, c={c} needs {4 ** (int(p) + int(c))}")
    rp = _PLANS.get(N_edg_pos_chi_mat, nc, lambda: _RefPlan(N_edg_pos_chi_mat, nc))
    plan = rp.plan
    if plan.d != int(d) or chi.shape[0] != 2 * plan.E:
        raise ValueError(f"chi_mat {tuple(chi.shape)} / d={d} do not match N_edg_pos_chi_mat "
                         f"(2E={2 * plan.E}, d={plan.d})")
    b = _node_biases(biases_chi, rp, nc, chi.dtype)
    out = torch.empty_like(chi)
    wp, wm = _weights(lmbd_in, plan.n)
    rc = _lib.load().mjx_hpr_update(_code(chi.dtype), _device.ptr(chi), _device.ptr(out), _device.ptr(b),
                                    _device.ptr(plan.nbr), _device.ptr(plan.in_row), _device.ptr(plan.out_row),
                                    plan.n, plan.d, int(p), int(c), int(attr_value), wp, wm, float(damppar),
                                    _device.stream_handle())
    if rc == _lib.MJX_ERANGE:
        from .hpr_er import HPr_dp_er
        out = HPr_dp_er(chi, b, plan.er_plan, p, c, attr_value, lmbd_in, damppar, out=out)
    else:
        _lib.check(rc, "mjx_hpr_update")
    return out.reshape(-1), out


def marginals_comp(chi_mat, pairs, pji, N_edges_pos, epsilon=1e-15):
    """code/HPR_pytorch_RRG.py:147-167 with its arguments: (n, 2) marginals,
    column 0 = spin +1.  ``N_edges_pos`` (n, d) is the row of every message
    leaving node i, in the reference's node numbering (:110-118)."""
    chi = _device.to_device(chi_mat)
    nc = chi.shape[1]
    T = int(round(math.log(nc, 4)))
    if 4 ** T != nc or T < 2:
        raise ValueError(f"chi_mat must have 4^T columns, T >= 2, got {nc}")
    out_row = _ROWS.get(N_edges_pos, None,
                        lambda: _device.to_device(_host(N_edges_pos).astype(np.int32)).contiguous())
    n, d = out_row.shape
    if n * d != chi.shape[0]:
        raise ValueError(f"N_edges_pos {tuple(out_row.shape)} does not match chi_mat {tuple(chi.shape)}")
    eps = float(epsilon.item()) if isinstance(epsilon, torch.Tensor) else float(epsilon)
    zwork = torch.empty(2 * chi.shape[0], dtype=chi.dtype, device=chi.device)
    marg = torch.empty((n, 2), dtype=chi.dtype, device=chi.device)
    # the kernel reads T = p + c only
    _lib.call("mjx_hpr_marginals", _code(chi.dtype), _device.ptr(chi), _device.ptr(out_row), n, d, T - 1, 1, eps,
              _device.ptr(zwork), _device.ptr(marg), _device.stream_handle())
    return marg


def new_biases_i(biases_i, pie, gamma, marginals, t):
    """code/HPR_pytorch_RRG.py:137-145: updates biases_i in place (a device
    tensor) with the reference's torch.rand(n) draw on the default CPU
    generator; returns (biases_i, s) with s = +-1 int32."""
    return _new_biases_i(biases_i, pie, gamma, marginals, t)
