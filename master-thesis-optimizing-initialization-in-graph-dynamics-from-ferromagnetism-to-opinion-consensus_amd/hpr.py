"""History-passing reinforcement (HPR) on random regular graphs, backed by HIP
kernels (code/HPR_pytorch_RRG.py).

Reference-shaped entry points (same names, argument meaning and layouts):

  HPr_dp(chi_mat, biases_i, plan, p, c, attr_value, lmbd_in, damppar)
                                  code/HPR_pytorch_RRG.py:183-218 (+ new_biases_chi :128-133)
  marginals_comp(chi_mat, plan, p, c, epsilon=1e-15)
                                  code/HPR_pytorch_RRG.py:147-167
  new_biases_i(biases_i, pie, gamma, marginals, t, u=None)
                                  code/HPR_pytorch_RRG.py:137-145
  hpr_run(d, n, p, c, ...)        the experiment loop code/HPR_pytorch_RRG.py:224-377

``chi_mat`` is the reference's (2E, 4^(p+c)) message matrix in its own row and
column order (row r < E: G.edges[r] = (u, v) as u->v, row r+E: v->u); it is
kept on the device.  ``plan`` (``HPRPlan``) replaces the reference's auxiliary
index arrays (edge_dict, N_edg_pos_chi_mat, N_edges_pos, N_nodes, pos_biases,
pairs, pji): they are all functions of the edge list and neighbour order.

Precision: ``dtype=torch.float32`` is the fast path (north star: fp32 edge
messages, 1e-5 row-normalised tolerance per step); ``torch.float64`` runs the
same kernels in the reference's default dtype (code/HPR_pytorch_RRG.py:11).
"""
import math

import numpy as np
import torch

from . import _device, _lib
from .dynamics import pack, rollout
from .graph import Graph

_DT = {torch.float32: _lib.MJX_F32, torch.float64: _lib.MJX_F64}


def _code(dtype):
    try:
        return _DT[dtype]
    except KeyError:
        raise _lib.MjxError(f"HPR messages must be float32 or float64, got {dtype}") from None


class HPRPlan:
    """Device-resident index plan of a d-regular graph for the HPR kernels.

    edges: (E, 2) list(G.edges) — fixes the message row order.
    nbrs:  (n, d) neighbours of each node in G.neighbors order (the reference's
           N_nodes, code/HPR_pytorch_RRG.py:110-118); optional, any order gives
           the same messages up to floating-point summation order.
    """

    def __init__(self, edges, n, d, nbrs=None):
        e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
        n, d = int(n), int(d)
        E = e.shape[0]
        if 2 * E != n * d:
            raise ValueError(f"{E} edges is not a {d}-regular graph on {n} nodes")
        u, v = e[:, 0], e[:, 1]
        if nbrs is None:
            src = np.concatenate([u, v])
            dst = np.concatenate([v, u])
            order = np.lexsort((dst, src))
            nbrs = dst[order].reshape(n, d)
            if not np.array_equal(src[order], np.repeat(np.arange(n), d)):
                raise ValueError("graph is not d-regular")
        nbrs = np.asarray(nbrs, dtype=np.int64).reshape(n, d)
        # row of the directed message x -> y: r for (u_r, v_r), r + E for (v_r, u_r)
        keys = np.concatenate([u * n + v, v * n + u])
        rows = np.concatenate([np.arange(E), np.arange(E) + E])
        srt = np.argsort(keys, kind="stable")
        keys, rows = keys[srt], rows[srt]

        def row_of(x, y):
            k = x * n + y
            pos = np.searchsorted(keys, k)
            if np.any(pos >= keys.size) or np.any(keys[np.minimum(pos, keys.size - 1)] != k):
                raise ValueError("neighbour array inconsistent with the edge list")
            return rows[pos]

        a = np.repeat(np.arange(n, dtype=np.int64), d)
        k = nbrs.reshape(-1)
        self.n, self.d, self.E = n, d, E
        self.edges = e
        self.nbrs_host = nbrs
        self.out_row_host = row_of(a, k).reshape(n, d)      # N_edges_pos (:110-118)
        self.in_row_host = row_of(k, a).reshape(n, d)
        dev = _device.require_gpu()
        self.nbr = torch.from_numpy(nbrs.astype(np.int32).reshape(-1)).to(dev)
        self.in_row = torch.from_numpy(self.in_row_host.astype(np.int32).reshape(-1)).to(dev)
        self.out_row = torch.from_numpy(self.out_row_host.astype(np.int32).reshape(-1)).to(dev)
        self._graph = None

    @classmethod
    def from_networkx(cls, G):
        n = G.number_of_nodes()
        d = max(deg for _, deg in G.degree())
        nbrs = np.array([list(G.neighbors(i)) for i in range(n)], dtype=np.int64)
        return cls(np.array(list(G.edges), dtype=np.int64), n, d, nbrs)

    @property
    def er_plan(self):
        """The same graph as a one-class HPRERPlan (the general kernel's form)."""
        if getattr(self, "_er_plan", None) is None:
            from .hpr_er import HPRERPlan
            rp = np.arange(self.n + 1, dtype=np.int64) * self.d
            self._er_plan = HPRERPlan(self.edges, rp, self.nbrs_host.reshape(-1))
        return self._er_plan

    @property
    def graph(self):
        """ELL graph for the majority-dynamics check (the reference's N_nodes)."""
        if self._graph is None:
            self._graph = Graph.ell(self.nbr.view(self.n, self.d))
        return self._graph

    def num_combs(self, p, c):
        return 4 ** (int(p) + int(c))


def _weights(lmbd_in, n):
    # torch.exp(-lmbd_in*xi[0]/n) with xi[0] = +1 / -1 (code/HPR_pytorch_RRG.py:39)
    return math.exp(-lmbd_in * 1 / n), math.exp(-lmbd_in * -1 / n)


def HPr_dp(chi_mat, biases_i, plan, p, c, attr_value, lmbd_in, damppar, out=None):
    """One HPR message update; returns the new (2E, 4^T) message matrix."""
    chi = _device.to_device(chi_mat)
    dt = chi.dtype
    nc = plan.num_combs(p, c)
    if chi.shape != (2 * plan.E, nc):
        raise ValueError(f"chi_mat must be ({2 * plan.E}, {nc}), got {tuple(chi.shape)}")
    b = _device.to_device(biases_i, dtype=dt)
    out = torch.empty_like(chi) if out is None else out
    wp, wm = _weights(lmbd_in, plan.n)
    rc = _lib.load().mjx_hpr_update(_code(dt), _device.ptr(chi), _device.ptr(out), _device.ptr(b),
                                    _device.ptr(plan.nbr), _device.ptr(plan.in_row), _device.ptr(plan.out_row),
                                    plan.n, plan.d, int(p), int(c), int(attr_value), wp, wm, float(damppar),
                                    _device.stream_handle())
    if rc == _lib.MJX_ERANGE:
        # beyond the register kernels (d > 6, or (d-1)^T count tables above 128
        # entries): the per-degree-class kernel, one class D = d-1
        from .hpr_er import HPr_dp_er
        return HPr_dp_er(chi, b, plan.er_plan, p, c, attr_value, lmbd_in, damppar, out=out)
    _lib.check(rc, "mjx_hpr_update")
    return out


def marginals_comp(chi_mat, plan, p, c, epsilon=1e-15, zwork=None, out=None):
    """(n, 2) node marginals, column 0 = spin +1."""
    chi = _device.to_device(chi_mat)
    dt = chi.dtype
    zwork = torch.empty(4 * plan.E, dtype=dt, device=chi.device) if zwork is None else zwork
    out = torch.empty((plan.n, 2), dtype=dt, device=chi.device) if out is None else out
    _lib.call("mjx_hpr_marginals", _code(dt), _device.ptr(chi), _device.ptr(plan.out_row), plan.n, plan.d,
              int(p), int(c), float(epsilon), _device.ptr(zwork), _device.ptr(out), _device.stream_handle())
    return out


def new_biases_i(biases_i, pie, gamma, marginals, t, u=None, generator=None, s_out=None):
    """Bias refresh (updates ``biases_i`` in place, like the reference) and the
    new trial configuration s (int32 +-1).  ``u``: the n uniforms the reference
    draws with torch.rand(n) on the CPU generator; drawn that way if None."""
    b = biases_i
    if not (isinstance(b, torch.Tensor) and b.is_cuda):
        raise _lib.MjxError("biases_i must be a device tensor (it is updated in place)")
    n = b.shape[0]
    if u is None:
        u = torch.rand(n, dtype=torch.float64, generator=generator)
    u = _device.to_device(u, dtype=torch.float64)
    s = torch.empty(n, dtype=torch.int32, device=b.device) if s_out is None else s_out
    thresh = 1 - (1 + t) ** (-gamma)                       # code/HPR_pytorch_RRG.py:142
    _lib.call("mjx_hpr_new_biases", _code(b.dtype), _device.ptr(b), _device.ptr(marginals), _device.ptr(u),
              float(thresh), float(pie), n, _device.ptr(s), _device.stream_handle())
    return b, s


class HPRState:
    """Device buffers of one HPR run; ``step`` is one iteration of the main loop
    (code/HPR_pytorch_RRG.py:345-356) and returns sum(s_endstate(s)).

    ``layout``: "ref" keeps the messages in the reference's (2E, 4^T) layout;
    "q" (the default where the library has it: fp32, p+c = 4, d <= 4) keeps
    them in the decay-split layout (mjx_hpr_impl.h): the entries with an
    invalid sender trajectory, which HPr_dp only damps ((1-damp)^t chi_0,
    :215), stay undecayed and are read with the scale, so an update moves 1.5
    instead of 3 KB per message.  ``messages()`` returns the reference layout
    either way."""

    def __init__(self, plan, p, c, chi0, biases0, dtype=torch.float32, damppar=0.4, attr_value=1,
                 lmbd_in=None, pie=0.3, gamma=0.1, layout=None):
        self.plan, self.p, self.c = plan, int(p), int(c)
        self.dtype = dtype
        self.damppar, self.attr_value = float(damppar), int(attr_value)
        self.lmbd_in = 25 * plan.n if lmbd_in is None else lmbd_in
        self.pie, self.gamma = float(pie), float(gamma)
        q_ok = _lib.load().mjx_hpr_q_supported(_code(dtype), plan.d, self.p, self.c) == 1
        if layout is None:
            layout = "q" if q_ok else "ref"
        if layout not in ("q", "ref") or (layout == "q" and not q_ok):
            raise _lib.MjxError(f"HPR state layout {layout!r} not available for dtype={dtype}, d={plan.d}, "
                                f"p={p}, c={c}")
        self.layout = layout
        chi0 = _device.to_device(chi0, dtype=dtype)
        if layout == "q":
            self.chi = torch.empty_like(chi0)
            _lib.call("mjx_hpr_qlayout", _code(dtype), _device.ptr(chi0), _device.ptr(self.chi), chi0.shape[0],
                      self.p, self.c, self.attr_value, 1, 1.0, _device.stream_handle())
            self.chi_b = self.chi.clone()        # both buffers carry chi_0's invalid-sender quadrants
            self._sc = torch.ones(2, dtype=dtype, device=chi0.device)
            # the II x II sums never change: once, so the marginals skip the II quadrants
            self._ii = torch.empty(4 * plan.E, dtype=dtype, device=chi0.device)
            _lib.call("mjx_hpr_q_ii", _code(dtype), _device.ptr(self.chi), plan.E, self.p, self.c,
                      _device.ptr(self._ii), _device.stream_handle())
        else:
            self.chi = chi0
            self.chi_b = torch.empty_like(self.chi)
        self.biases = _device.to_device(biases0, dtype=dtype).clone()
        dev = self.chi.device
        self.zwork = torch.empty(4 * plan.E, dtype=dtype, device=dev)
        self.marg = torch.empty((plan.n, 2), dtype=dtype, device=dev)
        self.s = torch.empty(plan.n, dtype=torch.int32, device=dev)
        self.cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        self.t = 0
        self._t0 = 0

    def s_from_biases(self):
        """s = 2*(b0 > b1) - 1 (code/HPR_pytorch_RRG.py:337-338): the bias kernel
        with no node selected for refresh (threshold below every uniform)."""
        u = torch.zeros(self.plan.n, dtype=torch.float64, device=self.s.device)
        _lib.call("mjx_hpr_new_biases", _code(self.dtype), _device.ptr(self.biases), _device.ptr(self.marg),
                  _device.ptr(u), -1.0, self.pie, self.plan.n, _device.ptr(self.s), _device.stream_handle())
        return self.s

    def sum_end(self, s=None):
        """sum(s_endstate(N_nodes, s, p, c)) via the majority rollout kernel."""
        s = self.s if s is None else s
        bits = pack(s)
        self.cnt.zero_()
        rollout(self.plan.graph, bits, self.p + self.c - 1, counts=self.cnt)
        return 2 * int(self.cnt.item()) - self.plan.n

    def decay(self, t):
        """(1-damp)^(t - t0): the scale of the invalid-sender quadrants after
        iteration t (t0 = the iteration the state was built at)."""
        return (1.0 - self.damppar) ** (t - self._t0)

    def messages(self):
        """The current messages in the reference's (2E, 4^T) layout."""
        if self.layout == "ref":
            return self.chi
        out = torch.empty_like(self.chi)
        _lib.call("mjx_hpr_qlayout", _code(self.dtype), _device.ptr(self.chi), _device.ptr(out), self.chi.shape[0],
                  self.p, self.c, self.attr_value, 0, self.decay(self.t), _device.stream_handle())
        return out

    def _update(self, src, dst, sc_in=None, sc_out=None, node=True):
        """HPr_dp src -> dst and marginals_comp(dst) (scales: device pointers,
        decay-split layout; ``node=False``: only the edge Z sums of the
        marginals, the node part left to mjx_hpr_node_step)."""
        st = _device.stream_handle()
        if self.layout == "q":
            plan = self.plan
            wp, wm = _weights(self.lmbd_in, plan.n)
            _lib.call("mjx_hpr_update_q", _code(self.dtype), _device.ptr(src), _device.ptr(dst),
                      _device.ptr(self.biases), _device.ptr(plan.nbr), _device.ptr(plan.in_row),
                      _device.ptr(plan.out_row), plan.n, plan.d, self.p, self.c, self.attr_value, wp, wm,
                      self.damppar, sc_in, st)
            _lib.call("mjx_hpr_marginals_q", _code(self.dtype), _device.ptr(dst), _device.ptr(plan.out_row), plan.n,
                      plan.d, self.p, self.c, 1e-15, sc_out, _device.ptr(self._ii), _device.ptr(self.zwork),
                      _device.ptr(self.marg) if node else None, st)
        else:
            HPr_dp(src, self.biases, self.plan, self.p, self.c, self.attr_value, self.lmbd_in, self.damppar, out=dst)
            marginals_comp(dst, self.plan, self.p, self.c, zwork=self.zwork, out=self.marg)

    def step(self, u=None, generator=None):
        if self.layout == "q":
            self._sc.copy_(torch.tensor([self.decay(self.t), self.decay(self.t + 1)], dtype=self.dtype))
            self._update(self.chi, self.chi_b, self._sc.data_ptr(), self._sc.data_ptr() + self._sc.element_size())
        else:
            self._update(self.chi, self.chi_b)
        self.chi, self.chi_b = self.chi_b, self.chi
        self._graph = None                   # a captured batch holds the old buffer roles
        new_biases_i(self.biases, self.pie, self.gamma, self.marg, self.t, u=u, generator=generator, s_out=self.s)
        self.t += 1
        return self.sum_end()

    # -- batches of the main loop on the device ----------------------------------
    def _batch_buffers(self, k):
        if getattr(self, "_bk", None) != k:
            n, dev = self.plan.n, self.s.device
            self._bk = k
            self._mask = torch.empty((k, n), dtype=torch.bool, device=dev)
            # host staging, double-buffered: batch i+1 is drawn while batch i runs
            self._pin = [(torch.empty((k, n), dtype=torch.bool).pin_memory(),
                          torch.empty(k + 1, dtype=self.dtype).pin_memory()) for _ in range(2)]
            self._pin_i = 0
            self._sums_host = torch.empty(k, dtype=torch.int64).pin_memory()
            self._done = torch.cuda.Event()
            self._s_hist = torch.empty((k, n), dtype=torch.int32, device=dev)
            self._cnt = torch.zeros(k, dtype=torch.int64, device=dev)
            self._scales = torch.ones(k + 1, dtype=self.dtype, device=dev)
            self._bits = torch.empty((n + 63) // 64, dtype=torch.int64, device=dev)
            self._rtmp = (torch.empty_like(self._bits), torch.empty_like(self._bits))
            self._graph = None

    def _batch_launches(self, k):
        """The launches of k iterations (code/HPR_pytorch_RRG.py:345-356) on the
        current stream, every argument fixed: iteration j reads the messages from
        buffer j % 2 and writes the other (k even: the batch ends where it
        started); its refresh decisions are row j of self._mask (the uniforms
        already compared with the reinforcement threshold on the host, see
        draw_batch), its trial configuration goes to row j of self._s_hist and
        sum(s_endstate(s)) to self._cnt[j]."""
        n, T, st = self.plan.n, self.p + self.c - 1, _device.stream_handle()
        self._cnt.zero_()
        sz = self._scales.element_size()
        q = self.layout == "q" and getattr(self, "fuse_node", True)
        for j in range(k):
            src, dst = (self.chi, self.chi_b) if j % 2 == 0 else (self.chi_b, self.chi)
            # decay-split layout: row j of self._scales is (1-damp)^(t+j), set before each replay
            self._update(src, dst, self._scales.data_ptr() + j * sz, self._scales.data_ptr() + (j + 1) * sz, node=not q)
            if q:
                # node marginals, new_biases_i and the packed trial configuration in one launch
                _lib.call("mjx_hpr_node_step", _code(self.dtype), _device.ptr(self.zwork), _device.ptr(self.plan.out_row),
                          n, self.plan.d, _device.ptr(self.marg), _device.ptr(self.biases), _device.ptr(self._mask[j]),
                          self.pie, _device.ptr(self._s_hist[j]), _device.ptr(self._bits), st)
            else:
                _lib.call("mjx_hpr_new_biases_mask", _code(self.dtype), _device.ptr(self.biases), _device.ptr(self.marg),
                          _device.ptr(self._mask[j]), self.pie, n, _device.ptr(self._s_hist[j]), st)
                _lib.call("mjx_pack_np", _device.ptr(self._s_hist[j]), _lib.MJX_I32, n, _device.ptr(self._bits), st)
            if T:
                rollout(self.plan.graph, self._bits, T, out=self._rtmp[0], tmp=self._rtmp[1],
                        counts=self._cnt[j:j + 1])
            else:
                _lib.call("mjx_popcount_np", _device.ptr(self._bits), n, _device.ptr(self._cnt[j:j + 1]), st)

    def draw_batch(self, k, generator, t0=None):
        """Host half of a batch of k iterations starting at iteration t0 (default
        self.t): the k uniform vectors drawn from the CPU generator in the
        reference's order (one torch.rand(n) per iteration, :142) and compared
        with each iteration's threshold 1-(1+t)^-gamma (the float64 comparison
        the reference makes) into pinned refresh masks.  Returns a handle for
        launch_batch holding the generator state before the draws."""
        if k % 2:
            raise ValueError("batch size must be even (the message buffers alternate)")
        self._batch_buffers(k)
        t0 = self.t if t0 is None else t0
        n = self.plan.n
        mask, scales = self._pin[self._pin_i]
        self._pin_i ^= 1
        g_state = generator.get_state()
        for j in range(k):
            u = torch.rand(n, dtype=torch.float64, generator=generator)
            torch.lt(u, 1 - (1 + (t0 + j)) ** (-self.gamma), out=mask[j])     # code/HPR_pytorch_RRG.py:142
        if self.layout == "q":
            scales.copy_(torch.tensor([self.decay(t0 + j) for j in range(k + 1)], dtype=self.dtype))
        return {"k": k, "t0": t0, "mask": mask, "scales": scales, "g_state": g_state}

    # -- the reference's CPU random stream continued on the device ---------------
    def rng_attach(self, generator):
        """Continue ``generator``'s stream (torch's CPU MT19937) on the device:
        its 624-word state and left/next counters (get_state(), bytes 8, 16 and
        24..5016) are copied in; draw_batch_device then produces the same
        uniforms torch.rand(n) would, on a stream of its own."""
        b = generator.get_state().numpy()
        if b.size != 5056:
            raise _lib.MjxError(f"unexpected CPU generator state size {b.size}")
        dev = self.s.device
        words = b[24:24 + 624 * 8].view(np.uint64).astype(np.uint32)
        left = int(b[8:12].view(np.int32)[0])
        nxt = int(b[16:24].view(np.uint64)[0])
        self._mt = torch.from_numpy(words.view(np.int32).copy()).to(dev)
        self._ln = torch.tensor([left, nxt], dtype=torch.int32, device=dev)
        self._gen_state_bytes = b.copy()
        self._gen_stream = torch.cuda.Stream(device=dev)
        self._gen_done = [torch.cuda.Event(), torch.cuda.Event()]
        self._mask_free = [torch.cuda.Event(), torch.cuda.Event()]
        self._gen_slot = 0

    def rng_state_bytes(self, slot=None):
        """The CPU generator state (uint8 tensor for set_state) at the start of
        the batch drawn in ``slot`` (None: the current device position)."""
        if slot is None:
            mt, ln = self._mt, self._ln
        else:
            mt, ln = self._snap[slot]
        b = self._gen_state_bytes.copy()
        b[24:24 + 624 * 8] = mt.cpu().numpy().view(np.uint32).astype(np.uint64).view(np.uint8)
        left, nxt = (int(x) for x in ln.cpu().numpy())
        b[8:12] = np.array([left], dtype=np.int32).view(np.uint8)
        b[16:24] = np.array([nxt], dtype=np.uint64).view(np.uint8)
        return torch.from_numpy(b)

    JUMP_CHUNKS = 256      # workgroups of the jump-ahead generator (one per CU)

    def _jump_table(self, k):
        """Device copy of the jump polynomials z^(jL-1) mod P for a batch of k
        iterations (mjx_mt_jump_table, host setup once per k), or None when
        the batch fits one chunk."""
        cache = self.__dict__.setdefault("_jump_tables", {})
        if k not in cache:
            lib = _lib.load()
            words = lib.mjx_mt_jump_table_words(self.plan.n, k, self.JUMP_CHUNKS)
            if words < 0:
                raise _lib.MjxError(f"no jump-ahead geometry for n={self.plan.n}, k={k}")
            if words == 0:
                cache[k] = None
            else:
                host = np.empty(words, dtype=np.uint64)
                _lib.call("mjx_mt_jump_table", self.plan.n, k, self.JUMP_CHUNKS, host.ctypes.data)
                cache[k] = torch.from_numpy(host.view(np.int64)).to(self.s.device)
        return cache[k]

    def draw_batch_device(self, k, t0=None):
        """draw_batch on the device (mjx_hpr_refresh_masks on the generator's
        own stream): the same masks, no host work but k thresholds."""
        if k % 2:
            raise ValueError("batch size must be even (the message buffers alternate)")
        self._batch_buffers(k)
        if getattr(self, "_gmask", None) is None or self._gmask[0].shape != (k, self.plan.n):
            n, dev = self.plan.n, self.s.device
            self._gmask = [torch.empty((k, n), dtype=torch.bool, device=dev) for _ in range(2)]
            self._gthr = [torch.empty(k, dtype=torch.float64, device=dev) for _ in range(2)]
            self._snap = [(torch.empty_like(self._mt), torch.empty_like(self._ln)) for _ in range(2)]
        t0 = self.t if t0 is None else t0
        slot = self._gen_slot
        self._gen_slot ^= 1
        thr = torch.tensor([1 - (1 + (t0 + j)) ** (-self.gamma) for j in range(k)], dtype=torch.float64)
        scales = self._pin[slot][1]
        if self.layout == "q":
            scales.copy_(torch.tensor([self.decay(t0 + j) for j in range(k + 1)], dtype=self.dtype))
        gs = self._gen_stream
        table = self._jump_table(k)
        with torch.cuda.stream(gs):
            gs.wait_event(self._mask_free[slot])           # the batch two back has copied its masks out
            self._snap[slot][0].copy_(self._mt)
            self._snap[slot][1].copy_(self._ln)
            self._gthr[slot].copy_(thr)
            # the batch-start state (the snapshot) in, the state after the batch out
            _lib.call("mjx_hpr_refresh_masks_jump", _device.ptr(self._snap[slot][0]), _device.ptr(self._snap[slot][1]),
                      _device.ptr(self._mt), _device.ptr(self._ln), self.plan.n, k, self.JUMP_CHUNKS,
                      _device.ptr(table) if table is not None else None, _device.ptr(self._gthr[slot]),
                      _device.ptr(self._gmask[slot]), gs.cuda_stream)
            self._gen_done[slot].record(gs)
        return {"k": k, "t0": t0, "slot": slot, "scales": scales, "device": True}

    def launch_batch(self, drawn, graph=True):
        """Device half: the batch's masks (and decay scales) copied in, its k
        iterations launched (a hipGraph replay after one eager batch), the sums
        queued for one host read (collect_batch).  Nothing here waits."""
        k = drawn["k"]
        if drawn["t0"] != self.t:
            raise ValueError("batch drawn for another iteration")
        if drawn.get("device"):
            slot = drawn["slot"]
            torch.cuda.current_stream().wait_event(self._gen_done[slot])
            self._mask.copy_(self._gmask[slot])
            self._mask_free[slot].record()
        else:
            self._mask.copy_(drawn["mask"], non_blocking=True)
        if self.layout == "q":
            self._scales.copy_(drawn["scales"], non_blocking=True)
        if graph and self._graph is not None:
            self._graph.replay()
        elif graph and getattr(self, "_warm", False):
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._batch_launches(k)
            self._graph.replay()
        else:
            self._batch_launches(k)
            self._warm = True
        self.t += k
        self.s.copy_(self._s_hist[k - 1])
        self._sums_host.copy_(self._cnt, non_blocking=True)
        self._done.record()

    def collect_batch(self):
        """The one host read of a batch: sum(s_endstate(s)) of every iteration."""
        self._done.synchronize()
        return 2 * self._sums_host.numpy().copy() - self.plan.n

    def steps_batched(self, k, generator, graph=True):
        """k iterations of the main loop (code/HPR_pytorch_RRG.py:345-356) with no
        host read in between (draw_batch + launch_batch + collect_batch).
        Returns (sums[k] int64 numpy, s_hist (k, n) int32 device tensor,
        generator state before the draws)."""
        drawn = self.draw_batch(k, generator)
        self.launch_batch(drawn, graph=graph)
        return self.collect_batch(), self._s_hist, drawn["g_state"]


def hpr_run(d, n, p, c, damppar=0.4, attr_value=1, lmbd_in=None, pie=0.3, gamma=0.1, TT=10000, edges=None,
            nbrs=None, seed=0, dtype=torch.float32, chi0=None, biases0=None, generator=None, batch=16, graph=True,
            layout=None, rng="device", init_generator=None):
    """The HPR experiment of code/HPR_pytorch_RRG.py:224-377 for one graph.

    Randomness follows the reference: with ``generator`` a torch CPU generator
    (default: seeded with ``seed``), chi0 = rand(2E, 4^T) row-normalised,
    biases0 = rand(n, 2) row-normalised (:329-335) and one rand(n) per
    iteration (:142), all float64 like the reference's default dtype.  The
    loop runs in device batches of ``batch`` iterations (one host read each,
    replayed as a hipGraph with ``graph``); on return the generator has made
    exactly the draws the reference makes up to its stop iteration.
    ``layout``: the message state's layout (HPRState).  ``rng``: "device"
    continues the generator's stream on the device beside the iterations
    (mjx_hpr_refresh_masks, bit-identical uniforms), "host" draws torch.rand
    on the CPU while the previous batch runs.
    ``init_generator``: the generator chi0 and biases0 are drawn from
    (default ``generator``).  The reference draws them with
    ``device=device`` (:102, :334), i.e. on a GPU box from torch's CUDA
    generator, and only the per-iteration rand(n) (:142) from the CPU one:
    pass a ``torch.Generator("cuda")`` to make those same draws, in the same
    order (chi0 first, :331), on the device.
    Returns the np.savez keys of :377 (mag_reached, conf, num_steps, graphs).
    """
    from .graph import random_regular_edges
    if edges is None:
        edges = random_regular_edges(d, n, seed=seed)
    plan = HPRPlan(edges, n, d, nbrs)
    if generator is None:
        generator = torch.Generator().manual_seed(int(seed))
    nc = 4 ** (p + c)
    ig = generator if init_generator is None else init_generator
    if chi0 is None:                                       # mes_init_mat, code/HPR_pytorch_RRG.py:101-103
        chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, device=ig.device, generator=ig)
        chi0 = chi0 / torch.sum(chi0, axis=1, keepdims=True)
    if biases0 is None:                                    # code/HPR_pytorch_RRG.py:334-335
        biases0 = torch.rand((n, 2), dtype=torch.float64, device=ig.device, generator=ig)
        biases0 = biases0 / torch.sum(biases0, axis=1, keepdims=True)
    st = HPRState(plan, p, c, chi0, biases0, dtype=dtype, damppar=damppar, attr_value=attr_value,
                  lmbd_in=lmbd_in, pie=pie, gamma=gamma, layout=layout)
    st.s_from_biases()
    total = st.sum_end()
    m_final = total / n
    s_dev = st.s
    B = batch + batch % 2 if batch else 0
    on_dev = rng == "device"
    if B > 1 and m_final < 1:
        if on_dev:
            st._batch_buffers(B)
            st.rng_attach(generator)
            draw = lambda t0=None: st.draw_batch_device(B, t0)  # noqa: E731
        else:
            draw = lambda t0=None: st.draw_batch(B, generator, t0)  # noqa: E731
        drawn = draw()
    while m_final < 1:                                     # code/HPR_pytorch_RRG.py:344-356
        if B > 1:
            # `batch` iterations per host read; the run stops at the first
            # iteration the reference would stop at (t > TT, or consensus).
            # The next batch's uniforms are drawn on the host while this one
            # runs on the device (and discarded if the run stops in it).
            t0 = st.t
            st.launch_batch(drawn, graph=graph)
            cur = drawn
            drawn = draw(t0 + B)
            sums, s_hist = st.collect_batch(), st._s_hist
            for j in range(B):
                t = t0 + j + 1
                if t > TT:
                    m_final = 2
                elif sums[j] / n >= 1:
                    m_final = sums[j] / n
                if m_final >= 1:
                    st.t = t
                    s_dev = s_hist[j]
                    # leave the generator where the reference's would be: j+1 draws
                    generator.set_state(st.rng_state_bytes(cur["slot"]) if on_dev else cur["g_state"])
                    for _ in range(j + 1):
                        torch.rand(n, dtype=torch.float64, generator=generator)
                    break
            else:
                s_dev = st.s
        else:
            total = st.step(generator=generator)
            s_dev = st.s
            if st.t > TT:
                m_final = 2
            else:
                m_final = total / n
    s = s_dev.cpu().numpy()
    return {
        "mag_reached": np.array([np.sum(s) / n]),
        "num_steps": np.array([float(st.t)]),
        "conf": s[None, :].astype(np.float64),
        "graphs": plan.nbrs_host[None, :, :].astype(np.float64),
    }
