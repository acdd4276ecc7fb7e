"""Simulated annealing for strategic initialisations (code/SA_RRG.py:44-92).

``SAReplicas`` runs R independent replicas of the reference's SA loop, all
replicas bit-packed into one spin array (64 per 64-bit word), on one graph or
on a graph per replica (the reference draws a fresh graph for each of its
N_stat replicas, code/SA_RRG.py:58-62: the graphs are stacked in HBM and
replica r reads the rows of its own).  Replica r is bit-identical to the
reference run

    np.random.seed(seeds[r])
    s = 2*np.random.binomial(n=1, p=0.5, size=[n]) - 1      # code/SA_RRG.py:65
    ... while(m_final<1): ...                                # code/SA_RRG.py:72-85

on the same neighbour array ``N`` — same proposals, same accept decisions,
same final ``conf``, ``num_steps`` and ``mag_reached``.  (The reference runs
its N_stat replicas back to back on one global numpy stream and a fresh graph
each; here each replica owns a seed, which is what makes them independent and
parallel.)

Two evaluation modes give bit-identical trajectories:

* ``"lightcone"`` (default where it fits): one persistent kernel runs many
  steps; each proposal's sum(s_endstate) change is computed only inside the
  radius-(p+c-1) ball around the flipped node from cached rollout levels
  (mjx_sa_lightcone_steps) — O(ball) instead of O(N).
* ``"rollout"``: per step the device draws (i, u) and flips s[i] for every
  running replica (k_sa_propose), rolls out the flipped configuration with the
  fused per-replica +1 count (mjx_rollout_ell_rp), then does the Metropolis
  test, annealing schedule and consensus check (k_sa_accept), un-flipping
  rejected proposals.
"""
import numpy as np
import torch

from . import _device, _lib
from .dynamics import as_graph, rollout, pack, unpack
from .graph import Graph

PAR_A = 1.0005   # code/SA_RRG.py:49
PAR_B = 1.0005   # code/SA_RRG.py:50


def schedule_constants(n):
    """(a0, b0, a_cap, b_cap, t_cap) exactly as the reference computes them
    in Python floats/ints (code/SA_RRG.py:67-68, 80-81, 84)."""
    return 0.015 * n, 0.01 * n, 4.5 * n, float(5 * n), 2 * n ** 3


KERNEL_FLAGS = {"no_spec": _lib.MJX_SA_NO_SPEC, "no_cone2": _lib.MJX_SA_NO_CONE2, "lds_serial": _lib.MJX_SA_LDS_SERIAL,
                "lds_single": _lib.MJX_SA_LDS_SINGLE, "lds_pair": _lib.MJX_SA_LDS_PAIR, "lds_wave": _lib.MJX_SA_LDS_WAVE,
                "lds_cu": _lib.MJX_SA_LDS_CU}


def _graph_stack(N, R, graph_of):
    """(device int32 (G*n, d) rows, n, d, device int32 rep_graph or None) for
    one neighbour array or a sequence of them (stacked, replica r on graph
    graph_of[r], default r)."""
    multi = isinstance(N, (list, tuple)) or (isinstance(N, np.ndarray) and N.ndim == 3) or \
        (isinstance(N, torch.Tensor) and N.dim() == 3)
    if not multi:
        if graph_of is not None:
            raise ValueError("graph_of needs a sequence of graphs")
        g = as_graph(N)
        if g.kind != "ell":
            raise ValueError("SA runs on random regular graphs (ELL adjacency), code/SA_RRG.py:59-61")
        return g, g.adj, g.n, g.d, None
    gl = [x.adj if isinstance(x, Graph) else x for x in N]
    if not gl:
        raise ValueError("no graphs")
    G = len(gl)
    gof = np.arange(R) if graph_of is None else np.asarray(graph_of, dtype=np.int64).reshape(-1)
    if gof.size != R or gof.min() < 0 or gof.max() >= G:
        raise ValueError(f"graph_of: one graph index in [0, {G}) per replica ({R})")
    if graph_of is None and G != R:
        raise ValueError(f"one graph per replica: {G} graphs for {R} replicas (or pass graph_of)")
    shapes = {tuple(x.shape) for x in gl}
    if len(shapes) != 1 or len(next(iter(shapes))) != 2:
        raise ValueError("every graph must be an (n, d) neighbour array of the same n and d")
    n, d = next(iter(shapes))
    if all(isinstance(x, torch.Tensor) and x.is_cuda for x in gl):
        stack = torch.stack([x.to(torch.int32) for x in gl]).reshape(G * n, d).contiguous()
        if stack.numel():
            # the kernels index LDS and HBM with these entries: one device reduction
            lo, hi = torch.aminmax(stack)
            if int(lo.item()) < 0 or int(hi.item()) >= n:
                raise ValueError("adjacency index out of range")
    else:
        a = np.stack([x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x) for x in gl])
        if a.size and (a.min() < 0 or a.max() >= n):
            raise ValueError("adjacency index out of range")
        stack = _device.to_device(np.ascontiguousarray(a.astype(np.int32).reshape(G * n, d)))
    rep = torch.from_numpy(gof.astype(np.int32)).to(stack.device)
    return None, stack, int(n), int(d), rep


class SAReplicas:
    """R bit-packed SA replicas on one random regular graph or on a graph per
    replica (device resident)."""

    def __init__(self, N, p, c, seeds, par_a=PAR_A, par_b=PAR_B, a0=None, b0=None, mode="auto", tape=4096,
                 mt_state=None, layout="auto", graph_of=None, kernel=None, rng="mt19937"):
        """``N``: one (n, d) neighbour array (or Graph) for every replica, or a
        sequence of them (or a (G, n, d) array): replica r runs on graph r, or
        on graph ``graph_of[r]``.  ``mt_state`` = (mt uint32 (R, 624), idx
        int32 (R,)): continue these MT19937 streams instead of seeding
        (``seeds`` then only fixes R); see ``mt_state()`` and
        ``sa_run(stream="global")``.  ``layout`` (light-cone mode): ``"lds"``
        keeps each replica's graph, levels and stream in LDS for a whole call
        (mjx_sa_lds_steps; n <= 65535, the reference's own sizes), ``"cone"``
        keeps the cached levels of one (node, word) side by side in HBM
        (mjx_sa_cone_steps), ``"rec"`` the cone with each node's adjacency
        row in front of its levels (mjx_sa_rec_steps; one shared graph, d <= 4),
        ``"levels"`` as separate arrays
        (mjx_sa_lightcone_steps); ``"auto"``: lds where it fits, else cone;
        same results in every layout.  ``kernel``: light-cone kernel
        selection passed to the ABI (tests, tuning): ``split`` (waves per word
        column), ``spec_k`` (8 or 16), ``no_spec``, ``no_cone2``, ``lds_serial``, ``lds_single``, ``lds_pair``,
        ``lds_wave`` (one wave per replica instead of the whole-CU kernels at
        p+c-1 >= 2), ``lds_cu`` (the whole CU level by level: the default at
        d = 3, 4, p+c-1 = 2, 3 where it fits; ``split`` = 16 for its 16-wave
        form), ``split`` = 4, 8 or 16 alone (the whole CU a proposal per wave,
        k_sa_lds_wg); the results never depend on it.  ``rng``: ``"mt19937"`` replays numpy's seeded
        stream (the reference's proposals, bit for bit); ``"philox"`` is the
        NON-parity throughput mode: the proposal of step t of
        replica r comes from Philox-4x32-10 keyed by its seed (a pure function
        of (seed, t), drawn into the tape: light-cone mode, a non-LDS layout,
        tape > 0; the initial configuration still from the seeded MT19937)."""
        seeds = np.asarray(seeds, dtype=np.int64).reshape(-1)
        if seeds.size == 0 or seeds.min() < 0 or seeds.max() > 0xFFFFFFFF:
            raise ValueError("seeds must be in [0, 2**32)")  # np.random.seed's range
        self.R = R = int(seeds.size)
        self.graph, self.adj, n, d, self.rep_graph = _graph_stack(N, R, graph_of)
        self.d = d
        dev = _device.require_gpu()
        self.p, self.c = int(p), int(c)
        self.n = n
        if rng not in ("mt19937", "philox"):
            raise ValueError(f"unknown rng {rng!r}")
        self.rng = rng
        if n < 2:
            raise ValueError("n must be >= 2")
        self.W = W = _device.words_for(R)
        a0d, b0d, self.a_cap, self.b_cap, self.t_cap = schedule_constants(n)
        self.a0 = a0d if a0 is None else float(a0)
        self.b0 = b0d if b0 is None else float(b0)
        self.par_a, self.par_b = float(par_a), float(par_b)
        if self.t_cap > 2 ** 63 - 1:
            self.t_cap = 2 ** 63 - 1
        i64 = torch.int64
        self.s = torch.zeros(n * W, dtype=i64, device=dev)
        self.tmp1 = torch.empty_like(self.s)
        self.tmp2 = torch.empty_like(self.s)
        self.seeds = torch.from_numpy(seeds.astype(np.uint32).view(np.int32)).to(dev)
        self.mt = torch.empty(R * 624, dtype=torch.int32, device=dev)
        self.mt_idx = torch.empty(R, dtype=torch.int32, device=dev)
        self.a = torch.empty(R, dtype=torch.float64, device=dev)
        self.b = torch.empty(R, dtype=torch.float64, device=dev)
        self.t = torch.zeros(R, dtype=i64, device=dev)
        self.sum_end = torch.zeros(R, dtype=i64, device=dev)
        self.done = torch.zeros(R, dtype=torch.int32, device=dev)
        self.prop_i = torch.empty(R, dtype=torch.int32, device=dev)
        self.prop_s = torch.empty(R, dtype=torch.int8, device=dev)
        self.prop_u = torch.empty(R, dtype=torch.float64, device=dev)
        self.cnt = torch.zeros(R, dtype=i64, device=dev)
        self.ties = torch.zeros(R, dtype=torch.int32, device=dev)
        self._state = _lib.MjxSaState()
        for f in ("mt", "mt_idx", "a", "b", "t", "sum_end", "done", "prop_i", "prop_s", "prop_u", "cnt"):
            setattr(self._state, f, getattr(self, f).data_ptr())
        self._state.tr_tie = self.ties.data_ptr()
        self._state.rep_graph = self.rep_graph.data_ptr() if self.rep_graph is not None else None
        kernel = dict(kernel or {})
        self._state.opt_split = int(kernel.pop("split", 0) or 0)
        self._state.opt_spec_k = int(kernel.pop("spec_k", 0) or 0)
        flags = 0
        for key, bit in KERNEL_FLAGS.items():
            if kernel.pop(key, False):
                flags |= bit
        if kernel:
            raise ValueError(f"unknown kernel options {sorted(kernel)}")
        self._state.opt_flags = flags
        self.philox_key = None
        if rng == "philox":
            self.philox_key = torch.from_numpy(seeds.astype(np.int64)).to(dev)
            self._state.philox_key = self.philox_key.data_ptr()
        T = self.p + self.c - 1
        if mt_state is None:
            _lib.call("mjx_sa_init", _device.ptr(self.adj), n, self.d, self.p, self.c, R,
                      _device.ptr(self.seeds), self.a0, self.b0, _device.ptr(self.s), _device.ptr(self.tmp1),
                      _device.ptr(self.tmp2) if T >= 2 else None, _lib.ctypes.byref(self._state),
                      _device.stream_handle())
        else:
            mt_in = np.ascontiguousarray(np.asarray(mt_state[0], dtype=np.uint32).reshape(R, 624))
            idx_in = np.ascontiguousarray(np.asarray(mt_state[1], dtype=np.int32).reshape(R))
            if idx_in.min() < 0 or idx_in.max() > 624:
                raise ValueError("MT19937 word index must be in [0, 624]")
            mt_d = torch.from_numpy(mt_in.view(np.int32)).to(dev)
            idx_d = torch.from_numpy(idx_in).to(dev)
            _lib.call("mjx_sa_init_mt", _device.ptr(self.adj), n, self.d, self.p, self.c, R,
                      _device.ptr(mt_d), _device.ptr(idx_d), self.a0, self.b0, _device.ptr(self.s),
                      _device.ptr(self.tmp1), _device.ptr(self.tmp2) if T >= 2 else None,
                      _lib.ctypes.byref(self._state), _device.stream_handle())
            torch.cuda.current_stream().synchronize()       # mt_d / idx_d are freed on return
        lds = _lib.load().mjx_sa_lightcone_lds(self.d, self.p, self.c)
        fits = T >= 1 and 0 < lds <= 150 * 1024
        if mode == "auto":
            mode = "lightcone" if fits else "rollout"
        if rng == "philox" and mode != "lightcone":
            raise ValueError("the Philox stream is drawn into the light-cone tape: mode='lightcone'")
        if mode == "lightcone" and not fits:
            raise ValueError(f"light-cone SA unsupported for d={self.d}, p+c-1={T}")
        if mode not in ("lightcone", "rollout"):
            raise ValueError(f"unknown SA mode {mode!r}")
        self.mode = mode
        if layout not in ("auto", "lds", "cone", "rec", "levels"):
            raise ValueError(f"unknown light-cone layout {layout!r}")
        # the LDS bytes and workgroup size of the LDS kernel these options select
        lds_threads = _lib.ctypes.c_int(64)
        lds_bytes = _lib.load().mjx_sa_lds_plan(n, self.d, self.p, self.c, flags, self._state.opt_split,
                                                _lib.ctypes.byref(lds_threads))
        lds_fits = 0 < lds_bytes <= 160 * 1024
        # A replica in LDS is one workgroup for a whole call: the lane-held step (d <= 4,
        # k_sa_lds_fast) runs SA_RRG.py's shapes fastest (d=4, n=1e4, 64 replicas: p=c=1
        # 0.83 us per step vs 1.42 in the speculative batches, p=3 1.78 vs 69 in the cone)
        # while the replicas fit the CUs in one round; more replicas than that go to the
        # speculative batches (k_sa_spec: d=3 at p+c-1 <= 2, d=4 at p+c-1 = 1), in the
        # record layout for one shared graph (configs[1]: 4.31 -> 4.20 us per step at
        # R = 4096 vs the plain cone, same box), else to the cone.
        spec = (self.d == 3 and T <= 2) or (self.d == 4 and T == 1)
        per_cu = max(1, min((160 * 1024) // max(lds_bytes, 1), 32 // max(1, lds_threads.value // 64)))
        one_round = lds_fits and R <= _device.cu_count() * per_cu
        if rng == "philox" and layout == "lds":
            raise ValueError("the LDS kernels replay MT19937 in the step: rng='philox' needs another layout")
        if rng == "philox" and not tape:
            raise ValueError("rng='philox' draws into the proposal tape: tape > 0")
        if layout == "auto":
            if lds_fits and (one_round or not spec) and rng != "philox":
                layout = "lds"
            elif spec and self.rep_graph is None:
                layout = "rec"
            else:
                layout = "cone"
        if mode == "lightcone" and layout == "lds" and not lds_fits:
            raise ValueError(f"LDS-resident SA unsupported for n={n}, d={self.d}, p+c-1={T}")
        if mode == "lightcone" and layout == "rec" and (self.rep_graph is not None or
                                                        _lib.load().mjx_sa_rec_words(self.d, self.p, self.c) < 0):
            raise ValueError("the record layout needs one graph shared by every replica and d <= 4")
        self.layout = layout if mode == "lightcone" else None
        self.cone = None
        self.adj_pad = None
        self._levels = None
        if mode == "lightcone" and layout == "lds":
            self.tape_cap = 0                    # the LDS kernel draws in the step, exactly
        elif mode == "lightcone":
            # levels s_1..s_T = onestep^t(s); the rollout ping-pong buffers are reused
            self._levels = [self.tmp1, self.tmp2][:T] + [torch.empty_like(self.s) for _ in range(T - 2)]
            self._lvl = (_lib.ctypes.c_void_p * T)(*[t.data_ptr() for t in self._levels])
            if layout == "cone":
                lv = _lib.load().mjx_sa_cone_words(self.p, self.c)
                self.cone = torch.empty(n * W * lv, dtype=i64, device=dev)
            elif layout == "rec":
                # the cone with each node's adjacency row in front of its levels
                lv = _lib.load().mjx_sa_rec_words(self.d, self.p, self.c)
                self.cone = torch.empty(n * W * lv, dtype=i64, device=dev)
            self._build_levels()
            if layout == "cone" and self.d == 3:
                # rows padded to 16 B: one load per row in the one-round-trip step
                # (graph g of a stack at rows g*n .. g*n + n - 1)
                rows = self.adj.numel() // 3
                self.adj_pad = torch.zeros((rows, 4), dtype=torch.int32, device=dev)
                self.adj_pad[:, :3] = self.adj.view(rows, 3)
            # proposal tape: (i, u) of `tape` steps per replica drawn ahead by
            # a wave per replica (0 = draw inside the step kernel); the library
            # draws the MT19937 tape in two halves, one chunk ahead on a side
            # stream (4096: chunks 128, 2048, 2048, ...: few step launches per
            # call, each ending on its slowest wave; 12 B per replica and row)
            self.tape_cap = int(tape) if tape else 0
            if self.tape_cap > 0:
                self.tape_i = torch.empty(self.tape_cap * R, dtype=torch.int32, device=dev)
                self.tape_u = torch.empty(self.tape_cap * R, dtype=torch.float64, device=dev)
                self._state.tape_i, self._state.tape_u = self.tape_i.data_ptr(), self.tape_u.data_ptr()
                self._state.tape_cap = self.tape_cap

    def _build_levels(self):
        """The cached levels onestep^t(s), t = 1..T, from s (light-cone layouts
        other than lds, which rebuilds them in LDS every call), packed into the
        cone / record layout when in use."""
        n, R = self.n, self.R
        _lib.call("mjx_sa_lightcone_prepare", _device.ptr(self.adj), n, self.d, self.p, self.c, R,
                  _device.ptr(self.rep_graph) if self.rep_graph is not None else None,
                  _device.ptr(self.s), self._lvl, _device.stream_handle())
        if self.layout == "cone":
            _lib.call("mjx_sa_cone_pack", n, self.p, self.c, R, _device.ptr(self.s), self._lvl,
                      _device.ptr(self.cone), _device.stream_handle())
        elif self.layout == "rec":
            _lib.call("mjx_sa_rec_pack", _device.ptr(self.adj), n, self.d, self.p, self.c, R,
                      _device.ptr(self.s), self._lvl, _device.ptr(self.cone), _device.stream_handle())

    # -- checkpoint / resume (long runs to consensus: SA_RRG.py's n = 1e4 runs
    # take 1e7-1e9 proposals per replica) -------------------------------------
    _CKPT_STATE = ("s", "mt", "mt_idx", "a", "b", "t", "sum_end", "done", "ties")

    def checkpoint(self):
        """Everything a resumed run needs, as host arrays: the configuration
        (replica-packed bits), every replica's MT19937 stream (numpy's state,
        exactly), a, b, t, sum(s_end), the done flags (code/SA_RRG.py:65-85's
        loop state) and the parameters.  ``resume`` continues it bit for bit."""
        if self.mode == "lightcone" and getattr(self, "tape_cap", 0) and self.rng != "philox":
            raise ValueError("the proposal tape draws ahead: checkpoint needs tape=0 (or the lds / rollout modes)")
        torch.cuda.current_stream().synchronize()
        out = {k: getattr(self, k).cpu().numpy().copy() for k in self._CKPT_STATE}
        out["params"] = np.array([self.n, self.d, self.p, self.c, self.R], dtype=np.int64)
        out["schedule"] = np.array([self.par_a, self.par_b, self.a0, self.b0, self.a_cap, self.b_cap],
                                   dtype=np.float64)
        out["t_cap"] = np.array(self.t_cap, dtype=np.int64)
        out["graphs_sha256"] = np.array(self.graphs_digest())
        out["rng"] = np.array(self.rng)
        if self.philox_key is not None:          # (the Philox stream's state: the key and t)
            out["philox_key"] = self.philox_key.cpu().numpy().copy()
        return out

    def graphs_digest(self):
        """SHA-256 of the graphs this run reads: the stacked int32 rows and the
        replica -> graph map (a resumed run must read the same ones)."""
        import hashlib
        h = hashlib.sha256()
        h.update(np.array([self.n, self.d], dtype=np.int64).tobytes())
        h.update(np.ascontiguousarray(self.adj.cpu().numpy().astype(np.int32)).tobytes())
        h.update(b"rep_graph" if self.rep_graph is not None else b"shared")
        if self.rep_graph is not None:
            h.update(np.ascontiguousarray(self.rep_graph.cpu().numpy().astype(np.int32)).tobytes())
        return h.hexdigest()

    def save_checkpoint(self, path):
        np.savez(path, **self.checkpoint())

    @classmethod
    def resume(cls, N, ckpt, graph_of=None, mode="auto", layout="auto", kernel=None, tape=0):
        """A run continued from ``checkpoint()`` (a dict, or the path of a
        ``save_checkpoint`` file) on the same graphs ``N``: the same proposals,
        accepts and final state as the uninterrupted run."""
        if not isinstance(ckpt, dict):
            with np.load(ckpt, allow_pickle=False) as z:
                ckpt = {k: z[k] for k in z.files}
        n, d, p, c, R = (int(x) for x in ckpt["params"])
        par_a, par_b, a0, b0 = (float(x) for x in ckpt["schedule"][:4])
        rng = str(ckpt["rng"]) if "rng" in ckpt else "mt19937"
        if rng == "philox":
            mode, tape = "lightcone", (tape or 1024)
        sa = cls(N, p, c, np.zeros(R, dtype=np.int64), par_a=par_a, par_b=par_b, a0=a0, b0=b0, mode=mode,
                 tape=tape, layout=layout, graph_of=graph_of, kernel=kernel, rng=rng)
        if (sa.n, sa.d, sa.R) != (n, d, R):
            raise ValueError(f"checkpoint of n={n}, d={d}, R={R} does not fit these graphs (n={sa.n}, d={sa.d})")
        if "graphs_sha256" in ckpt and str(ckpt["graphs_sha256"]) != sa.graphs_digest():
            raise ValueError("checkpoint was taken on other graphs (or another replica -> graph map) than these")
        a_cap, b_cap = (float(x) for x in ckpt["schedule"][4:6])
        if (a_cap, b_cap) != (sa.a_cap, sa.b_cap) or int(ckpt["t_cap"]) != int(sa.t_cap):
            raise ValueError(f"checkpoint caps a={a_cap}, b={b_cap}, t={int(ckpt['t_cap'])} differ from "
                             f"code/SA_RRG.py's for n={n} (a={sa.a_cap}, b={sa.b_cap}, t={sa.t_cap})")
        sa.t_cap = int(ckpt["t_cap"])
        for k in cls._CKPT_STATE:
            dst = getattr(sa, k)
            src = torch.from_numpy(np.ascontiguousarray(ckpt[k])).to(dst.device)
            if src.shape != dst.shape or src.dtype != dst.dtype:
                raise ValueError(f"checkpoint field {k}: {tuple(src.shape)} {src.dtype}, expected "
                                 f"{tuple(dst.shape)} {dst.dtype}")
            dst.copy_(src)
        if rng == "philox":
            sa.philox_key.copy_(torch.from_numpy(np.ascontiguousarray(ckpt["philox_key"], dtype=np.int64)))
        if sa.mode == "lightcone" and sa.layout != "lds":
            sa._build_levels()
        torch.cuda.current_stream().synchronize()
        return sa

    # -- stepping -----------------------------------------------------------
    def steps(self, k, trace=False):
        """Advance every running replica by k proposals.  With ``trace`` the
        per-step (i, accept, sum_end, delta_H) arrays of shape (k, R) are
        returned (i = -1 / accept = -1 once a replica is done)."""
        k = int(k)
        st = self._state
        tr = None
        if trace:
            dev = self.s.device
            tr = {
                "i": torch.empty((k, self.R), dtype=torch.int32, device=dev),
                "accept": torch.empty((k, self.R), dtype=torch.int8, device=dev),
                "sum_end": torch.empty((k, self.R), dtype=torch.int64, device=dev),
                "dE": torch.empty((k, self.R), dtype=torch.float64, device=dev),
            }
            st.tr_i, st.tr_acc = tr["i"].data_ptr(), tr["accept"].data_ptr()
            st.tr_sum, st.tr_dE = tr["sum_end"].data_ptr(), tr["dE"].data_ptr()
        else:
            st.tr_i = st.tr_acc = st.tr_sum = st.tr_dE = None
        T = self.p + self.c - 1
        if self.layout == "lds":
            _lib.call("mjx_sa_lds_steps", _device.ptr(self.adj), self.n, self.d, self.p, self.c, self.R,
                      _device.ptr(self.s), _lib.ctypes.byref(st), k, self.par_a, self.par_b, self.a_cap, self.b_cap,
                      int(self.t_cap), _device.stream_handle())
        elif self.layout == "rec":
            _lib.call("mjx_sa_rec_steps", _device.ptr(self.adj), None, self.n, self.d, self.p, self.c,
                      self.R, _device.ptr(self.s), _device.ptr(self.cone), _lib.ctypes.byref(st), k, self.par_a,
                      self.par_b, self.a_cap, self.b_cap, int(self.t_cap), _device.stream_handle())
        elif self.mode == "lightcone" and self.cone is not None:
            _lib.call("mjx_sa_cone_steps", _device.ptr(self.adj),
                      _device.ptr(self.adj_pad) if self.adj_pad is not None else None, self.n, self.d, self.p, self.c,
                      self.R, _device.ptr(self.s), _device.ptr(self.cone), _lib.ctypes.byref(st), k, self.par_a,
                      self.par_b, self.a_cap, self.b_cap, int(self.t_cap), _device.stream_handle())
        elif self.mode == "lightcone":
            _lib.call("mjx_sa_lightcone_steps", _device.ptr(self.adj), self.n, self.d, self.p, self.c,
                      self.R, _device.ptr(self.s), self._lvl, _lib.ctypes.byref(st), k, self.par_a, self.par_b,
                      self.a_cap, self.b_cap, int(self.t_cap), _device.stream_handle())
        else:
            _lib.call("mjx_sa_steps", _device.ptr(self.adj), self.n, self.d, self.p, self.c, self.R,
                      _device.ptr(self.s), _device.ptr(self.tmp1), _device.ptr(self.tmp2) if T >= 2 else None,
                      _lib.ctypes.byref(st), k, self.par_a, self.par_b, self.a_cap, self.b_cap,
                      int(self.t_cap), _device.stream_handle())
        st.tr_i = st.tr_acc = st.tr_sum = st.tr_dE = None
        return tr

    @property
    def levels(self):
        """The cached levels onestep^t(s), t = 1..T, as separate (n*W,) arrays
        (unpacked from the cone layout when that is in use)."""
        if self.mode != "lightcone":
            raise AttributeError("levels exist in the light-cone mode only")
        if self.layout == "lds":
            # kept in LDS during a call only: rebuilt here from s, as every call does
            T = self.p + self.c - 1
            self._levels = [torch.empty_like(self.s) for _ in range(T)]
            lvl = (_lib.ctypes.c_void_p * T)(*[t.data_ptr() for t in self._levels])
            _lib.call("mjx_sa_lightcone_prepare", _device.ptr(self.adj), self.n, self.d, self.p, self.c, self.R,
                      _device.ptr(self.rep_graph) if self.rep_graph is not None else None,
                      _device.ptr(self.s), lvl, _device.stream_handle())
            return self._levels
        self._unpack_cone()
        return self._levels

    def cone_level0(self):
        """Level 0 as the cone holds it (equal to ``s`` after every step)."""
        if self.cone is None:
            raise AttributeError("no cone layout in use")
        self._unpack_cone()
        return self._s0buf

    def _unpack_cone(self):
        if self.cone is None:
            return
        if getattr(self, "_s0buf", None) is None:
            self._s0buf = torch.empty_like(self.s)
        if self.layout == "rec":
            _lib.call("mjx_sa_rec_unpack", self.n, self.d, self.p, self.c, self.R, _device.ptr(self.cone),
                      _device.ptr(self._s0buf), self._lvl, _device.stream_handle())
        else:
            _lib.call("mjx_sa_cone_unpack", self.n, self.p, self.c, self.R, _device.ptr(self.cone),
                      _device.ptr(self._s0buf), self._lvl, _device.stream_handle())

    def all_done(self):
        return bool((self.done != 0).all().item())

    def mt_state(self):
        """Host copy (mt uint32 (R, 624), idx int32 (R,)) of every replica's
        MT19937 stream: exactly where numpy's stream would be after the same
        draws when the proposals are drawn in the step (``tape=0`` or the
        rollout mode); a proposal tape draws ahead of the stop."""
        if self.mode == "lightcone" and getattr(self, "tape_cap", 0):
            raise ValueError("the proposal tape draws ahead: use tape=0 (or mode='rollout') for an exact stream")
        mt = self.mt.cpu().numpy().view(np.uint32).reshape(self.R, 624).copy()
        return mt, self.mt_idx.cpu().numpy().copy()

    def run(self, max_steps=None, chunk=256, max_chunk=16384, max_seconds=None):
        """Step until every replica has reached consensus or the t cap
        (``while(m_final<1)``, code/SA_RRG.py:72), or ``max_steps``, or
        ``max_seconds`` of wall time.  The done flags are read once per
        chunk; chunks grow from ``chunk`` to ``max_chunk`` steps (a finished
        replica skips the rest of a chunk)."""
        import time
        t0 = time.perf_counter()
        taken = 0
        while not self.all_done():
            k = chunk if max_steps is None else min(chunk, max_steps - taken)
            if k <= 0 or (max_seconds is not None and time.perf_counter() - t0 >= max_seconds):
                break
            self.steps(k)
            taken += k
            chunk = min(2 * chunk, max_chunk)
        return taken

    # -- results (code/SA_RRG.py:86-88) ---------------------------------------
    def conf(self):
        """(R, n) int64 +-1 current configurations."""
        return unpack(self.s, self.n, self.R)

    def results(self):
        conf = self.conf().cpu().numpy()
        return {
            # m(s) = np.sum(s)/n with numpy's true division (code/SA_RRG.py:39-40,86)
            "mag_reached": np.sum(conf, axis=1) / self.n,
            "num_steps": self.t.cpu().numpy().astype(np.float64),
            "conf": conf,
            "done": self.done.cpu().numpy(),
            "near_ties": self.ties.cpu().numpy(),
        }


def _sum_end(g, s, T):
    """sum(s_endstate(s)) via one device rollout with the fused +1 count."""
    from .dynamics import popcount
    bits = pack(s)
    cnt = torch.zeros(1, dtype=torch.int64, device=bits.device)
    if T:
        rollout(g, bits, T, counts=cnt)
    else:
        popcount(bits, g.n, counts=cnt)
    return 2 * int(cnt.item()) - g.n


def E_delta(N, s0, a, b, p, c, i):
    """E(s with s_i flipped) - E(s) (code/SA_RRG.py:32-37), two device rollouts.

    The integer sums come from the kernels; the float combination keeps the
    reference's operation order ((-2*a)*s_i + b*D)/n in Python floats.
    """
    g = as_graph(N)
    s = _device.to_device(s0)
    T = int(p) + int(c) - 1
    s1 = s.clone()
    s1[int(i)] = -s1[int(i)]
    sum1 = _sum_end(g, s, T)
    sum2 = _sum_end(g, s1, T)
    si = int(s[int(i)].item())
    return (-2 * a * si + b * (sum1 - sum2)) / g.n


def _graph_list(d, n, N_stat, N, graphs, graph_seed):
    """One (n, d) neighbour array per replica (code/SA_RRG.py:58-61 draws a
    fresh random regular graph per replica)."""
    from .graph import random_regular_graph
    if graphs is not None:
        gl = [np.asarray(g) for g in graphs]
        if len(gl) != N_stat:
            raise ValueError(f"graphs: one neighbour array per replica ({N_stat}), got {len(gl)}")
        return gl
    if N is not None:                       # one given graph for every replica
        return [np.asarray(N)] * N_stat
    base = 0 if graph_seed is None else int(graph_seed)
    return [random_regular_graph(d, n, seed=base + k) for k in range(N_stat)]


def sa_run(d, n, p, c, par_a=PAR_A, par_b=PAR_B, N_stat=5, seed=0, seeds=None, N=None, graph_seed=None,
           max_steps=None, graphs=None, stream="independent", mode="auto", max_seconds=None):
    """Drop-in for the SA_RRG.py experiment (code/SA_RRG.py:44-92).

    Returns the reference's output arrays ``mag_reached, num_steps, conf,
    graphs`` (the np.savez keys of code/SA_RRG.py:92), row k = replica k.

    Graphs: ``graphs`` (one (n, d) neighbour array per replica), else ``N``
    for every replica, else a fresh random d-regular graph per replica
    (``graph_seed + k``), as the reference draws one per replica (:59).

    Randomness:
      * ``stream="global"`` — the reference's own semantics: ONE numpy stream
        seeded once (``np.random.seed(seed)``) and consumed by the replicas
        back to back, so replica k+1's s0 draws continue where replica k's
        last rand() left the stream (:58-88).  Replicas run one after the
        other (mjx_sa_init_mt hands the stream over); bit-identical to the
        script with the same graphs.
      * ``stream="independent"`` — replica k owns ``np.random.seed(seeds[k])``
        (default seed + k); all N_stat replicas run together, bit-packed, each
        on its own graph (graphs stacked in HBM, SAReplicas(graph_of=...)).

    ``max_seconds``: wall budget per replica (global stream) or for the whole
    run (independent streams); a replica stopped by it has ``done`` = 0, and
    with the global stream the replicas after it are not run (their draws
    would start where an unfinished run left the stream).  ``wall_s`` in the
    result: seconds per replica (global) or for the run (independent).
    """
    import time
    gl = _graph_list(d, n, N_stat, N, graphs, graph_seed)
    R = len(gl)
    res = {"mag_reached": np.zeros(R), "num_steps": np.zeros(R), "conf": np.zeros((R, n)),
           "done": np.zeros(R, dtype=np.int32), "near_ties": np.zeros(R, dtype=np.int32), "wall_s": np.zeros(R)}

    def store(k, out, j):
        for key in res:
            if key in out:
                res[key][k] = out[key][j]

    if stream == "global":
        # replica k+1's draws start where replica k's last rand() left the one
        # stream, so the replicas run one after another (tape=0: the stream is
        # consumed exactly, never drawn ahead)
        state = None
        for k, g in enumerate(gl):
            sa = SAReplicas(g, p, c, [int(seed) & 0xFFFFFFFF], par_a=par_a, par_b=par_b, mode=mode, tape=0,
                            mt_state=state)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sa.run(max_steps=max_steps, max_seconds=max_seconds)
            torch.cuda.synchronize()
            res["wall_s"][k] = time.perf_counter() - t0
            out = sa.results()
            store(k, out, 0)
            state = sa.mt_state()
            del sa
            if max_seconds is not None and out["done"][0] == 0 and (max_steps is None or out["num_steps"][0] < max_steps):
                break                       # stopped by the wall budget: the stream cannot be handed on
    elif stream == "independent":
        if seeds is None:
            seeds = [seed + k for k in range(R)]
        seeds = list(seeds)
        if len(seeds) != R:
            raise ValueError(f"seeds: one per replica ({R}), got {len(seeds)}")
        # every replica at once, bit-packed, each on its own graph of a stack
        # (graphs shared by several replicas are stored once)
        uniq, graph_of = {}, []
        for g in gl:
            graph_of.append(uniq.setdefault(id(g), len(uniq)))
        stack = [None] * len(uniq)
        for g in gl:
            stack[uniq[id(g)]] = g
        src = stack[0] if len(stack) == 1 else stack
        sa = SAReplicas(src, p, c, seeds, par_a=par_a, par_b=par_b, mode=mode,
                        graph_of=None if len(stack) == 1 else graph_of)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sa.run(max_steps=max_steps, max_seconds=max_seconds)
        torch.cuda.synchronize()
        res["wall_s"][:] = time.perf_counter() - t0
        out = sa.results()
        for k in range(R):
            store(k, out, k)
        del sa
    else:
        raise ValueError(f"stream must be 'global' or 'independent', got {stream!r}")
    res["graphs"] = np.stack([g.astype(int) for g in gl])
    return res
