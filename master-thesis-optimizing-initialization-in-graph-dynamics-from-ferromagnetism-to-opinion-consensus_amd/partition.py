"""One giant random regular graph partitioned by node range over the ranks of a
process group (config C5: a single d=6 RRG with N=1e9 over
8xMI355X).

Each rank owns a contiguous range of whole 64-node words [lo, hi) and the ELL
rows of those nodes only, generated on its own GPU from the shared seed
(mjx_rrg_generate: the stub pairing is a pure function of the seed, so no
adjacency moves between ranks; 3 GB per rank at C5).  The spin state is
node-packed and replicated: n/8 bytes per rank (125 MB at N=1e9).

One synchronous majority step (onestep_majority, code/SA_RRG.py:18-20) =
the local rows' update (mjx_sweep_ell_np_range) + an all-gather of every
rank's slice of words.  A random regular graph is an expander, so almost
every node is some remote rank's neighbour: the halo IS the whole state, and
the exchange is one in-place RCCL all-gather per sweep (each GPU receives
(P-1)/P * n/8 bytes over its direct xGMI links).  The consensus test
m(s_endstate) < 1 (code/SA_RRG.py:71-72) is one int64 all-reduce of the +1
count fused into the last sweep.

``local_sweep`` may be replaced (tests drive the same exchange logic on CPU
tensors over gloo with a reference sweep); the product path is the HIP kernel.
"""
import numpy as np
import torch

from . import _device, _lib


class NodeRange:
    """Word-aligned node ranges of ``rank`` among ``world`` ranks.

    The padded state of words_padded = sub*world*pieces words is cut into
    world*pieces sub-chunks of ``sub`` words; rank r owns sub-chunk g*world + r
    for every piece g (``pieces``: list of (w_lo, w_hi, lo, hi)).  Piece g of
    all ranks is then one contiguous stretch of words, so its exchange is one
    in-place all-gather, and piece g's exchange overlaps piece g+1's sweep.
    With pieces=1 rank r owns words [r*chunk, (r+1)*chunk) (lo, hi, w_lo, w_hi)."""

    def __init__(self, n, world, rank, pieces=1):
        self.n, self.world, self.rank, self.npieces = int(n), int(world), int(rank), int(pieces)
        if self.npieces < 1:
            raise ValueError("pieces must be >= 1")
        self.words = (self.n + 63) // 64
        self.sub = max(1, -(-self.words // (self.world * self.npieces)))
        self.chunk = self.sub * self.npieces           # words per rank
        self.words_padded = self.sub * self.world * self.npieces
        self.pieces = []
        for g in range(self.npieces):
            w0 = min(self.words, (g * self.world + self.rank) * self.sub)
            w1 = min(self.words, (g * self.world + self.rank + 1) * self.sub)
            self.pieces.append((w0, w1, min(self.n, w0 * 64), min(self.n, w1 * 64)))
        self.w_lo, self.w_hi, self.lo, self.hi = self.pieces[0]
        self.rows = sum(p[3] - p[2] for p in self.pieces)

    def piece_words(self, g):
        """Slice of the padded state that piece g's all-gather fills."""
        return slice(g * self.world * self.sub, (g + 1) * self.world * self.sub)

    def own_words(self, g):
        """This rank's sub-chunk of piece g (padded; may extend past the last node)."""
        w0 = (g * self.world + self.rank) * self.sub
        return slice(w0, w0 + self.sub)


def pack_host(s, words=None):
    """+-1 spins (n,) -> node-packed uint64 words as an int64 numpy array."""
    s = np.asarray(s)
    n = s.shape[0]
    nw = (n + 63) // 64 if words is None else words
    bits = np.zeros(nw * 64, dtype=np.uint8)
    bits[:n] = s > 0
    return np.packbits(bits.reshape(-1, 8), axis=1, bitorder="little").reshape(nw, 8).view(np.int64).reshape(nw)


def unpack_host(words, n):
    """Inverse of pack_host: int64 words -> +-1 int64 spins (n,)."""
    w = np.ascontiguousarray(np.asarray(words, dtype=np.int64))
    bits = np.unpackbits(w.view(np.uint8).reshape(-1, 8), axis=1, bitorder="little").reshape(-1)[:n]
    return 2 * bits.astype(np.int64) - 1


class BinnedPlan:
    """Source-binned sweep plan of the rows [lo, hi) of a d-regular graph
    (mjx_binned_plan_shape / mjx_binned_build / mjx_sweep_binned): the same
    words and counts as mjx_sweep_ell_np_range on those rows."""

    def __init__(self, adj_rows, n, d, lo, hi):
        import ctypes
        self.n, self.d, self.lo, self.hi = int(n), int(d), int(lo), int(hi)
        sizes = (ctypes.c_int64 * 6)()
        _lib.call("mjx_binned_plan_shape", self.n, self.d, self.lo, self.hi, sizes)
        lo_len, hi_len, off_len, index_len, msg_words, work_bytes = (int(x) for x in sizes)
        dev = adj_rows.device
        self.src_lo = torch.empty(max(lo_len, 1), dtype=torch.int16, device=dev)
        self.src_hi = torch.empty(max(hi_len, 1), dtype=torch.int16, device=dev)
        self.off = torch.empty(max(off_len, 1), dtype=torch.int16, device=dev)
        self.index = torch.empty(max(index_len, 1), dtype=torch.int64, device=dev)
        self.msg = torch.empty(max(msg_words, 1), dtype=torch.int64, device=dev)
        if self.hi > self.lo:
            work = torch.empty(work_bytes, dtype=torch.uint8, device=dev)
            _lib.call("mjx_binned_build", _device.ptr(adj_rows), self.n, self.d, self.lo, self.hi,
                      _device.ptr(self.src_lo), _device.ptr(self.src_hi), _device.ptr(self.off),
                      _device.ptr(self.index), _device.ptr(work),
                      work.numel(), _device.stream_handle())
            del work

    APPLY_FORMS = {"auto": 0, "flat": 1, "segments": 2}

    def sweep(self, s_in, s_out, counts=None, apply_form="auto"):
        """apply_form: phase-2 kernel, "auto" (the library's choice), "flat" or "segments"."""
        _lib.call("mjx_sweep_binned", _device.ptr(self.src_lo), _device.ptr(self.src_hi), _device.ptr(self.off),
                  _device.ptr(self.index),
                  self.n, self.d, self.lo, self.hi, _device.ptr(s_in), _device.ptr(self.msg), _device.ptr(s_out),
                  _device.ptr(counts) if counts is not None else None, self.APPLY_FORMS[apply_form],
                  _device.stream_handle())


class ShardedRRG:
    """This rank's part of one d-regular graph and the replicated spin state.

    ``pieces`` (default 1 on one rank, 2 otherwise): the rank's rows are cut
    into that many node ranges (NodeRange), each with its own sweep plan; the
    all-gather of piece g runs on RCCL's stream while piece g+1 is swept.
    ``local_sweep(s_in, s_out, counts, g)`` may replace the HIP sweep of piece
    g (CPU tests over gloo).  ``collective=True`` runs the exchange and the
    count all-reduce through the process group even on one rank (a world-1
    RCCL group on one GPU executes the same in-place all-gather calls as the
    8-GPU run; tests/test_rccl_gpu.py)."""

    def __init__(self, d, n, seed=0, group=None, adj_rows=None, local_sweep=None, device=None, mode="binned",
                 pieces=None, collective=False):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0
        self.backend = self.dist.get_backend(group) if self.dist else None
        self.collective = bool(collective) and self.dist is not None
        self.d, self.n, self.seed = int(d), int(n), int(seed)
        if pieces is None:
            pieces = 1 if self.world == 1 else 2
        self.range = r = NodeRange(n, self.world, self.rank, pieces)
        if adj_rows is not None and not isinstance(adj_rows, (list, tuple)):
            adj_rows = [adj_rows]
        if adj_rows is not None and len(adj_rows) != r.npieces:
            raise ValueError(f"adj_rows: one array per piece ({r.npieces}), got {len(adj_rows)}")
        self.plans = None
        if local_sweep is None:
            self.device = _device.require_gpu()
            if adj_rows is None:
                from .graph import random_regular_rows_device
                adj_rows = [random_regular_rows_device(self.d, self.n, self.seed, lo, hi)
                            for (_, _, lo, hi) in r.pieces]
            self.adj = [_device.to_device(a, dtype=torch.int32) for a in adj_rows]
            self._check_adj()
            if mode == "binned":
                self.plans = [BinnedPlan(a, self.n, self.d, lo, hi) for a, (_, _, lo, hi) in zip(self.adj, r.pieces)]
                self.local_sweep = self._binned_sweep
            elif mode == "gather":
                self.local_sweep = self._hip_sweep
            else:
                raise ValueError(f"unknown sweep mode {mode!r}")
            self.mode = mode
        else:
            self.device = torch.device("cpu") if device is None else device
            self.adj = adj_rows
            if self.adj is not None:
                self._check_adj()
            self.local_sweep = local_sweep
            self.mode = "custom"
        self.buf = [torch.zeros(r.words_padded, dtype=torch.int64, device=self.device) for _ in range(2)]
        self.cnt = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.cur = 0

    def _check_adj(self):
        for a, (_, _, lo, hi) in zip(self.adj, self.range.pieces):
            if tuple(a.shape) != (hi - lo, self.d):
                raise ValueError(f"rank {self.rank} owns rows [{lo}, {hi}): adjacency must be "
                                 f"({hi - lo}, {self.d}), got {tuple(a.shape)}")

    @property
    def plan(self):
        """The sweep plan of the first piece (the only one when pieces == 1)."""
        return self.plans[0] if self.plans else None

    # -- one rank's rows ------------------------------------------------------
    def _hip_sweep(self, s_in, s_out, counts, g=0):
        _, _, lo, hi = self.range.pieces[g]
        a = self.adj[g]
        _lib.call("mjx_sweep_ell_np_range", _device.ptr(a) if a.numel() else None, self.n, self.d,
                  lo, hi, _device.ptr(s_in), _device.ptr(s_out),
                  _device.ptr(counts) if counts is not None else None, _device.stream_handle())

    def _binned_sweep(self, s_in, s_out, counts, g=0):
        self.plans[g].sweep(s_in, s_out, counts)

    def drop_adjacency(self):
        """Free the ELL rows once the binned plans are built (24 GB at C5 on one GPU)."""
        if self.mode == "binned":
            self.adj = None

    def exchange(self, buf, g=0):
        """All-gather piece g of every rank into the replicated state (in place).
        Returns the pending collective (or None): the caller waits on it before
        the state is read again.  One code path for every backend: RCCL on the
        GPU runs it on its own stream so piece g+1's sweep overlaps it; gloo (the
        CPU tests) runs the identical in-place call."""
        if self.world == 1 and not self.collective:
            return None
        r = self.range
        whole, mine = buf[r.piece_words(g)], buf[r.own_words(g)]
        return self.dist.all_gather_into_tensor(whole, mine, group=self.group, async_op=True)

    # -- state ------------------------------------------------------------------
    @property
    def state_words(self):
        """Current node-packed state (padded words; tensor on this rank's device)."""
        return self.buf[self.cur]

    def set_state(self, s):
        """+-1 spins (n,) -> replicated packed state (every rank passes the same s)."""
        if self.device.type == "cuda":
            from .dynamics import pack
            bits = pack(_device.to_device(s))
            self.buf[self.cur].zero_()
            self.buf[self.cur][:bits.numel()].copy_(bits)
        else:
            self.buf[self.cur].copy_(torch.from_numpy(pack_host(s, self.range.words_padded)))

    def state(self):
        """Current +-1 spins (n,) as a numpy array."""
        return unpack_host(self.buf[self.cur].cpu().numpy(), self.n)

    # -- dynamics ---------------------------------------------------------------
    def sweep(self, count=False):
        src, dst = self.buf[self.cur], self.buf[1 - self.cur]
        if count:
            self.cnt.zero_()
        pending = []
        for g in range(self.range.npieces):
            self.local_sweep(src, dst, self.cnt if count else None, g)
            pending.append(self.exchange(dst, g))
        for w in pending:        # the next sweep reads the whole state
            if w is not None:
                w.wait()
        self.cur = 1 - self.cur

    def total_plus(self):
        """Global +1 count of the last counted sweep (one all-reduce)."""
        tot = self.cnt.clone()
        if self.world > 1 or self.collective:
            self.dist.all_reduce(tot, group=self.group)
        return int(tot.item())

    def rollout(self, steps):
        """s_endstate (code/SA_RRG.py:23-26) of the current state; returns
        sum(s_end) so that m = sum/n (code/SA_RRG.py:39-40)."""
        if steps < 1:
            raise ValueError("steps must be >= 1")
        for k in range(int(steps)):
            self.sweep(count=(k == steps - 1))
        return 2 * self.total_plus() - self.n
