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
    """Word-aligned node range of ``rank`` among ``world`` ranks: rank r owns
    words [r*chunk, (r+1)*chunk) of the padded state (chunk*world words)."""

    def __init__(self, n, world, rank):
        self.n, self.world, self.rank = int(n), int(world), int(rank)
        self.words = (self.n + 63) // 64
        self.chunk = max(1, -(-self.words // self.world))
        self.words_padded = self.chunk * self.world
        self.w_lo = min(self.words, self.rank * self.chunk)
        self.w_hi = min(self.words, (self.rank + 1) * self.chunk)
        self.lo = min(self.n, self.w_lo * 64)
        self.hi = min(self.n, self.w_hi * 64)


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

    def sweep(self, s_in, s_out, counts=None):
        _lib.call("mjx_sweep_binned", _device.ptr(self.src_lo), _device.ptr(self.src_hi), _device.ptr(self.off),
                  _device.ptr(self.index),
                  self.n, self.d, self.lo, self.hi, _device.ptr(s_in), _device.ptr(self.msg), _device.ptr(s_out),
                  _device.ptr(counts) if counts is not None else None, _device.stream_handle())


class ShardedRRG:
    """This rank's part of one d-regular graph and the replicated spin state."""

    def __init__(self, d, n, seed=0, group=None, adj_rows=None, local_sweep=None, device=None, mode="binned"):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0
        self.backend = self.dist.get_backend(group) if self.dist else None
        self.d, self.n, self.seed = int(d), int(n), int(seed)
        self.range = r = NodeRange(n, self.world, self.rank)
        if local_sweep is None:
            self.device = _device.require_gpu()
            if adj_rows is None:
                from .graph import random_regular_rows_device
                adj_rows = random_regular_rows_device(self.d, self.n, self.seed, r.lo, r.hi)
            self.adj = _device.to_device(adj_rows, dtype=torch.int32)
            if mode == "binned":
                self._build_binned()
                self.local_sweep = self._binned_sweep
            elif mode == "gather":
                self.local_sweep = self._hip_sweep
            else:
                raise ValueError(f"unknown sweep mode {mode!r}")
            self.mode = mode
        else:
            self.device = torch.device("cpu") if device is None else device
            self.adj = adj_rows
            self.local_sweep = local_sweep
            self.mode = "custom"
        if self.adj is not None and tuple(self.adj.shape) != (r.hi - r.lo, self.d):  # checked before the plan
            raise ValueError(f"rank {self.rank} owns rows [{r.lo}, {r.hi}): adjacency must be "
                             f"({r.hi - r.lo}, {self.d}), got {tuple(self.adj.shape)}")
        self.buf = [torch.zeros(r.words_padded, dtype=torch.int64, device=self.device) for _ in range(2)]
        self.cnt = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.cur = 0

    # -- one rank's rows ------------------------------------------------------
    def _hip_sweep(self, s_in, s_out, counts):
        r = self.range
        _lib.call("mjx_sweep_ell_np_range", _device.ptr(self.adj) if self.adj.numel() else None, self.n, self.d,
                  r.lo, r.hi, _device.ptr(s_in), _device.ptr(s_out),
                  _device.ptr(counts) if counts is not None else None, _device.stream_handle())

    def _build_binned(self):
        """Static source-binned plan of this rank's rows (mjx_binned_build)."""
        r = self.range
        if tuple(self.adj.shape) != (r.hi - r.lo, self.d):
            raise ValueError(f"rank {self.rank} owns rows [{r.lo}, {r.hi}): adjacency must be "
                             f"({r.hi - r.lo}, {self.d}), got {tuple(self.adj.shape)}")
        self.plan = BinnedPlan(self.adj, self.n, self.d, r.lo, r.hi)

    def _binned_sweep(self, s_in, s_out, counts):
        self.plan.sweep(s_in, s_out, counts)

    def drop_adjacency(self):
        """Free the ELL rows once the binned plan is built (24 GB at C5 on one GPU)."""
        if self.mode == "binned":
            self.adj = None

    def exchange(self, buf):
        """All-gather every rank's word slice into the replicated state (in place)."""
        if self.world == 1:
            return
        r = self.range
        mine = buf[self.rank * r.chunk:(self.rank + 1) * r.chunk]
        if self.backend == "nccl":
            self.dist.all_gather_into_tensor(buf, mine, group=self.group)
        else:
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            self.dist.all_gather(parts, mine.clone(), group=self.group)
            buf.view(self.world, r.chunk).copy_(torch.stack(parts))

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
        self.local_sweep(src, dst, self.cnt if count else None)
        self.exchange(dst)
        self.cur = 1 - self.cur

    def total_plus(self):
        """Global +1 count of the last counted sweep (one all-reduce)."""
        tot = self.cnt.clone()
        if self.world > 1:
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
