"""ORACLE (test infrastructure only): numpy restatement of the source-binned
sweep plan of one node range of a giant graph (configs[4], SURVEY.md 8a rows
a1/a3 at N=1e9; the device side is mjx_binned_build / mjx_sweep_binned in
csrc/mjx_graph.hip).

The plan is a re-layout of the (destination v, source u) slots of the rows
[lo, hi) of the adjacency the reference stores as N (code/SA_RRG.py:9-16);
a sweep through it computes onestep_majority (code/SA_RRG.py:18-20).  Layout
restated here, from the format described in csrc/mjx_graph.hip:
  * source block b = u >> 20, destination tile t = (v - lo) >> 16; segment
    (b, t) = the slots with that pair; every segment padded to 8 slots;
  * phase-1 order: b-major, t inside, each block's run padded to 512 slots:
    blk[b] (K+1 starts), p1T[t*K + b] = the segment's phase-1 start;
  * phase-2 order: t-major, b inside: p2[t*K + b] = padded start | pad count
    in the low 3 bits, p2[S] = the total;
  * the phase-1 stream: per 512-slot chunk, 512 16-bit words (u & 0xfffff) >> 4
    then 128 16-bit entries of four 4-bit bit positions (u & 15);
  * off (phase-2 order): the destination's offset inside its tile, 16 bits.
Slot order inside a segment is free (the device ranks by LDS atomics), so the
checker compares each segment's (source offset, destination offset) pairs as
a sorted list; pad and block-tail slots are zero.
"""
import numpy as np

SRC_SHIFT, TILE_SHIFT, CHUNK = 20, 16, 512
CHUNK_U16 = CHUNK + CHUNK // 4


def plan_index(adj_rows, n, d, lo, hi):
    """(K, T, counts (K, T), blk (K+1,), p1T (S,), p2 (S+1,)) of the rows
    [lo, hi): adj_rows is (hi - lo, d) of global node ids."""
    rows = hi - lo
    K = (n + (1 << SRC_SHIFT) - 1) >> SRC_SHIFT
    T = (rows + (1 << TILE_SHIFT) - 1) >> TILE_SHIFT
    u = np.asarray(adj_rows, dtype=np.int64).reshape(-1)
    v = np.repeat(np.arange(rows, dtype=np.int64), d)
    b, t = u >> SRC_SHIFT, v >> TILE_SHIFT
    cnt = np.bincount(b * T + t, minlength=K * T).reshape(K, T)
    pad = (cnt + 7) & ~7
    p1 = np.cumsum(pad, axis=1) - pad                      # b-major starts inside each block
    tot = pad.sum(axis=1)
    blen = (tot + CHUNK - 1) // CHUNK * CHUNK
    blk = np.concatenate([[0], np.cumsum(blen)]).astype(np.int64)
    p1T = (blk[:K, None] + p1).T.reshape(-1)               # index t*K + b
    padT = pad.T.reshape(-1)
    p2 = np.concatenate([[0], np.cumsum(padT)]).astype(np.int64)
    p2[:-1] |= (padT - cnt.T.reshape(-1))
    return K, T, cnt, blk, p1T, p2


def segments(adj_rows, n, d, lo, hi):
    """{(b, t): sorted int64 keys (u & 0xfffff) << 16 | (v - lo - t*2^16)}."""
    rows = hi - lo
    u = np.asarray(adj_rows, dtype=np.int64).reshape(-1)
    v = np.repeat(np.arange(rows, dtype=np.int64), d)
    b, t = u >> SRC_SHIFT, v >> TILE_SHIFT
    key = ((u & ((1 << SRC_SHIFT) - 1)) << 16) | (v & ((1 << TILE_SHIFT) - 1))
    T = (rows + (1 << TILE_SHIFT) - 1) >> TILE_SHIFT
    seg = b * T + t
    order = np.lexsort((key, seg))
    seg_s, key_s = seg[order], key[order]
    out = {}
    starts = np.flatnonzero(np.r_[True, seg_s[1:] != seg_s[:-1]])
    ends = np.r_[starts[1:], seg_s.size]
    for a, e in zip(starts, ends):
        s = int(seg_s[a])
        out[(s // T, s % T)] = key_s[a:e]
    return out


def decode_stream(stream, pos):
    """20-bit source offsets at phase-1 positions pos from the packed stream."""
    stream = np.asarray(stream).view(np.uint16).astype(np.int64)
    pos = np.asarray(pos, dtype=np.int64)
    c, w = pos >> 9, pos & 511
    word = stream[c * CHUNK_U16 + w]
    nib = (stream[c * CHUNK_U16 + CHUNK + (w >> 2)] >> (4 * (w & 3))) & 15
    return (word << 4) | nib


def sweep(adj_rows, n, d, lo, hi, s):
    """One majority sweep of the rows [lo, hi) through the plan's two phases
    (messages by source block, counts by destination tile, always-stay ties,
    code/SA_RRG.py:19-20): the new +-1 spins of the rows."""
    s = np.asarray(s, dtype=np.int64)
    cnt_plus = np.zeros(hi - lo, dtype=np.int64)
    for (b, t), keys in segments(adj_rows, n, d, lo, hi).items():
        src = (b << SRC_SHIFT) + (keys >> 16)              # phase 1: the message bit of every slot
        dst = (t << TILE_SHIFT) + (keys & 0xFFFF)
        np.add.at(cnt_plus, dst, (s[src] > 0).astype(np.int64))   # phase 2: +1 counts
    own = s[lo:hi]
    S = 2 * cnt_plus - d
    return np.where(S > 0, 1, np.where(S < 0, -1, own))
