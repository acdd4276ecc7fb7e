"""The source-binned plan's layout, restated in numpy (oracle/binned.py), on
CPU: a sweep through the plan's segments is onestep_majority
(code/SA_RRG.py:18-20) on the rows of a node range, and the index obeys the
format's alignment rules.  The device plan is compared with this restatement
segment for segment in tests/test_binned_plan_gpu.py."""
import numpy as np
import pytest

from oracle import binned as ob
from oracle import majority as orc


def multigraph(n, d, seed):
    """A d-regular multigraph by the configuration model (random stub pairing;
    self-loops and repeated edges allowed: the plan and the rule do not care)."""
    rng = np.random.default_rng(seed)
    stubs = rng.permutation(n * d)
    part = np.empty(n * d, dtype=np.int64)
    part[stubs[0::2]] = stubs[1::2]
    part[stubs[1::2]] = stubs[0::2]
    return (part // d).reshape(n, d)


N, D = (1 << 21) + 12_347 - 1, 6          # three 1M-node source blocks, n*d even


@pytest.fixture(scope="module")
def graph():
    return multigraph(N, D, 3)


@pytest.mark.parametrize("lo,hi", [(0, N), (64 * 7, 64 * 20_000), (64 * 20_000, N)])
def test_plan_sweep_is_onestep_majority(graph, lo, hi):
    s = 2 * np.random.default_rng(lo).integers(0, 2, N).astype(np.int64) - 1
    want = orc.onestep_majority(graph, s)[lo:hi]
    got = ob.sweep(graph[lo:hi], N, D, lo, hi, s)
    assert np.array_equal(got, want)


def test_plan_index_layout(graph):
    lo, hi = 0, N
    K, T, cnt, blk, p1T, p2 = ob.plan_index(graph[lo:hi], N, D, lo, hi)
    assert K == 3 and T == (N + 65535) // 65536
    assert cnt.sum() == N * D
    assert np.all(blk % 512 == 0) and np.all(np.diff(blk) >= 0)
    assert np.all(p1T % 8 == 0)
    starts = p2[:-1] & ~7
    assert np.all(starts % 8 == 0) and np.all(np.diff(starts) >= 0)
    pad = (cnt.T.reshape(-1) + 7) & ~7
    assert np.array_equal(p2[:-1] & 7, pad - cnt.T.reshape(-1))
    assert p2[-1] == pad.sum()
    # a block's segments tile its run: segment (b, t+1) starts where (b, t)'s padding ends
    p1 = p1T.reshape(T, K).T
    assert np.array_equal(p1[:, 1:], p1[:, :-1] + ((cnt[:, :-1] + 7) & ~7))
    assert np.array_equal(p1[:, 0], blk[:K])
    segs = ob.segments(graph[lo:hi], N, D, lo, hi)
    assert sum(v.size for v in segs.values()) == N * D
    for (b, t), keys in segs.items():
        assert keys.size == cnt[b, t]
