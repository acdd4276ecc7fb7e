"""The device source-binned plan (mjx_binned_build: LDS-staged quads straight
into the packed phase-1 stream and the phase-2 offsets) against the numpy
restatement of its layout (oracle/binned.py), segment for segment: the index
(blk, p1T, p2) equal, every segment's (source offset, destination offset)
pairs equal as sorted lists, every pad slot and every block's tail zero; and
the plan's sweep equals onestep_majority (code/SA_RRG.py:18-20)."""
import numpy as np
import pytest
import torch

from oracle import binned as ob
from oracle import majority as orc
from test_binned_oracle import multigraph

pytestmark = pytest.mark.gpu

N, D = (1 << 21) + 12_347 - 1, 6


@pytest.fixture(scope="module")
def graph():
    return multigraph(N, D, 3)


@pytest.mark.parametrize("lo,hi", [(0, N), (64 * 7, 64 * 20_000), (64 * 20_000, N)])
def test_device_plan_equals_oracle_segment_for_segment(mjx_mod, graph, lo, hi):
    rows = torch.from_numpy(np.ascontiguousarray(graph[lo:hi]).astype(np.int32)).cuda()
    plan = mjx_mod.BinnedPlan(rows, N, D, lo, hi)
    torch.cuda.synchronize()
    K, T, cnt, blk, p1T, p2 = ob.plan_index(graph[lo:hi], N, D, lo, hi)
    S = K * T
    index = plan.index.cpu().numpy()
    assert np.array_equal(index[:K + 1], blk)
    assert np.array_equal(index[K + 1:K + 1 + S], p1T)
    assert np.array_equal(index[K + 1 + S:K + 2 + 2 * S], p2)
    stream = plan.src_lo.cpu().numpy()
    off = plan.off.cpu().numpy().view(np.uint16).astype(np.int64)
    segs = ob.segments(graph[lo:hi], N, D, lo, hi)
    for b in range(K):
        for t in range(T):
            c = int(cnt[b, t])
            pad = (c + 7) & ~7
            a1, a2 = int(p1T[t * K + b]), int(p2[t * K + b]) & ~7
            u = ob.decode_stream(stream, np.arange(a1, a1 + pad))
            v = off[a2:a2 + pad]
            keys = np.sort((u[:c] << 16) | v[:c])
            want = segs.get((b, t), np.zeros(0, dtype=np.int64))
            assert np.array_equal(keys, want), (b, t)
            assert not u[c:].any() and not v[c:].any(), (b, t)     # pad slots
        # the block's tail after its last segment, up to the next block's start
        end = int(p1T[(T - 1) * K + b]) + ((int(cnt[b, T - 1]) + 7) & ~7)
        assert not ob.decode_stream(stream, np.arange(end, int(blk[b + 1]))).any(), b
    # and the plan's sweep is the rule
    s = 2 * np.random.default_rng(lo).integers(0, 2, N).astype(np.int64) - 1
    words = (N + 63) // 64
    s_in = torch.zeros(words + 1, dtype=torch.int64, device="cuda")
    s_in[:words] = mjx_mod.pack(s)
    out = torch.zeros_like(s_in)
    plan.sweep(s_in, out)
    got = mjx_mod.unpack(out[:words], N).cpu().numpy()[lo:hi]
    assert np.array_equal(got, orc.onestep_majority(graph, s)[lo:hi])
