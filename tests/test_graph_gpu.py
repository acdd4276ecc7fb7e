"""Device graph generation and the node-range partitioned rollout (rows a7,
(e) of SURVEY.md 8).

Generation parity with networkx is distributional (the reference's graphs
come from nx.random_regular_graph, code/SA_RRG.py:59): every graph must be
simple and d-regular, generation must be deterministic per seed and
row-range independent, and its triangle count must match the random-regular
law (mean (d-1)^3/6).  The partitioned sweep is bit-exact against the
single-GPU rollout and the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import majority as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,n", [(3, 1000), (4, 1000), (6, 1000), (4, 100_000), (3, 64), (5, 10)])
def test_device_rrg_is_simple_and_regular(mjx_mod, d, n):
    adj = mjx_mod.random_regular_rows_device(d, n, seed=d * n).cpu().numpy()
    assert adj.shape == (n, d)
    rows = np.arange(n)[:, None]
    assert not np.any(adj == rows), "self loop"
    srt = np.sort(adj, axis=1)
    assert not np.any(srt[:, 1:] == srt[:, :-1]), "multi-edge"
    assert np.array_equal(np.bincount(adj.reshape(-1), minlength=n), np.full(n, d))
    fwd = np.sort(np.repeat(np.arange(n), d) * n + adj.reshape(-1))
    bwd = np.sort(adj.reshape(-1).astype(np.int64) * n + np.repeat(np.arange(n), d))
    assert np.array_equal(fwd, bwd), "asymmetric"
    g = mjx_mod.Graph.ell(torch.from_numpy(adj).cuda())
    assert mjx_mod.check_ell(g) == (0, 0, 0)


def test_device_rrg_deterministic_and_row_range_independent(mjx_mod):
    d, n = 4, 5000
    full = mjx_mod.random_regular_rows_device(d, n, seed=11)
    assert torch.equal(full, mjx_mod.random_regular_rows_device(d, n, seed=11))
    assert not torch.equal(full, mjx_mod.random_regular_rows_device(d, n, seed=12))
    for (lo, hi) in ((0, 64), (64, 1000), (1000, 4999), (4999, 5000), (2500, 2500)):
        part = mjx_mod.random_regular_rows_device(d, n, seed=11, row_lo=lo, row_hi=hi)
        assert torch.equal(part, full[lo:hi])


def test_device_rrg_triangle_law(mjx_mod):
    """Triangles of a random d-regular graph are asymptotically Poisson with mean
    (d-1)^3/6 (4.5 at d=4): the mean over 12 graphs must be close."""
    d, n = 4, 20000
    tri = []
    for seed in range(12):
        adj = mjx_mod.random_regular_rows_device(d, n, seed=seed).cpu().numpy().astype(np.int64)
        nb = [set(r) for r in adj.tolist()]
        t = 0
        for u in range(n):
            for v in adj[u]:
                if v > u:
                    t += len(nb[u] & nb[v])
        tri.append(t / 3)
    assert abs(np.mean(tri) - (d - 1) ** 3 / 6) < 1.6, tri


def test_device_rrg_large_is_simple(mjx_mod):
    n, d = 10_000_000, 6
    g = mjx_mod.random_regular_graph_device(d, n, seed=1)
    assert g.adj.shape == (n, d)
    assert mjx_mod.check_ell(g) == (0, 0, 0)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partitioned_sweeps_equal_single_gpu(mjx_mod, world):
    """Every rank's rows swept into one shared state buffer (what the in-place
    all-gather assembles) equals the single-graph rollout, bit for bit."""
    n, d, T, seed = 100_003 + 1, 6, 3, 5
    full = mjx_mod.random_regular_graph_device(d, n, seed=seed)
    rng = np.random.default_rng(0)
    s0 = 2 * rng.integers(0, 2, n).astype(np.int64) - 1
    want_bits = mjx_mod.rollout(full, mjx_mod.pack(s0), T)
    ranges = [mjx_mod.NodeRange(n, world, r) for r in range(world)]
    rows = [mjx_mod.random_regular_rows_device(d, n, seed=seed, row_lo=r.lo, row_hi=r.hi) for r in ranges]
    W = ranges[0].words_padded
    cur = torch.zeros(W, dtype=torch.int64, device="cuda")
    b0 = mjx_mod.pack(s0)
    cur[:b0.numel()] = b0
    lib = mjx_mod.load_library()
    for k in range(T):
        nxt = torch.zeros_like(cur)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        for r, a in zip(ranges, rows):
            rc = lib.mjx_sweep_ell_np_range(a.data_ptr() if a.numel() else None, n, d, r.lo, r.hi, cur.data_ptr(),
                                            nxt.data_ptr(), cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0
        cur = nxt
    assert torch.equal(cur[:want_bits.numel()], want_bits)
    assert int(cnt.item()) == int((mjx_mod.unpack(want_bits, n) > 0).sum())
    want = orc.s_endstate(full.adj.cpu().numpy(), s0, T, 1)
    assert np.array_equal(mjx_mod.unpack(cur[:want_bits.numel()], n).cpu().numpy(), want)


@pytest.mark.parametrize("mode,pieces", [("binned", 1), ("binned", 3), ("gather", 1), ("gather", 4)])
def test_sharded_rrg_single_rank(mjx_mod, mode, pieces):
    n, d = 50_000, 6
    sh = mjx_mod.ShardedRRG(d, n, seed=3, mode=mode, pieces=pieces)
    g = mjx_mod.random_regular_graph_device(d, n, seed=3)
    s0 = 2 * np.random.default_rng(1).integers(0, 2, n).astype(np.int64) - 1
    sh.set_state(s0)
    tot = sh.rollout(4)
    want = mjx_mod.s_endstate(g, s0, 4, 1)
    assert np.array_equal(sh.state(), want)
    assert tot == int(want.sum())


def test_range_sweep_argument_checks(mjx_mod):
    lib = mjx_mod.load_library()
    EINVAL = 1
    assert lib.mjx_sweep_ell_np_range(None, 1000, 4, 10, 100, None, None, None, None) == EINVAL   # unaligned lo
    assert lib.mjx_sweep_ell_np_range(None, 1000, 4, 64, 100, None, None, None, None) == EINVAL   # unaligned hi
    assert lib.mjx_sweep_ell_np_range(None, 1000, 4, 1000, 1000, None, None, None, None) == 0     # empty rank


@pytest.mark.parametrize("n,d,world", [(100_000, 6, 1), (100_037 + 1, 3, 3), (40_000_000, 3, 2), (5000, 4, 8),
                                        (3_000_000, 16, 1), (2_500_002, 5, 4)])
@pytest.mark.parametrize("form", ["flat", "segments"])
def test_binned_sweep_equals_gather_sweep(mjx_mod, n, d, world, form):
    """The source-binned plan (several 1M-node source blocks and 64K-node
    destination tiles from n = 2.5e6 on) gives the gather sweep's words and
    counts for every rank's rows; d = 16 fills the byte counters to the top.
    Both phase-2 forms (flat tile stream, per-segment loop) are run, selected
    by the ABI's apply_form argument."""
    seed = 9
    ranges = [mjx_mod.NodeRange(n, world, r) for r in range(world)]
    lib = mjx_mod.load_library()
    st = torch.cuda.current_stream().cuda_stream
    W = ranges[0].words_padded
    s_in = torch.randint(-2 ** 62, 2 ** 62, (W,), dtype=torch.int64, device="cuda")
    want = torch.zeros_like(s_in)
    got = torch.zeros_like(s_in)
    cw = torch.zeros(1, dtype=torch.int64, device="cuda")
    cg = torch.zeros(1, dtype=torch.int64, device="cuda")
    for r in ranges:
        rows = mjx_mod.random_regular_rows_device(d, n, seed=seed, row_lo=r.lo, row_hi=r.hi)
        sh = mjx_mod.ShardedRRG(d, n, adj_rows=rows, mode="binned") if world == 1 else None
        if r.hi == r.lo:
            continue
        assert lib.mjx_sweep_ell_np_range(rows.data_ptr(), n, d, r.lo, r.hi, s_in.data_ptr(), want.data_ptr(),
                                          cw.data_ptr(), st) == 0
        # a plan per rank range, built through the same entry points ShardedRRG uses
        plan = mjx_mod.BinnedPlan(rows, n, d, r.lo, r.hi)
        plan.sweep(s_in, got, cg, apply_form=form)
        if sh is not None:
            out = torch.zeros_like(s_in)
            c3 = torch.zeros(1, dtype=torch.int64, device="cuda")
            sh.local_sweep(s_in, out, c3)
            assert torch.equal(out, want) and int(c3.item()) == int(cw.item())
    assert torch.equal(got, want)
    assert int(cg.item()) == int(cw.item())
