"""Device Erdos-Renyi generator (mjx_er_generate).

The notebook draws nx.erdos_renyi_graph(n, p) (code/ER_BDCM_entropy.ipynb,
nb:278-282) and drops isolated nodes with an order-preserving relabelling
(nb:283-291).  networkx is absent here, so parity is distributional: the CSR
must be a simple undirected graph with sorted rows, the edge count must follow
Binomial(n(n-1)/2, p), degrees Poisson(np) in the sparse regime, generation
deterministic per seed, and isolate removal must equal the host restatement
(mjx.remove_isolated) applied to the device's own edge list.  Dynamics on the
device CSR are bit-exact against the oracle.
"""
import math

import numpy as np
import pytest
import torch

from oracle import majority as orc

pytestmark = pytest.mark.gpu


def _host(g):
    return g.row_ptr.cpu().numpy(), g.col.cpu().numpy()


def _check_simple_sorted(rp, col, n):
    assert rp[0] == 0 and rp[-1] == col.size and np.all(np.diff(rp) >= 0)
    assert col.size == 0 or (col.min() >= 0 and col.max() < n)
    row = np.repeat(np.arange(n), np.diff(rp))
    assert not np.any(col == row), "self loop"
    # sorted strictly ascending inside every row (no multi-edges)
    same = row[1:] == row[:-1]
    assert np.all(col[1:][same] > col[:-1][same])
    fwd = np.sort(row.astype(np.int64) * n + col)
    bwd = np.sort(col.astype(np.int64) * n + row)
    assert np.array_equal(fwd, bwd), "not symmetric"


@pytest.mark.parametrize("n,mean_deg", [(1000, 5.0), (100_000, 5.0), (20_000, 1.0), (3000, 40.0), (1, 0.0)])
def test_er_simple_symmetric_sorted(mjx_mod, n, mean_deg):
    p = mean_deg / max(n - 1, 1)
    g = mjx_mod.erdos_renyi_device(n, p, seed=n)
    rp, col = _host(g)
    assert g.n == n
    _check_simple_sorted(rp, col, n)


def test_er_edge_count_and_degree_law(mjx_mod):
    n, c = 1_000_000, 5.0
    p = c / (n - 1)
    g = mjx_mod.erdos_renyi_device(n, p, seed=7)
    rp, col = _host(g)
    m = col.size // 2
    mean = n * (n - 1) / 2 * p
    sd = math.sqrt(mean * (1 - p))
    assert abs(m - mean) < 6 * sd, (m, mean, sd)
    deg = np.diff(rp)
    for k in range(0, 11):   # Poisson(c) frequencies, 6 sigma of the binomial count
        want = n * math.exp(-c) * c ** k / math.factorial(k)
        got = int((deg == k).sum())
        assert abs(got - want) < 6 * math.sqrt(want) + 5, (k, got, want)
    # pairs are uniform over i < j: the span |i - j| of an edge is ~ uniform pair distance
    row = np.repeat(np.arange(n), deg)
    span = np.abs(col.astype(np.int64) - row)
    assert abs(span.mean() / (n / 3) - 1) < 0.01


def test_er_deterministic_per_seed(mjx_mod):
    n, p = 50_000, 5.0 / 49_999
    a = _host(mjx_mod.erdos_renyi_device(n, p, seed=3))
    b = _host(mjx_mod.erdos_renyi_device(n, p, seed=3))
    c = _host(mjx_mod.erdos_renyi_device(n, p, seed=4))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert not (a[1].size == c[1].size and np.array_equal(a[1], c[1]))


@pytest.mark.parametrize("n,mean_deg", [(30_000, 1.0), (5000, 3.0)])
def test_er_drop_isolated_matches_host_relabelling(mjx_mod, n, mean_deg):
    p = mean_deg / (n - 1)
    full = mjx_mod.erdos_renyi_device(n, p, seed=11)
    rp, col = _host(full)
    row = np.repeat(np.arange(n), np.diff(rp))
    up = row < col
    n2, u2, v2, iso = mjx_mod.remove_isolated(n, row[up], col[up])
    want_rp, want_col = mjx_mod.csr_from_edges(n2, u2, v2)
    g, iso_dev = mjx_mod.erdos_renyi_device(n, p, seed=11, drop_isolated=True)
    got_rp, got_col = _host(g)
    assert iso_dev == iso and g.n == n2
    assert np.array_equal(got_rp, want_rp)
    # csr_from_edges' in-row order may differ; compare sorted rows
    srt = np.concatenate([np.sort(want_col[want_rp[i]:want_rp[i + 1]]) for i in range(n2)]) if n2 else want_col
    assert np.array_equal(got_col, srt)
    assert np.all(np.diff(got_rp) > 0)


def test_er_dynamics_on_device_csr_match_oracle(mjx_mod):
    n, p = 20_000, 5.0 / 19_999
    g = mjx_mod.erdos_renyi_device(n, p, seed=5)
    rp, col = _host(g)
    rng = np.random.default_rng(2)
    S0 = 2 * rng.integers(0, 2, size=(64, n)).astype(np.int64) - 1
    got = mjx_mod.s_endstate(g, S0, 2, 1)
    for r in (0, 17, 63):
        assert np.array_equal(got[r], orc.s_endstate_er(rp, col, S0[r], 2, 1))


def test_gather_floor_moves_the_class_sweep_rows(mjx_mod):
    """The measurement kernel behind bench.py's er.floor_ms
    (mjx_gather_floor_class) reads exactly a class sweep's rows: row v of its
    output is the XOR of v's neighbour rows, and of v's own row where deg(v)
    is even (nb:113-117: the own spin only breaks ties, which need an even
    degree) -- on a device ER graph with isolated nodes and a D > 8 tail."""
    from mjx import _lib as L, _device as D
    n, W = 20_000, 2
    g = mjx_mod.erdos_renyi_device(n, 6.0 / (n - 1), seed=5)          # ~50 isolated nodes, a D > 8 tail
    order, cell, classes = g.class_ell()
    assert int(classes[:, 2].max()) > 8 and int(classes[0, 2]) == 0
    s = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda")
    out = torch.zeros_like(s)
    L.call("mjx_gather_floor_class", D.ptr(order), D.ptr(cell), classes.ctypes.data, classes.shape[0], n, W,
           D.ptr(s), D.ptr(out), D.stream_handle())
    rp, col = g.row_ptr.cpu().numpy(), g.col.cpu().numpy()
    sh = s.view(n, W).cpu().numpy()
    want = np.zeros_like(sh)
    deg = np.diff(rp)
    for v in range(n):
        acc = np.bitwise_xor.reduce(sh[col[rp[v]:rp[v + 1]]], axis=0) if deg[v] else np.zeros(W, dtype=np.int64)
        if deg[v] % 2 == 0:
            acc = acc ^ sh[v]
        want[v] = acc
    assert np.array_equal(out.view(n, W).cpu().numpy(), want)
