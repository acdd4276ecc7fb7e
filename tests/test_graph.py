"""Host graph builders (CPU only): distributional parity with networkx, shape
and simplicity invariants."""
import numpy as np
import pytest


@pytest.mark.parametrize("d,n", [(3, 100), (4, 1000), (6, 5000), (4, 100000)])
def test_random_regular_graph_is_simple_and_regular(mjx_mod, d, n):
    adj = mjx_mod.random_regular_graph(d, n, seed=3)
    assert adj.shape == (n, d) and adj.dtype == np.int32
    rows = np.arange(n)[:, None]
    assert not np.any(adj == rows), "self loop"
    srt = np.sort(adj, axis=1)
    assert not np.any(srt[:, 1:] == srt[:, :-1]), "multi-edge"
    # symmetric: every (i, j) has (j, i)
    src = np.repeat(np.arange(n), d)
    fwd = set(zip(src.tolist(), adj.reshape(-1).tolist()))
    assert all((j, i) in fwd for (i, j) in list(fwd)[:5000])
    assert np.bincount(adj.reshape(-1), minlength=n).tolist() == [d] * n


def test_random_regular_graph_rejects_odd(mjx_mod):
    with pytest.raises(ValueError):
        mjx_mod.random_regular_graph(3, 7)


def test_erdos_renyi_degree_distribution(mjx_mod):
    n, c = 200000, 5.0
    rp, col = mjx_mod.erdos_renyi(n, c / (n - 1), seed=1)
    deg = np.diff(rp)
    assert abs(deg.mean() - c) < 0.05
    assert abs(deg.var() - c) < 0.15          # Poisson(5): variance ~ 5
    assert abs((deg == 0).mean() - np.exp(-c)) < 0.002
    # no self loops, symmetric
    src = np.repeat(np.arange(n), deg)
    assert not np.any(src == col)
    key_f = src.astype(np.int64) * n + col
    key_b = col.astype(np.int64) * n + src
    assert np.array_equal(np.sort(key_f), np.sort(key_b))


def test_remove_isolated_relabels(mjx_mod):
    u = np.array([0, 5, 5])
    v = np.array([5, 7, 9])
    n2, u2, v2, iso = mjx_mod.remove_isolated(10, u, v)
    assert n2 == 4 and iso == 6
    assert u2.tolist() == [0, 1, 1] and v2.tolist() == [1, 2, 3]


def test_neighbours_matches_reference_layout(mjx_mod):
    nx = pytest.importorskip("networkx")
    import random
    random.seed(5)
    G = nx.random_regular_graph(4, 50)
    N = mjx_mod.neighbours(G)
    for i in range(50):
        assert N[i].tolist() == list(G.neighbors(i))
