"""GPU parity of the majority rollout kernels (rows a1-a4 of SURVEY.md 8a).

Bar: bit-exact.  Small cases against the reference's golden vectors; larger
seeded cases against the CPU oracle; full-size cases through
size-independent properties.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import majority as orc

pytestmark = pytest.mark.gpu

PC = [(1, 1), (2, 1), (2, 2), (3, 1)]


@pytest.mark.parametrize("d", [3, 4, 6])
@pytest.mark.parametrize("n", [64, 1000])
def test_rrg_rollout_golden(mjx_mod, d, n):
    z = load_golden("rrg_dyn.npz")
    key = f"d{d}_n{n}"
    N, S0 = z[f"{key}_N"], z[f"{key}_s0"]
    g = mjx_mod.Graph.ell(N)
    for (p, c) in PC:
        want = z[f"{key}_p{p}c{c}"]
        # single replica, node-packed layout
        for r in range(S0.shape[0]):
            got = mjx_mod.s_endstate(g, S0[r], p, c)
            assert got.dtype == np.int64
            assert np.array_equal(got, want[r]), (p, c, r)
        # batch of replicas, replica-packed layout
        assert np.array_equal(mjx_mod.s_endstate(g, S0, p, c), want)
    # numpy-array adjacency straight in (drop-in signature)
    assert np.array_equal(mjx_mod.onestep_majority(N, S0[0]), z[f"{key}_p1c1"][0])


def test_torch_inputs_like_hpr(mjx_mod):
    """code/HPR_pytorch_RRG.py passes int32 tensors; results come back as
    tensors on the caller's device."""
    z = load_golden("rrg_dyn.npz")
    N, S0 = z["d4_n1000_N"], z["d4_n1000_s0"]
    s = torch.tensor(S0[1], dtype=torch.int32, device="cuda")
    out = mjx_mod.s_endstate(torch.tensor(N, dtype=torch.int32), s, 2, 2)
    assert isinstance(out, torch.Tensor) and out.is_cuda
    assert np.array_equal(out.cpu().numpy(), z["d4_n1000_p2c2"][1])


def test_er_rollout_golden(mjx_mod):
    z = load_golden("er_dyn.npz")
    keys = sorted(k[:-len("_row_ptr")] for k in z if k.endswith("_row_ptr"))
    for key in keys:
        g = mjx_mod.Graph.csr(z[f"{key}_row_ptr"], z[f"{key}_col"])
        S0 = z[f"{key}_s0"]
        for (p, c) in PC:
            want = z[f"{key}_p{p}c{c}"]
            assert np.array_equal(mjx_mod.s_endstate(g, S0, p, c), want), (key, p, c)
            assert np.array_equal(mjx_mod.s_endstate(g, S0[0], p, c), want[0]), (key, p, c)


@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 6, 7, 8, 10])
@pytest.mark.parametrize("R", [1, 64, 100, 128, 192])
def test_rollout_vs_oracle_random(mjx_mod, d, R):
    """Generic-degree and specialised kernels, ragged replica counts
    (R not a multiple of 64 -> padding replicas) and n not a multiple of 64."""
    n = 1234 if d % 2 == 0 else 1236
    if (n * d) % 2:
        n += 1
    adj = mjx_mod.random_regular_graph(d, n, seed=d * 31 + R)
    rng = np.random.default_rng(R + d)
    S0 = 2 * rng.integers(0, 2, size=(R, n)).astype(np.int64) - 1
    g = mjx_mod.Graph.ell(adj)
    for T in (0, 1, 2, 3):
        want = orc.s_endstate_batch(adj, S0, T, 1)
        got = mjx_mod.s_endstate(g, S0 if R > 1 else S0[0], T, 1)
        assert np.array_equal(got.reshape(want.shape), want), (d, R, T)


def test_er_with_isolated_and_high_degree(mjx_mod):
    n = 3000
    rng = np.random.default_rng(0)
    # skewed degrees incl. isolated nodes and a hub of degree 200
    u = rng.integers(0, n, 6000)
    v = rng.integers(0, n, 6000)
    keep = u != v
    u, v = u[keep], v[keep]
    hub_u = np.zeros(200, np.int64) + 7
    hub_v = rng.choice(np.arange(8, n), 200, replace=False)
    key = np.unique(np.minimum(np.r_[u, hub_u], np.r_[v, hub_v]) * n + np.maximum(np.r_[u, hub_u], np.r_[v, hub_v]))
    rp, col = mjx_mod.csr_from_edges(n, key // n, key % n)
    assert (np.diff(rp) == 0).any()
    S0 = 2 * rng.integers(0, 2, size=(130, n)).astype(np.int64) - 1
    g = mjx_mod.Graph.csr(rp, col)
    for T in (1, 2, 5):
        want = orc.s_endstate_er(rp, col, S0, T, 1)
        assert np.array_equal(mjx_mod.s_endstate(g, S0, T, 1), want)
        assert np.array_equal(mjx_mod.s_endstate(g, S0[3], T, 1), want[3])


@pytest.mark.parametrize("R", [64, 128, 192, 4096])
def test_class_ell_equals_csr_layout(mjx_mod, R):
    """The degree-class ELL sweep (nb:113-117's per-class layout; every class
    kernel D = 0..8 and the runtime-degree one) against the CSR sweep and the
    oracle, fused counts included; W odd (R=192) takes the 8-byte units."""
    n = 2500
    rng = np.random.default_rng(R)
    u, v = rng.integers(0, n, 5000), rng.integers(0, n, 5000)
    hub_u = np.zeros(40, np.int64) + 11
    hub_v = rng.choice(np.arange(12, n), 40, replace=False)
    a, b = np.r_[u, hub_u], np.r_[v, hub_v]
    keep = a != b
    key = np.unique(np.minimum(a, b)[keep] * n + np.maximum(a, b)[keep])
    rp, col = mjx_mod.csr_from_edges(n, key // n, key % n)
    degs = set(np.diff(rp).tolist())
    assert set(range(9)) <= degs and max(degs) > 8
    g = mjx_mod.Graph.csr(rp, col)
    order, cell, classes = g.class_ell()
    assert classes[:, 1].sum() == n and (classes[:, 3] % 4 == 0).all()
    o = order.cpu().numpy()
    c = cell.cpu().numpy()
    for i0, cnt, D, base in classes:           # rows of the class cells are the CSR rows
        for k in (0, cnt // 2, cnt - 1):
            vtx = o[i0 + k]
            assert D == rp[vtx + 1] - rp[vtx]
            assert np.array_equal(c[base + k * D: base + k * D + D], col[rp[vtx]:rp[vtx + 1]])
    W = (R + 63) // 64
    S0 = 2 * rng.integers(0, 2, size=(R, n)).astype(np.int64) - 1
    bits = mjx_mod.pack(S0)
    for T in (1, 2, 3):
        res = {}
        for layout in ("class", "csr"):
            g.rp_layout = layout
            cnt = torch.zeros(W * 64, dtype=torch.int64, device="cuda")
            out = mjx_mod.rollout(g, bits, T, words=W, counts=cnt)
            res[layout] = (out.cpu().numpy(), cnt.cpu().numpy())
        g.rp_layout = "class"
        assert np.array_equal(res["class"][0], res["csr"][0]), T
        assert np.array_equal(res["class"][1], res["csr"][1]), T
        want = orc.s_endstate_er(rp, col, S0, T, 1)
        assert np.array_equal(res["class"][1][:R], (want > 0).sum(axis=1)), T
        assert np.array_equal(mjx_mod.s_endstate(g, S0, T, 1), want), T


def test_pack_unpack_roundtrip(mjx_mod):
    rng = np.random.default_rng(1)
    for (R, n) in [(1, 1), (1, 65), (3, 1000), (64, 777), (65, 300), (4096, 50)]:
        S = 2 * rng.integers(0, 2, size=(R, n)).astype(np.int64) - 1
        for dt in (torch.int8, torch.int32, torch.int64):
            t = torch.tensor(S, dtype=dt, device="cuda")
            if R == 1:
                b = mjx_mod.pack(t[0])
                assert torch.equal(mjx_mod.unpack(b, n, dtype=dt), t[0])
            b = mjx_mod.pack(t)
            assert b.numel() == n * ((R + 63) // 64)
            assert torch.equal(mjx_mod.unpack(b, n, R, dtype=dt), t)


def test_popcount_counts(mjx_mod):
    rng = np.random.default_rng(2)
    for (R, n) in [(1, 100), (64, 300), (200, 5000), (4096, 1000), (16384, 70)]:
        S = 2 * rng.integers(0, 2, size=(R, n)).astype(np.int64) - 1
        b = mjx_mod.pack(torch.tensor(S, device="cuda"))
        W = (R + 63) // 64
        cnt = mjx_mod.popcount(b, n, words=W).cpu().numpy()
        assert np.array_equal(cnt[:R], (S > 0).sum(axis=1))
        assert not cnt[R:].any()
        if R == 1:
            b1 = mjx_mod.pack(torch.tensor(S[0], device="cuda"))
            assert int(mjx_mod.popcount(b1, n).item()) == int((S[0] > 0).sum())


@pytest.mark.parametrize("R", [64, 4096, 16384])
def test_fused_count_equals_popcount(mjx_mod, R):
    n = 20000
    adj = mjx_mod.random_regular_graph(3, n, seed=R)
    g = mjx_mod.Graph.ell(adj)
    W = R // 64
    gen = torch.Generator(device="cuda").manual_seed(R)
    bits = torch.randint(-2 ** 62, 2 ** 62, (n * W,), device="cuda", generator=gen)
    cnt = torch.zeros(R, dtype=torch.int64, device="cuda")
    out = mjx_mod.rollout(g, bits, 2, words=W, counts=cnt)
    ref = mjx_mod.popcount(out, n, words=W)
    assert torch.equal(cnt, ref)
    # rollout(2) == rollout(1) twice
    o1 = mjx_mod.rollout(g, bits, 1, words=W)
    o2 = mjx_mod.rollout(g, o1, 1, words=W)
    assert torch.equal(o2, out)


def test_full_size_properties_d4(mjx_mod):
    """Bench-size graph (N=1e6, d=4, R=4096): consensus states are fixed
    points, the replica-packed and node-packed kernels agree on sampled
    replicas, and the spin-flip symmetry s -> -s commutes with the dynamics."""
    n, d, R = 10 ** 6, 4, 4096
    W = R // 64
    adj = mjx_mod.random_regular_graph(d, n, seed=0)
    g = mjx_mod.Graph.ell(adj)
    ones = torch.full((n * W,), -1, dtype=torch.int64, device="cuda")   # all bits set = all +1
    cnt = torch.zeros(R, dtype=torch.int64, device="cuda")
    out = mjx_mod.rollout(g, ones, 3, words=W, counts=cnt)
    assert torch.equal(out, ones) and bool((cnt == n).all())
    gen = torch.Generator(device="cuda").manual_seed(0)
    bits = torch.randint(-2 ** 62, 2 ** 62, (n * W,), device="cuda", generator=gen)
    out = mjx_mod.rollout(g, bits, 2, words=W)
    neg = mjx_mod.rollout(g, ~bits, 2, words=W)
    assert torch.equal(neg, ~out)
    # replica r of the packed rollout == node-packed rollout of replica r alone
    S = mjx_mod.unpack(bits.view(n, W)[:, :1].contiguous(), n, 64)   # first 64 replicas
    outS = mjx_mod.unpack(out.view(n, W)[:, :1].contiguous(), n, 64)
    for r in (0, 17, 63):
        single = mjx_mod.rollout(g, mjx_mod.pack(S[r]), 2)
        assert torch.equal(mjx_mod.unpack(single, n), outS[r])
    # oracle on a sample replica (numpy, ~1 s)
    want = orc.s_endstate(adj, S[5].cpu().numpy(), 2, 1)
    assert np.array_equal(outS[5].cpu().numpy(), want)


def test_numpy_neighbour_array_uploaded_once(mjx_mod):
    """The drop-in onestep_majority(N, s) with the reference's numpy N reuses
    the device adjacency across calls on the same array; a different array
    (or new contents) is uploaded again and still gives the oracle's result."""
    from oracle import majority as orc
    N = mjx_mod.random_regular_graph(4, 1000, seed=3).astype(np.int64)
    g1 = mjx_mod.as_graph(N)
    assert mjx_mod.as_graph(N) is g1
    s = 2 * np.random.default_rng(0).integers(0, 2, 1000).astype(np.int64) - 1
    for _ in range(3):
        assert np.array_equal(mjx_mod.onestep_majority(N, s), orc.onestep_majority(N, s))
    assert mjx_mod.as_graph(N) is g1
    N2 = mjx_mod.random_regular_graph(4, 1000, seed=4).astype(np.int64)
    assert mjx_mod.as_graph(N2) is not g1
    assert np.array_equal(mjx_mod.s_endstate(N2, s, 2, 1), orc.s_endstate(N2, s, 2, 1))


def test_class_sweep_long_degree_tail(mjx_mod):
    """About 90 degree classes: the counting sweep runs the D <= 8 classes in
    one launch (k_sweep_cls_all_rp) and the long D > 8 tail as several
    32-class table launches (k_sweep_cls_gen_rp); rollout and fused counts
    equal the oracle."""
    n, R = 3000, 128
    rng = np.random.default_rng(9)
    a, b = [], []
    for hub in range(90):                      # hub h gets h + 1 extra neighbours -> ~90 distinct degrees
        nb = rng.choice(np.arange(100, n), hub + 1, replace=False)
        a += [hub] * len(nb)
        b += nb.tolist()
    u, v = rng.integers(100, n, 4000), rng.integers(100, n, 4000)
    a, b = np.r_[a, u], np.r_[b, v]
    keep = a != b
    key = np.unique(np.minimum(a, b)[keep] * n + np.maximum(a, b)[keep])
    rp, col = mjx_mod.csr_from_edges(n, key // n, key % n)
    g = mjx_mod.Graph.csr(rp, col)
    _, _, classes = g.class_ell()
    assert len(classes) > 64
    W = R // 64
    S0 = 2 * rng.integers(0, 2, size=(R, n)).astype(np.int64) - 1
    bits = mjx_mod.pack(S0)
    for T in (1, 2):
        cnt = torch.zeros(R, dtype=torch.int64, device="cuda")
        out = mjx_mod.rollout(g, bits, T, words=W, counts=cnt)
        want = orc.s_endstate_er(rp, col, S0, T, 1)
        assert np.array_equal(cnt.cpu().numpy(), (want > 0).sum(axis=1)), T
        assert torch.equal(out, mjx_mod.pack(want)), T
