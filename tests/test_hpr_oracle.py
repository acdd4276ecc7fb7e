"""Pin the HPR oracle (oracle/hpr.py) against vectors produced by the
reference's own functions (tests/golden/make_golden.py gen_hpr).  CPU only."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import hpr

CASES = sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "hpr_d*.npz")))


def test_fixtures_present():
    assert len(CASES) >= 6


@pytest.mark.parametrize("name", CASES)
def test_hpr_oracle_matches_reference(name):
    z = load_golden(name)
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    inr, src = hpr.incoming_rows(z["edges"], z["N_nodes"])
    # the reference's own index arrays (code/HPR_pytorch_RRG.py:81-118)
    assert np.array_equal(inr * 4 ** (p + c), z["N_edg_pos_chi_mat"])
    ep = hpr.edges_pos(z["edges"], z["N_nodes"])
    assert np.array_equal(ep, z["N_edges_pos"])
    chi, b = z["chi0"], z["biases0"]
    for k in range(int(z["chain"])):
        new = hpr.HPr_dp(chi, b, inr, src, n, d, p, c, int(z["attr_value"]), int(z["lmbd_in"]), float(z["damppar"]))
        ref = z[f"it{k}_chi"]
        err = np.max(np.abs(new - ref) / np.max(np.abs(ref), axis=1, keepdims=True))
        assert err < 1e-12, (k, err)
        sub = hpr.HPr_dp(chi, b, inr, src, n, d, p, c, int(z["attr_value"]), int(z["lmbd_in"]),
                         float(z["damppar"]), rows=[3, 0, 2 * n * d // 2 - 1])
        assert np.allclose(sub, new[[3, 0, -1]], rtol=0, atol=1e-15)
        marg = hpr.marginals_comp(ref, ep, p, c)
        assert np.max(np.abs(marg - z[f"it{k}_marg"])) < 1e-12
        b2, s = hpr.new_biases_i(b, float(z["pie"]), float(z["gamma"]), z[f"it{k}_marg"], k, z[f"it{k}_u"])
        assert np.array_equal(b2, z[f"it{k}_biases"]) and np.array_equal(s, z[f"it{k}_s"])
        chi, b = ref, b2


@pytest.mark.parametrize("name", CASES)
def test_er_hpr_oracle_equals_reference_on_regular_graphs(name):
    """The ER restatement (per-message degree) on the reference's own d-regular
    fixtures: the same messages and marginals as the reference's HPr_dp /
    marginals_comp (the ER variant has no reference implementation; on a
    d-regular graph it must be HPR itself)."""
    z = load_golden(name)
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    e = z["edges"]
    nb = z["N_nodes"].astype(np.int64)
    rp = np.arange(n + 1, dtype=np.int64) * d
    classes, src, out_rows = hpr.er_classes(e, rp, nb.reshape(-1))
    assert [D for D, _, _ in classes] == [d - 1]
    assert np.array_equal(out_rows.reshape(n, d), z["N_edges_pos"])
    new = hpr.HPr_dp_er(z["chi0"], z["biases0"], classes, src, n, p, c, int(z["attr_value"]), int(z["lmbd_in"]),
                        float(z["damppar"]))
    ref = z["it0_chi"]
    assert np.max(np.abs(new - ref) / np.max(np.abs(ref), axis=1, keepdims=True)) < 1e-12
    marg = hpr.marginals_comp_csr(ref, rp, out_rows, p, c)
    assert np.max(np.abs(marg - z["it0_marg"])) < 1e-12


def test_er_hpr_oracle_on_mixed_degrees_is_normalised():
    """Leaves (D = 0) and several degree classes: rows stay normalised and the
    damping keeps the invalid x_a[T-1] blocks at (1 - damp) * old."""
    rng = np.random.default_rng(0)
    # a small graph: a path 0-1-2 plus a triangle 2-3-4 and a pendant 4-5
    e = np.array([[0, 1], [1, 2], [2, 3], [3, 4], [2, 4], [4, 5]])
    n = 6
    src = np.concatenate([e[:, 0], e[:, 1]])
    dst = np.concatenate([e[:, 1], e[:, 0]])
    order = np.lexsort((dst, src))
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(src, minlength=n), out=rp[1:])
    classes, srcs, out_rows = hpr.er_classes(e, rp, dst[order])
    assert sorted(D for D, _, _ in classes) == [0, 1, 2]
    p, c = 1, 2
    nc = 4 ** (p + c)
    chi = rng.random((2 * len(e), nc))
    chi /= chi.sum(1, keepdims=True)
    b = rng.random((n, 2))
    b /= b.sum(1, keepdims=True)
    new = hpr.HPr_dp_er(chi, b, classes, srcs, n, p, c, 1, 25 * n, 0.4)
    assert np.allclose(new.sum(1), 1.0)
    X = 2 ** (p + c)
    inval = [xa for xa in range(X) if hpr.traj_table(p + c)[xa][-1] != 1]
    blk = np.concatenate([np.arange(xa * X, xa * X + X) for xa in inval])
    assert np.allclose(new[:, blk], 0.6 * chi[:, blk])


def test_torch_cpu_restatement_equals_numpy_oracle():
    """bench.py's CPU baseline (oracle/hpr_torch.py) computes the same rows as
    the pinned numpy oracle."""
    import torch
    from oracle import hpr_torch
    z = load_golden("hpr_d4_n64_p2c2.npz")
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    inr, src = hpr.incoming_rows(z["edges"], z["N_nodes"])
    rows = np.array([0, 5, 77, 2 * z["edges"].shape[0] - 1])
    want = hpr.HPr_dp(z["chi0"], z["biases0"], inr, src, n, d, p, c, 1, 25 * n, 0.4, rows=rows)
    got = hpr_torch.HPr_dp(torch.from_numpy(z["chi0"]), torch.from_numpy(z["biases0"]), inr, src, n, d, p, c, 1,
                           25 * n, 0.4, rows)
    assert np.max(np.abs(got.numpy() - want)) < 1e-13


def test_numpy_oracle_loop_reproduces_reference_whole_script():
    """The oracle's HPR functions chained as the reference's main loop
    (code/HPR_pytorch_RRG.py:327-362: torch's CPU stream for chi0, biases0 and
    the per-iteration rand(n), float64) reproduce the reference's own
    whole-script runs exactly -- num_steps and conf for every fixture key,
    including the p+c = 4 runs and the d = 3 runs whose marginals tie exactly
    (the numpy sums break those ties as torch's do).  Pins the oracle to the
    reference's end-to-end output, not only to single steps."""
    import torch
    from oracle import majority
    z = load_golden("hpr_fullscript.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in z if k.endswith("_params")})
    assert len(keys) >= 4
    for key in keys:
        n, d, p, c, TT, tseed = (int(x) for x in z[f"{key}_params"])
        nbrs = z[f"{key}_graphs"][0].astype(np.int64)
        edges = z[f"{key}_edges"]
        inr, src = hpr.incoming_rows(edges, nbrs)
        ep = hpr.edges_pos(edges, nbrs)
        g = torch.Generator().manual_seed(tseed)
        chi = torch.rand((2 * len(edges), 4 ** (p + c)), dtype=torch.float64, generator=g)
        chi = (chi / chi.sum(1, keepdim=True)).numpy()
        b = torch.rand((n, 2), dtype=torch.float64, generator=g)
        b = (b / b.sum(1, keepdim=True)).numpy()
        s = 2 * (b[:, 0] > b[:, 1]).astype(np.int32) - 1

        def m_end(x):
            x = x.astype(np.int64)
            for _ in range(p + c - 1):
                x = majority.onestep_majority(nbrs, x)
            return x.sum() / n

        t, m = 0, m_end(s)
        while m < 1:                                                  # code/HPR_pytorch_RRG.py:344-356
            chi = hpr.HPr_dp(chi, b, inr, src, n, d, p, c, 1, 25 * n, 0.4)
            marg = hpr.marginals_comp(chi, ep, p, c)
            u = torch.rand(n, dtype=torch.float64, generator=g).numpy()
            b, s = hpr.new_biases_i(b, 0.3, 0.1, marg, t, u)
            t += 1
            m = 2 if t > TT else m_end(s)
        assert t == z[f"{key}_num_steps"][0], key
        assert np.array_equal(s, z[f"{key}_conf"][0]), key
