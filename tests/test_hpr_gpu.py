"""GPU parity of the HPR kernels (rows a9-a11 of SURVEY.md 8a).

Bar (SURVEY 8a tolerances): after one step from identical inputs,
max_row max_col |chi_gpu - chi_ref| / max_col |chi_ref| <= 1e-5 for the fp32
kernels (1e-12 for the same kernels in float64); marginals within the same
tolerance; biases and the trial configuration s identical (no near-ties in
these fixtures).  Reference vectors: tests/golden/hpr_*.npz, produced by the
reference's own HPr_dp / marginals_comp / new_biases_i.
"""
import glob
import os

import warnings

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden
from oracle import hpr as orc

pytestmark = pytest.mark.gpu

CASES = sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "hpr_d*.npz")))
TOL = {torch.float32: 1e-5, torch.float64: 1e-12}


def rownorm_err(got, ref):
    got = np.asarray(got, dtype=np.float64)
    return float(np.max(np.abs(got - ref) / np.max(np.abs(ref), axis=1, keepdims=True)))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("name", CASES)
def test_hpr_step_vs_reference(mjx_mod, name, dtype):
    z = load_golden(name)
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    plan = mjx_mod.HPRPlan(z["edges"], n, d, z["N_nodes"])
    assert np.array_equal(plan.out_row_host, z["N_edges_pos"])
    attr, lmbd, damp = int(z["attr_value"]), int(z["lmbd_in"]), float(z["damppar"])
    chi = torch.tensor(z["chi0"], dtype=dtype, device="cuda")
    b = torch.tensor(z["biases0"], dtype=dtype, device="cuda")
    for k in range(int(z["chain"])):
        # every step starts from the reference's own state (per-step tolerance)
        new = mjx_mod.HPr_dp(chi, b, plan, p, c, attr, lmbd, damp)
        assert new.dtype == dtype
        err = rownorm_err(new.cpu().numpy(), z[f"it{k}_chi"])
        assert err <= TOL[dtype], (k, err)
        ref_chi = torch.tensor(z[f"it{k}_chi"], dtype=dtype, device="cuda")
        marg = mjx_mod.marginals_comp(ref_chi, plan, p, c)
        merr = float(np.max(np.abs(marg.cpu().numpy() - z[f"it{k}_marg"])))
        assert merr <= TOL[dtype], (k, merr)
        bb = b.clone()
        ref_marg = torch.tensor(z[f"it{k}_marg"], dtype=dtype, device="cuda")
        _, s = mjx_mod.new_biases_i(bb, float(z["pie"]), float(z["gamma"]), ref_marg, k, u=z[f"it{k}_u"])
        assert np.array_equal(s.cpu().numpy(), z[f"it{k}_s"])
        np.testing.assert_allclose(bb.cpu().numpy(), z[f"it{k}_biases"], rtol=0, atol=TOL[dtype])
        chi = ref_chi
        b = torch.tensor(z[f"it{k}_biases"], dtype=dtype, device="cuda")


@pytest.mark.parametrize("name", CASES)
def test_hpr_loop_state_chain(mjx_mod, name):
    """HPRState.step chains update -> marginals -> biases -> majority check on
    the device; float64 follows the reference's chain step for step."""
    z = load_golden(name)
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    plan = mjx_mod.HPRPlan(z["edges"], n, d, z["N_nodes"])
    st = mjx_mod.HPRState(plan, p, c, z["chi0"], z["biases0"], dtype=torch.float64, damppar=float(z["damppar"]),
                          attr_value=int(z["attr_value"]), lmbd_in=int(z["lmbd_in"]), pie=float(z["pie"]),
                          gamma=float(z["gamma"]))
    for k in range(int(z["chain"])):
        tot = st.step(u=z[f"it{k}_u"])
        assert rownorm_err(st.messages().cpu().numpy(), z[f"it{k}_chi"]) < 1e-12
        assert np.array_equal(st.s.cpu().numpy(), z[f"it{k}_s"])
        assert tot / n == float(z[f"it{k}_m_end"])


def test_hpr_full_script_float64(mjx_mod):
    """Whole-script runs of code/HPR_pytorch_RRG.py (CPU, seeded): the device
    loop in float64 with the reference's torch CPU random stream reproduces
    num_steps, conf and mag_reached.

    The d = 3 runs (n30_d3_p2c1, n40_d3_p3c1) reach EXACT marginal ties
    (marg(-1) == marg(+1), decided by ``>=`` in code/HPR_pytorch_RRG.py:138):
    the outcome there depends on the last bit of float64 sums whose order the
    device kernels do not share with torch's CPU ops (the numpy oracle, which
    does, reproduces them: tests/test_hpr_oracle.py), so only their step counts
    (TT cap) are compared."""
    full = load_golden("hpr_fullscript.npz")
    exact_ties = {"n30_d3_p2c1", "n40_d3_p3c1"}   # marginals tie exactly (min margin 0)
    keys = sorted({k.rsplit("_", 1)[0] for k in full if k.endswith("_params")})
    assert keys
    for key in keys:
        n, d, p, c, TT, tseed = (int(x) for x in full[f"{key}_params"])
        nbrs = full[f"{key}_graphs"][0].astype(np.int64)
        res = mjx_mod.hpr_run(d, n, p, c, TT=TT, edges=full[f"{key}_edges"], nbrs=nbrs, seed=tseed,
                              dtype=torch.float64)
        assert res["num_steps"][0] == full[f"{key}_num_steps"][0], key
        if key in exact_ties:
            continue
        assert np.array_equal(res["conf"][0], full[f"{key}_conf"][0]), key
        assert res["mag_reached"][0] == full[f"{key}_mag_reached"][0], key
        assert np.array_equal(res["graphs"][0], full[f"{key}_graphs"][0])


def test_hpr_c3_size_against_sampled_oracle_rows(mjx_mod):
    """Config 3 size (d=4, N=1e5, p=2, c=2, fp32): rows stay normalised, and a
    random sample of rows matches the float64 oracle within 1e-5."""
    n, d, p, c = 100_000, 4, 2, 2
    edges = mjx_mod.random_regular_edges(d, n, seed=3)
    plan = mjx_mod.HPRPlan(edges, n, d)
    g = torch.Generator().manual_seed(0)
    nc = 4 ** (p + c)
    chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, generator=g)
    chi0 /= chi0.sum(1, keepdim=True)
    b0 = torch.rand((n, 2), dtype=torch.float64, generator=g)
    b0 /= b0.sum(1, keepdim=True)
    chi = chi0.to(torch.float32).cuda()
    b = b0.to(torch.float32).cuda()
    new = mjx_mod.HPr_dp(chi, b, plan, p, c, 1, 25 * n, 0.4)
    rs = new.sum(1).cpu().numpy()
    assert np.max(np.abs(rs - 1)) < 1e-5
    inr, src = orc.incoming_rows(edges, plan.nbrs_host)
    rows = np.random.default_rng(0).choice(2 * plan.E, 300, replace=False)
    # oracle from the same fp32-rounded inputs
    want = orc.HPr_dp(chi.cpu().double().numpy(), b.cpu().double().numpy(), inr, src, n, d, p, c, 1, 25 * n, 0.4,
                      rows=rows)
    assert rownorm_err(new[torch.from_numpy(rows).cuda()].cpu().numpy(), want) <= 1e-5
    marg = mjx_mod.marginals_comp(new, plan, p, c)
    m = marg.cpu().numpy()
    assert np.all(np.isfinite(m)) and np.max(np.abs(m.sum(1) - 1)) < 1e-5


@pytest.mark.parametrize("n,p,c", [(4102, 2, 2), (3000, 1, 3), (2050, 3, 1)])
def test_hpr_t4_pipelined_update_partial_tiles(mjx_mod, n, p, c):
    """T = 4 fp32 runs the software-pipelined kernel: sizes whose last tile is
    partial and that give several tiles per workgroup, every P, against the
    float64 oracle on sampled rows (1e-5 row-normalised)."""
    d = 4
    edges = mjx_mod.random_regular_edges(d, n, seed=n)
    plan = mjx_mod.HPRPlan(edges, n, d)
    g = torch.Generator().manual_seed(n)
    nc = 4 ** (p + c)
    chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, generator=g)
    chi0 /= chi0.sum(1, keepdim=True)
    b0 = torch.rand((n, 2), dtype=torch.float64, generator=g)
    b0 /= b0.sum(1, keepdim=True)
    chi = chi0.to(torch.float32).cuda()
    b = b0.to(torch.float32).cuda()
    inr, src = orc.incoming_rows(edges, plan.nbrs_host)
    rows = np.concatenate([np.arange(64), np.arange(2 * plan.E - 64, 2 * plan.E),
                           np.random.default_rng(1).choice(2 * plan.E, 200, replace=False)])
    for attr in (1, -1):
        new = mjx_mod.HPr_dp(chi, b, plan, p, c, attr, 25 * n, 0.4)
        want = orc.HPr_dp(chi.cpu().double().numpy(), b.cpu().double().numpy(), inr, src, n, d, p, c, attr, 25 * n,
                          0.4, rows=rows)
        assert rownorm_err(new[torch.from_numpy(rows).cuda()].cpu().numpy(), want) <= 1e-5, attr


def test_hpr_run_graph_batches_equal_eager_loop(mjx_mod):
    """hpr_run in hipGraph-replayed device batches (one host read per batch)
    equals the per-iteration eager loop: same stop, same conf, and the CPU
    generator left exactly where the reference's would be."""
    n, d, p, c = 200, 3, 2, 1
    edges = mjx_mod.random_regular_edges(d, n, seed=5)
    out = {}
    for mode in ("eager", "batch", "graph"):
        g = torch.Generator().manual_seed(11)
        kw = dict(batch=0) if mode == "eager" else dict(batch=8, graph=(mode == "graph"))
        res = mjx_mod.hpr_run(d, n, p, c, TT=150, edges=edges, seed=11, dtype=torch.float64, generator=g, **kw)
        out[mode] = (res, torch.rand(4, dtype=torch.float64, generator=g))
    for mode in ("batch", "graph"):
        assert out[mode][0]["num_steps"][0] == out["eager"][0]["num_steps"][0]
        assert np.array_equal(out[mode][0]["conf"], out["eager"][0]["conf"])
        assert torch.equal(out[mode][1], out["eager"][1])


@pytest.mark.parametrize("d,p,c", [(5, 2, 2), (6, 1, 3), (7, 1, 1), (8, 2, 1)])
def test_hpr_any_degree_through_the_class_kernel(mjx_mod, d, p, c):
    """Degrees and trajectory lengths beyond the register kernels (count
    tables above 128 entries, d > 6) run through the per-degree-class kernel:
    sampled rows against the float64 oracle, fp64 1e-12 and fp32 1e-5."""
    n = 60 if d * (p + c) > 16 else 120
    edges = mjx_mod.random_regular_edges(d, n, seed=d + 10 * p)
    plan = mjx_mod.HPRPlan(edges, n, d)
    rng = np.random.default_rng(d)
    nc = 4 ** (p + c)
    chi = rng.random((2 * plan.E, nc))
    chi /= chi.sum(1, keepdims=True)
    b = rng.random((n, 2))
    b /= b.sum(1, keepdims=True)
    inr, src = orc.incoming_rows(edges, plan.nbrs_host)
    rows = np.random.default_rng(2).choice(2 * plan.E, 24, replace=False)
    want = orc.HPr_dp(chi, b, inr, src, n, d, p, c, 1, 25 * n, 0.4, rows=rows)
    for dtype in (torch.float64, torch.float32):
        got = mjx_mod.HPr_dp(torch.tensor(chi, dtype=dtype, device="cuda"), torch.tensor(b, dtype=dtype, device="cuda"),
                             plan, p, c, 1, 25 * n, 0.4)
        assert rownorm_err(got[torch.from_numpy(rows).cuda()].cpu().numpy(), want) <= TOL[dtype], dtype


def _fp64_min_margin(mjx_mod, plan, p, c, TT, tseed):
    """The float64 device loop step by step on the reference's torch CPU stream
    (hpr_run's draws): (iterations, min over iterations and nodes of
    |marg+ - marg-| / (marg+ + marg-)), the margin of the decision
    code/HPR_pytorch_RRG.py:138 takes."""
    gen = torch.Generator().manual_seed(tseed)
    nc = 4 ** (p + c)
    chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, generator=gen)
    chi0 = chi0 / torch.sum(chi0, axis=1, keepdims=True)
    b0 = torch.rand((plan.n, 2), dtype=torch.float64, generator=gen)
    b0 = b0 / torch.sum(b0, axis=1, keepdims=True)
    st = mjx_mod.HPRState(plan, p, c, chi0, b0, dtype=torch.float64, layout="ref")
    st.s_from_biases()
    m, margin = st.sum_end() / plan.n, float("inf")
    while m < 1:
        total = st.step(generator=gen)
        mg = st.marg.double()
        margin = min(margin, float(((mg[:, 1] - mg[:, 0]).abs() / mg.sum(dim=1)).min()))
        m = 2 if st.t > TT else total / plan.n
    return st.t, margin


@pytest.mark.parametrize("key,first_tie", [("n30_d3_p2c1", 61), ("n40_d3_p3c1", 61)])
def test_hpr_exact_tie_runs_equal_oracle_before_the_tie(mjx_mod, key, first_tie):
    """The whole-script runs whose marginals tie EXACTLY: the
    device loop, float64 (reference layout) and float32 (hpr_run's default
    layout), equals the pinned numpy oracle's loop (which reproduces the
    reference's whole script, tests/test_hpr_oracle.py) in s after every
    iteration BEFORE the first exact tie.  The oracle's first tie is at
    iteration ``first_tie`` (recorded here: a change of fixture or oracle shows
    up); before it the smallest relative margin is >= 0.22, so no rounding
    order can flip a decision there."""
    from oracle import hpr as ohpr
    full = load_golden("hpr_fullscript.npz")
    n, d, p, c, TT, tseed = (int(x) for x in full[f"{key}_params"])
    nbrs = full[f"{key}_graphs"][0].astype(np.int64)
    edges = full[f"{key}_edges"]
    inr, src = ohpr.incoming_rows(edges, nbrs)
    ep = ohpr.edges_pos(edges, nbrs)
    nc = 4 ** (p + c)
    # the oracle's loop (code/HPR_pytorch_RRG.py:327-356) on torch's CPU stream
    g = torch.Generator().manual_seed(tseed)
    chi = torch.rand((2 * len(edges), nc), dtype=torch.float64, generator=g)
    chi = (chi / chi.sum(1, keepdim=True)).numpy()
    b = torch.rand((n, 2), dtype=torch.float64, generator=g)
    b = (b / b.sum(1, keepdim=True)).numpy()
    want, t0 = [], None
    for t in range(first_tie + 1):
        chi = ohpr.HPr_dp(chi, b, inr, src, n, d, p, c, 1, 25 * n, 0.4)
        marg = ohpr.marginals_comp(chi, ep, p, c)
        if t0 is None and np.min(np.abs(marg[:, 1] - marg[:, 0])) == 0:
            t0 = t
        u = torch.rand(n, dtype=torch.float64, generator=g).numpy()
        b, s = ohpr.new_biases_i(b, 0.3, 0.1, marg, t, u)
        want.append(s.copy())
    assert t0 == first_tie, t0
    plan = mjx_mod.HPRPlan(edges, n, d, nbrs)
    for dtype, layout in ((torch.float64, "ref"), (torch.float32, None)):
        gen = torch.Generator().manual_seed(tseed)
        chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, generator=gen)
        chi0 = chi0 / torch.sum(chi0, axis=1, keepdims=True)
        b0 = torch.rand((n, 2), dtype=torch.float64, generator=gen)
        b0 = b0 / torch.sum(b0, axis=1, keepdims=True)
        st = mjx_mod.HPRState(plan, p, c, chi0.to(dtype), b0.to(dtype), dtype=dtype, layout=layout)
        st.s_from_biases()
        for t in range(first_tie):
            st.step(generator=gen)
            assert np.array_equal(st.s.cpu().numpy(), want[t]), (str(dtype), t)


def test_hpr_full_script_float32_loop(mjx_mod):
    """fp32 whole loop (hpr_run's default: the decay-split layout where p+c = 4,
    the reference layout otherwise) against the reference's own whole-script
    runs (code/HPR_pytorch_RRG.py:342-362, run in float64 by the reference,
    :11).  Where the float64 loop's marginals never come within 1e-5 of a tie
    (relative, the decision of :138), the fp32 run must reproduce num_steps and
    conf exactly; runs with a near-tie are listed, and counted (VERDICT r03
    item 4)."""
    full = load_golden("hpr_fullscript.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in full if k.endswith("_params")})
    report, strict = [], 0
    for key in keys:
        n, d, p, c, TT, tseed = (int(x) for x in full[f"{key}_params"])
        nbrs = full[f"{key}_graphs"][0].astype(np.int64)
        plan = mjx_mod.HPRPlan(full[f"{key}_edges"], n, d, nbrs)
        steps64, margin = _fp64_min_margin(mjx_mod, plan, p, c, TT, tseed)
        res = mjx_mod.hpr_run(d, n, p, c, TT=TT, edges=full[f"{key}_edges"], nbrs=nbrs, seed=tseed,
                              dtype=torch.float32)
        same = (res["num_steps"][0] == full[f"{key}_num_steps"][0] and
                np.array_equal(res["conf"][0], full[f"{key}_conf"][0]))
        layout = "q" if mjx_mod._lib.load().mjx_hpr_q_supported(mjx_mod._lib.MJX_F32, d, p, c) == 1 else "ref"
        near = margin < 1e-5
        report.append(f"{key}: layout {layout}, fp64 steps {steps64}, min margin {margin:.3g}"
                      f"{' NEAR-TIE' if near else ''}, fp32 {'equal' if same else 'differs'}")
        if not near:
            strict += 1
            assert same, report[-1]
    summary = ("fp32 whole-loop vs reference script:\n  " + "\n  ".join(report) +
               f"\n  {strict} of {len(keys)} runs without a near-tie, all reproduced; "
               f"{len(keys) - strict} near-tie runs listed")
    print("\n" + summary)
    warnings.warn(summary)               # shown in the pytest summary of the GPU run's log
    assert strict >= 1
