"""GPU parity of the ER ("general") HPR (code/README.md:1):
the per-degree-class update, the CSR marginals and the loop against the
float64 oracle restatement (oracle/hpr.py HPr_dp_er, pinned to the
reference's own HPR fixtures on d-regular graphs).  Bars: 1e-12 row-normalised
in float64, 1e-5 in float32; on a d-regular graph the ER kernels equal the
RRG kernels."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import hpr as orc

pytestmark = pytest.mark.gpu
TOL = {torch.float32: 1e-5, torch.float64: 1e-12}


def rownorm_err(got, ref):
    got = np.asarray(got, dtype=np.float64)
    return float(np.max(np.abs(got - ref) / np.max(np.abs(ref), axis=1, keepdims=True)))


def _random_state(E, n, p, c, seed):
    rng = np.random.default_rng(seed)
    chi = rng.random((2 * E, 4 ** (p + c)))
    chi /= chi.sum(1, keepdims=True)
    b = rng.random((n, 2))
    b /= b.sum(1, keepdims=True)
    return chi, b


_ORACLE = {}


def _oracle_step(plan, chi, b, p, c, attr):
    key = (plan.n, plan.E, p, c, attr, float(chi[0, 0]))
    if key not in _ORACLE:
        classes, src, _ = orc.er_classes(plan.edges, plan.row_ptr_host, plan.col_host)
        _ORACLE[key] = orc.HPr_dp_er(chi, b, classes, src, plan.n, p, c, attr, 25 * plan.n, 0.4)
    return _ORACLE[key]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("n,mean,p,c", [(300, 3.0, 1, 1), (200, 2.5, 2, 1), (150, 2.0, 1, 2), (80, 3.0, 2, 2),
                                         (120, 4.0, 1, 1), (100, 5.0, 2, 2), (100, 6.0, 1, 2)])
def test_er_hpr_step_vs_oracle(mjx_mod, dtype, n, mean, p, c):
    """(100, 5.0, 2, 2): degree-10 hubs, whose T = 4 count tables exceed the
    LDS budget and run from the global scratch slab."""
    plan, _ = mjx_mod.hpr_er_plan(n, mean / (n - 1), seed=n)
    classes, src, out_rows = orc.er_classes(plan.edges, plan.row_ptr_host, plan.col_host)
    assert np.array_equal(out_rows, plan.out_rows_host)
    chi, b = _random_state(plan.E, plan.n, p, c, n)
    for attr in (1, -1):
        got = mjx_mod.HPr_dp_er(torch.tensor(chi, dtype=dtype, device="cuda"),
                                torch.tensor(b, dtype=dtype, device="cuda"), plan, p, c, attr, 25 * plan.n, 0.4)
        want = _oracle_step(plan, chi, b, p, c, attr)
        assert rownorm_err(got.cpu().numpy(), want) <= TOL[dtype], attr
    marg = mjx_mod.marginals_comp_er(torch.tensor(want, dtype=dtype, device="cuda"), plan, p, c)
    wm = orc.marginals_comp_csr(want, plan.row_ptr_host, out_rows, p, c)
    assert float(np.max(np.abs(marg.cpu().numpy() - wm))) <= TOL[dtype]


@pytest.mark.parametrize("name", ["hpr_d4_n64_p1c1.npz", "hpr_d3_n50_p2c1.npz", "hpr_d4_n40_p1c2.npz"])
def test_er_hpr_equals_reference_on_regular_fixtures(mjx_mod, name):
    """On the reference's own d-regular fixtures the ER kernels reproduce the
    reference's HPr_dp and marginals_comp (float64, 1e-12)."""
    z = load_golden(name)
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    rp = np.arange(n + 1, dtype=np.int64) * d
    plan = mjx_mod.HPRERPlan(z["edges"], rp, z["N_nodes"].reshape(-1))
    got = mjx_mod.HPr_dp_er(torch.tensor(z["chi0"], device="cuda"), torch.tensor(z["biases0"], device="cuda"), plan,
                            p, c, int(z["attr_value"]), int(z["lmbd_in"]), float(z["damppar"]))
    assert rownorm_err(got.cpu().numpy(), z["it0_chi"]) < 1e-12
    marg = mjx_mod.marginals_comp_er(torch.tensor(z["it0_chi"], device="cuda"), plan, p, c)
    assert float(np.max(np.abs(marg.cpu().numpy() - z["it0_marg"]))) < 1e-12


def test_er_hpr_run_reaches_consensus_or_cap(mjx_mod):
    """The loop on a small ER core graph: a trial configuration whose ER
    majority rollout (oracle, nb:113-123) is all +1 when the run reports m = 1."""
    from oracle import majority as om
    plan, iso = mjx_mod.hpr_er_plan(200, 3.0 / 199, seed=4)
    res = mjx_mod.hpr_er_run(plan=plan, p=1, c=1, TT=300, seed=2, dtype=torch.float64)
    s = res["conf"][0].astype(np.int64)
    end = om.s_endstate_er(res["row_ptr"], res["col"], s, 1, 1)
    if res["num_steps"][0] <= 300:
        assert np.all(end == 1)
    assert res["mag_reached"][0] == np.sum(s) / plan.n
