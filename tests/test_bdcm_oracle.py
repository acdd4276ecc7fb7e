"""Pin the BDCM oracle (oracle/bdcm.py) against vectors produced by the
notebook's own functions (tests/golden/make_golden.py gen_bdcm).  CPU only."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import bdcm

CASES = sorted(os.path.basename(f) for f in glob.glob(os.path.join(GOLDEN, "bdcm_er_*.npz")))


def plan_of(z):
    return bdcm.Plan.from_csr(z["edges"], z["row_ptr"], z["col"], int(z["n"]), int(z["n_iso"]))


def rowrel(got, ref):
    return float(np.max(np.abs(got - ref) / np.max(np.abs(ref), axis=1, keepdims=True)))


def test_fixtures_present():
    assert len(CASES) >= 4


@pytest.mark.parametrize("name", CASES)
def test_oracle_sweep_and_observables(name):
    z = load_golden(name)
    p, c, lm = int(z["p"]), int(z["c"]), float(z["sweep_lmbd"])
    plan = plan_of(z)
    ch = z["chi0"].copy()
    if 0 in plan.class_rows:
        ch[plan.class_rows[0]] = bdcm.leaf_message(p, c, 1, lm)[None, :]
    assert rowrel(ch, z["sweep_leaf"]) < 1e-14
    new = bdcm.BDCM_ER(z["sweep_leaf"], plan, p, c, 1, lm, float(z["damppar"]))
    assert rowrel(new, z["sweep_chi"]) < 1e-12
    ref = z["sweep_chi"]
    np.testing.assert_allclose(bdcm.Zi_ER(ref, plan, p, c, 1, lm), z["sweep_zi"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(bdcm.Zij(ref, plan, p, c, 1), z["sweep_zij"], rtol=1e-12, atol=0)
    assert abs(bdcm.phi_BP(ref, plan, p, c, 1, lm) - float(z["sweep_phi"])) < 1e-12
    assert abs(bdcm.avg_m_init(ref, plan, p, c, 1) - float(z["sweep_m_init"])) < 1e-12


@pytest.mark.parametrize("name", ["bdcm_er_n300_deg2_p1c1.npz", "bdcm_er_n120_deg3_p1c2.npz"])
def test_oracle_entropy_procedure(name):
    z = load_golden(name)
    p, c = int(z["p"]), int(z["c"])
    m_init, ent1, ent, counts, iters, chi = bdcm.entropy_procedure(
        z["chi0"], plan_of(z), p, c, 1, z["lambdas"], float(z["damppar"]), eps=float(z["eps"]),
        T_max=int(z["T_max"]))
    L = len(z["iters"])
    assert np.array_equal(iters[:L], z["iters"])
    np.testing.assert_allclose(m_init, z["m_init"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(ent1, z["ent1"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(ent, z["ent"], rtol=1e-10, atol=1e-12)
    assert rowrel(chi, z["chi_final"]) < 1e-10
