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
