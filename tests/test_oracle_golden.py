"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import majority as orc
from oracle.mt19937 import MT19937

PC = [(1, 1), (2, 1), (2, 2), (3, 1)]


@pytest.mark.parametrize("d", [3, 4, 6])
@pytest.mark.parametrize("n", [64, 1000])
def test_rrg_rollout_matches_reference(d, n):
    z = load_golden("rrg_dyn.npz")
    key = f"d{d}_n{n}"
    N, S0 = z[f"{key}_N"], z[f"{key}_s0"]
    for (p, c) in PC:
        want = z[f"{key}_p{p}c{c}"]
        got = np.stack([orc.s_endstate(N, s0, p, c) for s0 in S0])
        assert got.dtype == np.int64
        assert np.array_equal(got, want), (p, c)
        assert np.array_equal(orc.s_endstate_batch(N, S0, p, c), want)
    np.testing.assert_array_equal(orc.m(S0), z[f"{key}_m"])


def test_er_rollout_matches_reference():
    z = load_golden("er_dyn.npz")
    keys = sorted(k[:-len("_row_ptr")] for k in z if k.endswith("_row_ptr"))
    assert len(keys) == 3
    for key in keys:
        rp, col, S0 = z[f"{key}_row_ptr"], z[f"{key}_col"], z[f"{key}_s0"]
        for (p, c) in PC:
            want = z[f"{key}_p{p}c{c}"]
            got = orc.s_endstate_er(rp, col, S0, p, c)
            assert np.array_equal(got, want), (key, p, c)


@pytest.mark.parametrize("seed", [0, 1, 12345, 2 ** 32 - 1])
def test_mt19937_restatement_matches_numpy(seed):
    rs = np.random.RandomState(seed)
    mt = MT19937(seed)
    n = 10000
    b = rs.binomial(n=1, p=0.5, size=[n])
    assert np.array_equal(b, [mt.binomial_half() for _ in range(n)])
    for _ in range(500):
        assert rs.randint(low=0, high=n) == mt.randint(n)
        assert rs.rand() == mt.random_double()
    for high in (1, 2, 3, 200, 65537, 2 ** 31):
        assert rs.randint(low=0, high=high) == mt.randint(high)


def test_global_stream_equals_randomstate():
    np.random.seed(77)
    a = (np.random.binomial(1, .5, 50), np.random.randint(low=0, high=300), np.random.rand())
    rs = np.random.RandomState(77)
    b = (rs.binomial(1, .5, 50), rs.randint(low=0, high=300), rs.rand())
    assert np.array_equal(a[0], b[0]) and a[1] == b[1] and a[2] == b[2]


SA_FIXTURES = ["sa_d4_n200_p3c1.npz", "sa_d3_n300_p2c1.npz", "sa_d4_n200_p1c1.npz", "sa_d4_n1000_p2c2.npz"]


@pytest.mark.parametrize("name", SA_FIXTURES)
def test_sa_oracle_matches_reference_trace(name):
    z = load_golden(name)
    N, p, c = z["N"], int(z["p"]), int(z["c"])
    seeds = [int(s) for s in z["seeds"]]
    for sd in seeds[:2]:
        steps = int(z[f"seed{sd}_num_steps"])
        cap = min(steps, 3000)
        r = orc.sa_loop(N, p, c, sd, max_steps=cap, trace=True)
        tr = r["trace"]
        assert np.array_equal(tr["i"], z[f"seed{sd}_i"][:cap])
        assert np.array_equal(tr["accept"], z[f"seed{sd}_accept"][:cap])
        assert np.array_equal(tr["sum_end"], z[f"seed{sd}_sum_end"][:cap])
        assert np.array_equal(tr["dE"], z[f"seed{sd}_dE"][:cap])   # bit-exact float64
        if cap == steps and int(z[f"seed{sd}_converged"]):
            assert np.array_equal(r["conf"], z[f"seed{sd}_conf"])
            assert r["mag_reached"] == z[f"seed{sd}_mag_reached"]


def test_sa_harness_matches_full_reference_script():
    """The per-step fixtures come from a harness around the reference's
    functions; the whole-script runs pin that harness."""
    full = load_golden("sa_fullscript.npz")
    for key, fx, seed in (("n200_d4_p3", "sa_d4_n200_p3c1.npz", 0), ("n300_d3_p2", "sa_d3_n300_p2c1.npz", 5)):
        z = load_golden(fx)
        assert np.array_equal(full[f"{key}_graphs"][0], z["N"])
        assert float(full[f"{key}_num_steps"][0]) == float(z[f"seed{seed}_num_steps"])
        assert np.array_equal(full[f"{key}_conf"][0], z[f"seed{seed}_conf"])
        assert float(full[f"{key}_mag_reached"][0]) == float(z[f"seed{seed}_mag_reached"])
