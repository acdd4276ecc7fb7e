"""Pin the C restatement (oracle/orc_majority.c) against the reference's own
golden vectors and the numpy oracle.  CPU only."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import fast
from oracle import majority as orc

PC = [(1, 1), (2, 1), (2, 2), (3, 1)]


@pytest.mark.parametrize("d", [3, 4, 6])
@pytest.mark.parametrize("n", [64, 1000])
def test_c_rrg_rollout_matches_reference(d, n):
    z = load_golden("rrg_dyn.npz")
    key = f"d{d}_n{n}"
    N, S0 = z[f"{key}_N"], z[f"{key}_s0"]
    for (p, c) in PC:
        want = z[f"{key}_p{p}c{c}"]
        got = np.stack([fast.s_endstate(N, s0, p, c) for s0 in S0])
        assert np.array_equal(got, want), (p, c)


def test_c_er_rollout_matches_reference():
    z = load_golden("er_dyn.npz")
    keys = sorted(k[:-len("_row_ptr")] for k in z if k.endswith("_row_ptr"))
    for key in keys:
        rp, col, S0 = z[f"{key}_row_ptr"], z[f"{key}_col"], z[f"{key}_s0"]
        for (p, c) in PC:
            want = z[f"{key}_p{p}c{c}"]
            got = np.stack([fast.s_endstate_er(rp, col, s0, p, c) for s0 in S0])
            assert np.array_equal(got, want), (key, p, c)


@pytest.mark.parametrize("name", ["sa_d4_n200_p3c1.npz", "sa_d3_n300_p2c1.npz", "sa_d4_n200_p1c1.npz",
                                  "sa_d4_n1000_p2c2.npz"])
def test_c_sa_matches_reference_trace(name):
    z = load_golden(name)
    N, p, c = z["N"], int(z["p"]), int(z["c"])
    for sd in [int(s) for s in z["seeds"]]:
        steps = int(z[f"seed{sd}_num_steps"])
        L = len(z[f"seed{sd}_i"])
        r = fast.sa_loop(N, p, c, sd, max_steps=L, trace=True)
        tr = r["trace"]
        assert np.array_equal(tr["i"], z[f"seed{sd}_i"])
        assert np.array_equal(tr["accept"], z[f"seed{sd}_accept"])
        assert np.array_equal(tr["sum_end"], z[f"seed{sd}_sum_end"])
        assert np.array_equal(tr["dE"], z[f"seed{sd}_dE"])        # bit-exact float64
        if L == steps and int(z[f"seed{sd}_converged"]):
            assert r["done"] == 1 and r["num_steps"] == steps
            assert np.array_equal(r["conf"], z[f"seed{sd}_conf"])
            assert r["mag_reached"] == z[f"seed{sd}_mag_reached"]


def test_c_sa_full_script():
    full = load_golden("sa_fullscript.npz")
    for key, p, c in (("n200_d4_p3", 3, 1), ("n300_d3_p2", 2, 1)):
        N = full[f"{key}_graphs"][0]
        seed = 0 if key.startswith("n200") else 5
        r = fast.sa_loop(N, p, c, seed)
        assert r["done"] == 1
        assert float(r["num_steps"]) == float(full[f"{key}_num_steps"][0])
        assert np.array_equal(r["conf"], full[f"{key}_conf"][0])
        assert r["mag_reached"] == full[f"{key}_mag_reached"][0]


def test_c_sa_matches_numpy_oracle_on_c1_sizes():
    """C1's graph size (d=4, N=1e4, p=c=1): 300 steps of two seeds, C vs numpy."""
    from mjx import random_regular_graph
    adj = random_regular_graph(4, 10_000, seed=1000)
    for seed in (0, 63):
        a = fast.sa_loop(adj, 1, 1, seed, max_steps=300, trace=True)
        b = orc.sa_loop(adj, 1, 1, seed, max_steps=300, trace=True)
        for k in ("i", "accept", "sum_end", "dE"):
            assert np.array_equal(a["trace"][k], b["trace"][k]), k
        assert np.array_equal(a["conf"], b["conf"])


def test_c_sa_global_stream_two_replicas():
    """The reference script with N_stat = 2 (one numpy stream, seeded once,
    consumed by replica 0 then replica 1, each on its own graph)."""
    from oracle.mt19937 import MT19937
    full = load_golden("sa_fullscript.npz")
    key = "n200_d4_p3_nstat2"
    graphs = full[f"{key}_graphs"]
    m = MT19937(11)                                     # np.random.seed(11) before the replica loop
    state = (np.array(m.mt, dtype=np.uint32), m.idx)
    for k in range(2):
        r = fast.sa_loop(graphs[k], 3, 1, 0, mt_state=state)
        state = r["mt_state"]
        assert r["done"] == 1
        assert float(r["num_steps"]) == float(full[f"{key}_num_steps"][k])
        assert np.array_equal(r["conf"], full[f"{key}_conf"][k])
        assert r["mag_reached"] == full[f"{key}_mag_reached"][k]


# Random123's known-answer vectors for philox4x32_10 (counter, key, result):
# the library's non-parity proposal stream is pinned by them
PHILOX_KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox4x32_10_known_answers(ctr, key, want):
    assert [int(x) for x in fast.philox4x32_10(ctr, key)] == list(want)


def philox_proposal(seed, t, n):
    """Proposal t of a replica keyed by its seed (include/mjx.h philox_key):
    restated in Python integers from the KAT-pinned block."""
    x = [int(v) for v in fast.philox4x32_10([t & 0xFFFFFFFF, t >> 32, 0, 0], [seed & 0xFFFFFFFF, seed >> 32])]
    i = ((x[0] | (x[1] << 32)) * n) >> 64
    u = ((x[2] >> 5) * 67108864.0 + (x[3] >> 6)) / 9007199254740992.0
    return i, u


def test_c_sa_philox_loop_is_the_sa_loop_on_philox_proposals():
    """orc_sa_loop_philox: the reference's loop (the same code as orc_sa_loop)
    with proposal t = Philox(seed, t): its trace's i are the Python-restated
    proposals, each accept is u < min(1, exp(-dE)), the initial configuration
    is the seeded MT one and the final one is it with the accepted flips."""
    from mjx import random_regular_graph
    n, d, p, c, K = 300, 3, 2, 1, 400
    adj = random_regular_graph(d, n, seed=12)
    for seed in (0, 5, 4095):
        r = fast.sa_loop_philox(adj, p, c, seed, max_steps=K, trace=True)
        tr = r["trace"]
        s = fast.sa_loop(adj, p, c, seed, max_steps=0)["conf"].copy()
        for t in range(r["num_steps"]):
            i, u = philox_proposal(seed, t, n)
            assert tr["i"][t] == i
            assert bool(tr["accept"][t]) == (u < min(1.0, float(np.exp(-tr["dE"][t]))))
            if tr["accept"][t]:
                s[i] = -s[i]
        assert np.array_equal(s, r["conf"])
        assert tr["sum_end"][-1] == int(np.sum(orc.s_endstate(adj, r["conf"], p, c)))
    # another key, the same initial configuration, another run
    a = fast.sa_loop_philox(adj, p, c, 5, max_steps=50, trace=True, key=6)
    b = fast.sa_loop_philox(adj, p, c, 5, max_steps=50, trace=True)
    assert not np.array_equal(a["trace"]["i"], b["trace"]["i"])
