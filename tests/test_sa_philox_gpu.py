"""The NON-parity SA mode (SAReplicas(rng="philox")): the
proposal of step t of replica r is Philox-4x32-10 keyed by r's seed, drawn
into the light-cone tape (include/mjx.h, mjx_sa_state.philox_key).  Checked
bit for bit against the C oracle's loop on the same stream
(oracle/orc_majority.c orc_sa_loop_philox; its Philox block is pinned by
Random123's known-answer vectors in tests/test_oracle_c.py): i, accept,
sum(s_end) and delta_H of every step, the final configuration; the same run
whatever the tape chunking, layout or call sizes; the MT-only paths refuse it."""
import numpy as np
import pytest

from oracle import fast

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout,tape,d,p,c", [("rec", 1024, 3, 2, 1), ("cone", 1024, 3, 2, 1),
                                               ("levels", 1024, 3, 2, 1), ("cone", 7, 3, 2, 1),
                                               ("rec", 1024, 4, 1, 1), ("cone", 64, 4, 3, 1)])
def test_sa_philox_trace_bit_exact(mjx_mod, layout, tape, d, p, c):
    n, R, K = 600, 130, 500                              # ragged R: three words, padding bits
    adj = mjx_mod.random_regular_graph(d, n, seed=21)
    seeds = list(range(100, 100 + R))
    sa = mjx_mod.SAReplicas(adj, p, c, seeds, mode="lightcone", layout=layout, tape=tape, rng="philox")
    parts = [sa.steps(k, trace=True) for k in (170, 1, 329)]           # ragged calls
    tr = {k: np.concatenate([pt[k].cpu().numpy() for pt in parts]) for k in parts[0]}
    res = sa.results()
    for r in (0, 1, 63, 64, 129):
        o = fast.sa_loop_philox(adj, p, c, seeds[r], max_steps=K, trace=True)
        L = o["num_steps"]
        for key in ("i", "accept", "sum_end", "dE"):
            assert np.array_equal(tr[key][:L, r], o["trace"][key]), (r, key)
        assert np.array_equal(res["conf"][r], o["conf"])
        assert res["num_steps"][r] == L


def test_sa_philox_runs_to_consensus_like_the_oracle(mjx_mod):
    """Small graphs run to consensus: num_steps, mag_reached, conf as the oracle's."""
    n, d, p, c = 120, 3, 2, 1
    adj = mjx_mod.random_regular_graph(d, n, seed=8)
    seeds = [1, 2, 3, 4]
    sa = mjx_mod.SAReplicas(adj, p, c, seeds, mode="lightcone", layout="cone", rng="philox")
    for _ in range(200):
        if sa.all_done():
            break
        sa.steps(4096)
    res = sa.results()
    for r, sd in enumerate(seeds):
        o = fast.sa_loop_philox(adj, p, c, sd)
        assert o["done"] == 1 and res["done"][r] == 1
        assert res["num_steps"][r] == o["num_steps"]
        assert np.array_equal(res["conf"][r], o["conf"])


def test_sa_philox_checkpoint_resume(mjx_mod):
    """The Philox stream's state is (key, t): a checkpoint taken with the tape
    in use resumes to the uninterrupted run."""
    n, d, p, c, R = 400, 3, 2, 1, 70
    adj = mjx_mod.random_regular_graph(d, n, seed=4)
    seeds = list(range(R))
    a = mjx_mod.SAReplicas(adj, p, c, seeds, mode="lightcone", layout="rec", rng="philox")
    a.steps(300)
    ck = a.checkpoint()
    assert str(ck["rng"]) == "philox"
    a.steps(250)
    b = mjx_mod.SAReplicas.resume(adj, ck, layout="cone")
    b.steps(250)
    ra, rb = a.results(), b.results()
    assert np.array_equal(ra["conf"], rb["conf"]) and np.array_equal(ra["num_steps"], rb["num_steps"])


def test_sa_philox_refused_where_mt_is_drawn_in_the_step(mjx_mod):
    adj = mjx_mod.random_regular_graph(3, 200, seed=1)
    with pytest.raises(ValueError):
        mjx_mod.SAReplicas(adj, 2, 1, [0, 1], mode="lightcone", layout="lds", rng="philox")
    with pytest.raises(ValueError):
        mjx_mod.SAReplicas(adj, 2, 1, [0, 1], mode="rollout", rng="philox")
    with pytest.raises(ValueError):
        mjx_mod.SAReplicas(adj, 2, 1, [0, 1], mode="lightcone", layout="cone", tape=0, rng="philox")
    # the C ABI refuses the key on the in-step paths too
    sa = mjx_mod.SAReplicas(adj, 2, 1, [0, 1], mode="lightcone", layout="cone", rng="philox")
    sa.layout, sa.cone = "lds", None
    with pytest.raises(mjx_mod.MjxError):
        sa.steps(3)


def test_sa_steps_under_graph_capture_equal_eager(mjx_mod):
    """A stream under hipGraph capture keeps the one-stream MT tape (no side
    stream inside a capture): steps captured once and replayed twice equal the
    same steps run eagerly."""
    import torch
    n, d, p, c, R = 500, 3, 2, 1, 70
    adj = mjx_mod.random_regular_graph(d, n, seed=9)
    seeds = list(range(R))
    a = mjx_mod.SAReplicas(adj, p, c, seeds, mode="lightcone", layout="rec")
    b = mjx_mod.SAReplicas(adj, p, c, seeds, mode="lightcone", layout="rec")
    a.steps(300)                                      # warm-up outside the capture (LDS opt-ins)
    b.steps(300)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        b.steps(300)
    g.replay()
    g.replay()
    a.steps(300)
    a.steps(300)
    torch.cuda.synchronize()
    ra, rb = a.results(), b.results()
    assert np.array_equal(ra["conf"], rb["conf"]) and np.array_equal(ra["num_steps"], rb["num_steps"])
