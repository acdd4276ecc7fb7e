"""SA replicas on distinct graphs, run together (code/SA_RRG.py:58-62 draws a
fresh random regular graph for every replica), and the light-cone kernels'
own-bit re-reads under stress.  Every replica is checked bit for bit against
the C restatement of the reference's SA loop (oracle/orc_majority.c,
code/SA_RRG.py:63-88) on ITS graph: proposals, accepts, sum(s_end), delta_H,
final conf and step count."""
import numpy as np
import pytest
import torch

from oracle import fast

pytestmark = pytest.mark.gpu


def _graphs(mjx_mod, d, n, G, base):
    return [mjx_mod.random_regular_graph(d, n, seed=base + g) for g in range(G)]


def _check(tr, conf, t, graphs, graph_of, seeds, p, c, K, replicas):
    for r in replicas:
        o = fast.sa_loop(graphs[graph_of[r]], p, c, seeds[r], max_steps=K, trace=True)
        L = len(o["trace"]["i"])
        assert L == t[r], r
        for key in ("i", "accept", "sum_end", "dE"):
            assert np.array_equal(tr[key][:L, r], o["trace"][key]), (r, key)
        assert np.array_equal(conf[r], o["conf"]), r


@pytest.mark.parametrize("d,n,p,c,R,K,kernel,mode,layout", [
    (3, 500, 2, 1, 70, 400, {}, "lightcone", "cone"),                       # speculative batches
    (3, 500, 2, 1, 70, 400, {"spec_k": 16}, "lightcone", "cone"),
    (3, 500, 2, 1, 70, 300, {"no_spec": True}, "lightcone", "cone"),        # one round trip
    (3, 500, 2, 1, 70, 300, {"no_spec": True, "no_cone2": True}, "lightcone", "cone"),
    (4, 400, 1, 1, 130, 400, {}, "lightcone", "cone"),
    (4, 300, 3, 1, 65, 300, {}, "lightcone", "cone"),                       # SA_RRG.py's p=3, c=1
    (6, 200, 2, 1, 20, 200, {}, "lightcone", "cone"),
    (3, 500, 2, 1, 70, 400, {}, "lightcone", "lds"),                        # LDS-resident replicas
    (4, 400, 1, 1, 130, 400, {}, "lightcone", "lds"),
    (4, 400, 1, 1, 130, 400, {"lds_pair": True}, "lightcone", "lds"),
    (3, 64, 1, 1, 70, 600, {}, "lightcone", "lds"),                          # eight proposals, many conflicts
    (4, 64, 1, 1, 70, 600, {}, "lightcone", "lds"),
    (4, 300, 3, 1, 65, 300, {}, "lightcone", "lds"),
    (6, 200, 2, 1, 20, 200, {}, "lightcone", "lds"),
    (5, 200, 2, 2, 20, 200, {}, "lightcone", "lds"),                        # runtime degree, T = 3
    (4, 300, 3, 1, 65, 300, {"lds_serial": True}, "lightcone", "lds"),     # the list-based LDS step
    (4, 300, 3, 1, 65, 300, {"lds_single": True}, "lightcone", "lds"),     # one proposal per LDS step
    (4, 64, 2, 2, 40, 400, {"lds_single": True}, "lightcone", "lds"),
    (4, 150, 3, 2, 20, 300, {}, "lightcone", "lds"),                        # T = 4, pair and single
    (4, 150, 3, 2, 20, 300, {"lds_single": True}, "lightcone", "lds"),
    (3, 200, 2, 3, 20, 300, {}, "lightcone", "lds"),
    (3, 64, 2, 1, 40, 400, {}, "lightcone", "lds"),                         # small graph: many non-tree balls
    (4, 64, 2, 2, 40, 400, {}, "lightcone", "lds"),                         # T = 3, levels beyond one wave
    (4, 400, 1, 1, 130, 400, {"lds_wave": True}, "lightcone", "lds"),      # one wave, eight proposals
    (4, 64, 1, 1, 70, 600, {"lds_wave": True}, "lightcone", "lds"),
    (3, 30, 1, 1, 40, 800, {}, "lightcone", "lds"),                          # n=30: 32 in flight, most cut
    (4, 300, 3, 1, 65, 300, {"lds_wave": True}, "lightcone", "lds"),       # one wave per replica (pair)
    (4, 300, 3, 1, 65, 300, {"split": 4}, "lightcone", "lds"),              # whole CU, 4 waves
    (4, 300, 3, 1, 65, 300, {"split": 8}, "lightcone", "lds"),              # whole CU, 8 waves
    (4, 300, 3, 1, 65, 300, {"split": 16}, "lightcone", "lds"),             # whole CU, a proposal per wave, 16 waves
    (3, 64, 2, 1, 40, 400, {"split": 16}, "lightcone", "lds"),
    (4, 64, 2, 2, 40, 400, {"split": 16}, "lightcone", "lds"),
    (4, 40, 3, 1, 40, 600, {"split": 8}, "lightcone", "lds"),
    (3, 64, 2, 1, 40, 400, {"split": 8}, "lightcone", "lds"),
    (4, 64, 2, 2, 40, 400, {"lds_wave": True}, "lightcone", "lds"),
    (3, 64, 2, 1, 40, 400, {"split": 4}, "lightcone", "lds"),               # many conflicts, 4 waves
    (4, 300, 3, 1, 65, 300, {"lds_cu": True}, "lightcone", "lds"),          # level-synchronous whole CU (the default)
    (4, 40, 3, 1, 40, 600, {"lds_cu": True}, "lightcone", "lds"),
    (3, 64, 2, 1, 40, 400, {"lds_cu": True}, "lightcone", "lds"),
    (4, 64, 2, 2, 40, 400, {"lds_cu": True}, "lightcone", "lds"),           # T = 3
    (3, 30, 2, 2, 40, 600, {"lds_cu": True}, "lightcone", "lds"),           # T = 3, balls cover the graph
    (4, 300, 3, 1, 65, 300, {"lds_cu": True, "split": 16}, "lightcone", "lds"),   # 16 waves
    (3, 64, 2, 1, 40, 400, {"lds_cu": True, "split": 16}, "lightcone", "lds"),
    (4, 40, 3, 1, 40, 600, {}, "lightcone", "lds"),                         # n=40: most rounds conflict
    (3, 30, 2, 2, 40, 600, {}, "lightcone", "lds"),
    (4, 200, 1, 1, 5, 40, {}, "rollout", None),
])
def test_distinct_graphs_match_oracle(mjx_mod, d, n, p, c, R, K, kernel, mode, layout):
    graphs = _graphs(mjx_mod, d, n, R, 100)
    seeds = list(range(1000, 1000 + R))
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, mode=mode, kernel=kernel, layout=layout or "auto")
    assert sa.rep_graph is not None and sa.mode == mode and sa.layout == layout
    tr = {k: v.cpu().numpy() for k, v in sa.steps(K, trace=True).items()}
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    _check(tr, conf, t, graphs, list(range(R)), seeds, p, c, K, sorted({0, 1, R // 2, R - 1, min(64, R - 1)}))


def test_shared_graph_stack_with_graph_of(mjx_mod):
    """Several replicas per graph (graph_of): each replica equals the oracle
    on its graph, and replicas of one graph equal a single-graph run."""
    d, n, p, c, K = 3, 400, 2, 1, 300
    graphs = _graphs(mjx_mod, d, n, 3, 7)
    R = 96
    graph_of = [r % 3 for r in range(R)]
    seeds = list(range(R))
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, graph_of=graph_of, layout="cone")
    tr = {k: v.cpu().numpy() for k, v in sa.steps(K, trace=True).items()}
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    _check(tr, conf, t, graphs, graph_of, seeds, p, c, K, (0, 1, 2, 50, 95))
    one = mjx_mod.SAReplicas(graphs[1], p, c, [seeds[r] for r in range(1, R, 3)], layout="lds")
    tr1 = one.steps(K, trace=True)
    assert np.array_equal(tr1["accept"].cpu().numpy(), tr["accept"][:, 1::3])


@pytest.mark.parametrize("multi,layout", [(False, "cone"), (False, "rec"), (True, "cone"), (True, "lds")])
def test_own_bit_rereads_stress(mjx_mod, multi, layout):
    """Built to expose stale own-bit reads: n = 64, d = 3,
    R = 4096 replicas, 16-proposal speculative batches, p+c-1 = 2 -- every
    batch re-reads words its lane has just flipped (the graph has 64 nodes),
    most balls are not trees (the list path), and 64 replicas share each word.
    Every replica's final configuration and step count equal the oracle's,
    and sampled traces match."""
    d, n, p, c, R, K = 3, 64, 2, 1, 4096, 400
    graphs = _graphs(mjx_mod, d, n, 16 if multi else 1, 31)
    graph_of = [r % 16 for r in range(R)] if multi else [0] * R
    seeds = list(range(R))
    src = graphs if multi else graphs[0]
    sa = mjx_mod.SAReplicas(src, p, c, seeds, graph_of=graph_of if multi else None, kernel={"spec_k": 16},
                            layout=layout)
    assert sa.layout == layout
    tr = {k: v.cpu().numpy() for k, v in sa.steps(K, trace=True).items()}
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    _check(tr, conf, t, graphs, graph_of, seeds, p, c, K, (0, 63, 64, 2047, 4095))
    for r in range(R):
        o = fast.sa_loop(graphs[graph_of[r]], p, c, seeds[r], max_steps=K)
        assert o["num_steps"] == t[r] and np.array_equal(conf[r], o["conf"]), r


@pytest.mark.parametrize("n,N_stat,seed,graph_seed", [(400, 6, 11, 60), (1000, 1, 5, 50)])
def test_sa_run_distinct_graphs_to_consensus(mjx_mod, n, N_stat, seed, graph_seed):
    """sa_run with the reference's shape -- a fresh graph per replica, run to
    m_final = 1 (code/SA_RRG.py:58-88) at SA_RRG.py's p=3, c=1 -- all
    replicas in one SAReplicas; conf / num_steps / mag_reached equal the
    oracle's runs to consensus on the same graphs (1.1e4-3e4 proposals per
    replica at n=400, 2.1e5 at n=1000; the steps-to-consensus distribution
    has a heavy tail -- another seed at n=1000 runs past 2e7)."""
    d, p, c = 4, 3, 1
    res = mjx_mod.sa_run(d, n, p, c, N_stat=N_stat, seed=seed, graph_seed=graph_seed)
    for k in range(N_stat):
        g = mjx_mod.random_regular_graph(d, n, seed=graph_seed + k)
        assert np.array_equal(res["graphs"][k], g)
        o = fast.sa_loop(g, p, c, seed + k)
        assert o["done"] == 1
        assert res["num_steps"][k] == o["num_steps"]
        assert np.array_equal(res["conf"][k], o["conf"])
        assert res["mag_reached"][k] == o["mag_reached"]
        assert res["done"][k] == 1


@pytest.mark.parametrize("d,n,p,c,kernel", [
    (3, 64, 1, 1, {}), (4, 64, 1, 1, {}), (3, 1000, 1, 1, {}), (4, 1000, 1, 1, {}),   # k_sa_lds_wg1<D,4,8,false>
    (4, 64, 3, 1, {}), (4, 1000, 3, 1, {}), (3, 500, 2, 1, {}),                       # k_sa_lds_cu<D,T,8,false>
    (4, 64, 3, 1, {"split": 16}), (4, 1000, 3, 1, {"split": 16}), (3, 500, 2, 1, {"split": 16}),   # k_sa_lds_wg<D,T,16,false>
    (4, 1000, 3, 1, {"split": 8}), (4, 64, 3, 1, {"split": 8}),                      # k_sa_lds_wg<D,T,8,false>
    (4, 1000, 3, 1, {"split": 4}), (4, 1000, 3, 1, {"lds_wave": True}), (4, 1000, 1, 1, {"lds_wave": True}),
    (4, 1000, 3, 1, {"lds_cu": True}), (4, 64, 3, 1, {"lds_cu": True}), (3, 500, 2, 1, {"lds_cu": True}),
    (4, 1000, 3, 1, {"lds_cu": True, "split": 16}),
])
def test_lds_no_trace_matches_oracle(mjx_mod, d, n, p, c, kernel):
    """The kernels run() and the bench use (no trace buffers: TRACE=false
    instantiations) against the oracle on conf, t and the MT19937 stream each
    replica hands back, over two ragged calls."""
    R, K1, K2 = 70, 700, 233
    graphs = _graphs(mjx_mod, d, n, R, 300)
    seeds = list(range(2000, 2000 + R))
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, layout="lds", kernel=kernel)
    sa.steps(K1)
    sa.steps(K2)
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    mt, idx = sa.mt_state()
    for r in (0, 1, 35, 64, 69):
        st = np.random.RandomState(seeds[r]).get_state()
        o = fast.sa_loop(graphs[r], p, c, seeds[r], max_steps=K1 + K2, mt_state=(st[1], st[2]))
        assert o["num_steps"] == t[r], r
        assert np.array_equal(conf[r], o["conf"]), r
        assert np.array_equal(mt[r], o["mt_state"][0]) and idx[r] == o["mt_state"][1], r


@pytest.mark.parametrize("n,N_stat,seed,graph_seed", [(1000, 2, 5, 70)])
def test_sa_run_global_stream_to_consensus(mjx_mod, n, N_stat, seed, graph_seed):
    """SA_RRG.py's own semantics at n = 1000: ONE numpy
    stream seeded once, the replicas back to back on it, each on a fresh graph,
    run to m_final = 1 at the script's p=3, c=1 (code/SA_RRG.py:58-88); the
    whole-CU LDS kernel on one replica at a time.  Equal to the C oracle
    continued on one MT19937 stream (4.4e4 + 4.5e4 proposals)."""
    d, p, c = 4, 3, 1
    res = mjx_mod.sa_run(d, n, p, c, N_stat=N_stat, seed=seed, graph_seed=graph_seed, stream="global")
    st = np.random.RandomState(seed).get_state()
    state = (st[1], st[2])
    for k in range(N_stat):
        g = mjx_mod.random_regular_graph(d, n, seed=graph_seed + k)
        o = fast.sa_loop(g, p, c, seed, mt_state=state)
        state = o["mt_state"]
        assert o["done"] == 1 and res["done"][k] == 1
        assert res["num_steps"][k] == o["num_steps"], k
        assert np.array_equal(res["conf"][k], o["conf"]), k
        assert res["mag_reached"][k] == o["mag_reached"], k
        assert res["wall_s"][k] > 0


@pytest.mark.parametrize("d,n,p,c,mode,layout", [
    (4, 300, 3, 1, "lightcone", "lds"),          # whole-CU kernel
    (4, 400, 1, 1, "lightcone", "lds"),          # eight proposals per step
    (3, 500, 2, 1, "lightcone", "cone"),         # HBM levels rebuilt from s on resume
    (4, 200, 1, 1, "rollout", None),
])
def test_checkpoint_resume_equals_uninterrupted(mjx_mod, tmp_path, d, n, p, c, mode, layout):
    """A long SA run (SA_RRG.py's n = 1e4 runs take 1e7-1e9 proposals per
    replica) checkpointed after K1 proposals and resumed in a new object from
    the file makes exactly the uninterrupted run's proposals: same conf, t,
    a, b, sum(s_end) and MT19937 streams after K1 + K2."""
    R, K1, K2 = 20, 600, 500
    graphs = _graphs(mjx_mod, d, n, R, 500)
    seeds = list(range(77, 77 + R))
    kw = dict(mode=mode, layout=layout or "auto", tape=0)
    ref = mjx_mod.SAReplicas(graphs, p, c, seeds, **kw)
    ref.steps(K1)
    ref.steps(K2)
    run = mjx_mod.SAReplicas(graphs, p, c, seeds, **kw)
    run.steps(K1)
    path = tmp_path / "sa_ckpt.npz"
    run.save_checkpoint(path)
    del run
    # other graphs of the same shape (or the stack reordered) are refused
    with pytest.raises(ValueError, match="other graphs"):
        mjx_mod.SAReplicas.resume(graphs[1:] + graphs[:1], str(path), mode=mode, layout=layout or "auto")
    res = mjx_mod.SAReplicas.resume(graphs, str(path), mode=mode, layout=layout or "auto")
    res.steps(K2)
    for k in ("t", "a", "b", "sum_end", "done"):
        assert torch.equal(getattr(res, k), getattr(ref, k)), k
    assert torch.equal(res.conf(), ref.conf())
    m1, i1 = res.mt_state()
    m2, i2 = ref.mt_state()
    assert np.array_equal(m1, m2) and np.array_equal(i1, i2)


@pytest.mark.parametrize("d,n,p,c,layout,kernel", [
    (4, 300, 3, 1, "lds", None),                       # k_sa_lds_cu, T = 3
    (3, 300, 2, 1, "lds", None),                       # k_sa_lds_cu, T = 2
    (4, 300, 3, 1, "lds", {"split": 16}),              # k_sa_lds_wg
    (4, 300, 3, 1, "lds", {"lds_wave": True}),         # one wave per replica
    (4, 400, 1, 1, "lds", None),                       # k_sa_lds_wg1
    (3, 500, 2, 1, "cone", None),                      # speculative batches
    (3, 500, 2, 1, "cone", {"no_spec": True}),         # one round trip
])
@pytest.mark.parametrize("cap", [29, 137])
def test_t_cap_stops_like_the_reference(mjx_mod, d, n, p, c, layout, kernel, cap):
    """The loop's other exit, t > 2n^3 (code/SA_RRG.py:84), on the device: with
    the cap lowered to `cap` every replica takes step cap+1, stops there with
    done = 2 and takes no step in later calls; its configuration and MT19937
    stream equal the reference loop's after cap+1 steps (orc_sa_loop, which
    breaks after the same step)."""
    R = 8
    graphs = [mjx_mod.random_regular_graph(d, n, seed=9100 + 10 * d + k) for k in range(R)]
    seeds = list(range(700, 700 + R))
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, layout=layout, kernel=kernel)
    sa.t_cap = cap
    sa.steps(cap // 2 + 3)                         # the cap lands inside the second call
    sa.steps(400)
    sa.steps(50)                                   # nothing left to take
    t, done = sa.t.cpu().numpy(), sa.done.cpu().numpy()
    conf = sa.conf().cpu().numpy()
    mt, idx = sa.mt_state() if layout == "lds" else (None, None)     # (a tape draws ahead of the stop)
    for r in range(R):
        st = np.random.RandomState(seeds[r]).get_state()
        o = fast.sa_loop(graphs[r], p, c, seeds[r], max_steps=cap + 1, mt_state=(st[1], st[2]))
        assert o["done"] == 0 and o["num_steps"] == cap + 1, r      # (no consensus this early)
        assert t[r] == cap + 1 and done[r] == 2, (r, t[r], done[r])
        assert np.array_equal(conf[r], o["conf"]), r
        if mt is not None:
            assert np.array_equal(mt[r], o["mt_state"][0]) and idx[r] == o["mt_state"][1], r
