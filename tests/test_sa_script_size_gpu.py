"""SA_RRG.py's OWN configuration on the device:
d = 4, n = 10000, p = 3, c = 1 (code/SA_RRG.py:44-52), a fresh graph per
replica (:58-62), against the C restatement of the reference's loop
(oracle/orc_majority.c, :63-88) on the same graphs and seeds.

At n = 1e4 the LDS kernels run far past the sizes of the other SA tests: the
level-synchronous whole-CU kernel k_sa_lds_cu<4,3,8> (the default here) holds
~156 KB of LDS per replica (rows as uint16 node ids, levels, 16-bit marks, the
level lists), k_sa_lds_wg<4,3,8> ~138 KB, so offsets pass 64 KB and node ids
pass 8192; k_sa_lds_wg1<4,4,8> (p = c = 1) the same graph at T = 1.  Every
check is bit for bit: conf, t, the MT19937 stream each replica hands back
(two ragged calls), and with the trace the per-step proposal, accept,
sum(s_end) and delta_H."""
import numpy as np
import pytest

from oracle import fast

pytestmark = pytest.mark.gpu

N_SCRIPT, D_SCRIPT = 10_000, 4          # code/SA_RRG.py:44-45
R_SCRIPT = 64


def _graphs(mjx_mod, R, base, n=N_SCRIPT):
    return [mjx_mod.random_regular_graph(D_SCRIPT, n, seed=base + g) for g in range(R)]


def _plan(mjx_mod, n, p, c, sa):
    lib = mjx_mod._lib.load()
    threads = mjx_mod._lib.ctypes.c_int(0)
    nbytes = lib.mjx_sa_lds_plan(n, D_SCRIPT, p, c, sa._state.opt_flags, sa._state.opt_split,
                                 mjx_mod._lib.ctypes.byref(threads))
    return int(nbytes), int(threads.value)


@pytest.mark.parametrize("p,c,K1,K2,threads_want,kernel", [
    (3, 1, 1900, 1133, 512, None),           # SA_RRG.py's p=3, c=1: k_sa_lds_cu<4,3,8,false>
    (3, 1, 1900, 1133, 1024, {"split": 16}),  # k_sa_lds_wg<4,3,16,false>, a proposal per wave
    (3, 1, 1900, 1133, 512, {"split": 8}),   # its 8-wave form (byte marks)
    (3, 1, 1900, 1133, 512, {"lds_cu": True}),   # k_sa_lds_cu<4,3,8,false>, level-synchronous
    (2, 2, 1900, 1133, 512, {"lds_cu": True}),   # k_sa_lds_cu<4,3,8,false>, T = 3 via c = 2
    (3, 1, 1900, 1133, 1024, {"lds_cu": True, "split": 16}),   # k_sa_lds_cu<4,3,16,false>
    (1, 1, 2900, 1733, 320, None),           # configs[0]'s p=c=1: k_sa_lds_wg1<4,4,8,false>, 4 waves + the parser
])
def test_script_size_no_trace_matches_oracle(mjx_mod, p, c, K1, K2, threads_want, kernel):
    """The kernels run() and the bench use (TRACE = false) at n = 1e4, 64
    replicas on 64 graphs, two ragged calls: conf, t and MT19937 stream of
    replicas 0, 1, 31 and 63 equal the oracle's."""
    graphs = _graphs(mjx_mod, R_SCRIPT, 7000 + 100 * p)
    seeds = list(range(3000, 3000 + R_SCRIPT))
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, layout="lds", kernel=kernel)
    assert sa.layout == "lds" and sa.rep_graph is not None
    nbytes, threads = _plan(mjx_mod, N_SCRIPT, p, c, sa)
    assert threads == threads_want, threads        # the whole-CU kernel
    if p + c - 1 >= 2:
        assert nbytes > 96 * 1024, nbytes          # LDS offsets well past 64 KB
    sa.steps(K1)
    sa.steps(K2)
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    mt, idx = sa.mt_state()
    assert np.all(t == K1 + K2)                    # nobody reaches consensus this early
    for r in (0, 1, 31, 63):
        st = np.random.RandomState(seeds[r]).get_state()
        o = fast.sa_loop(graphs[r], p, c, seeds[r], max_steps=K1 + K2, mt_state=(st[1], st[2]))
        assert o["num_steps"] == t[r], r
        assert np.array_equal(conf[r], o["conf"]), r
        assert np.array_equal(mt[r], o["mt_state"][0]) and idx[r] == o["mt_state"][1], r


def test_script_size_trace_matches_oracle(mjx_mod):
    """The TRACE instantiation of the whole-CU kernel at n = 1e4, p = 3:
    proposals, accepts, sum(s_end) and delta_H of replicas 0 and 63 over two
    ragged calls equal the reference loop's, step for step."""
    p, c, K1, K2 = 3, 1, 1300, 777
    graphs = _graphs(mjx_mod, R_SCRIPT, 7700)
    seeds = list(range(4000, 4000 + R_SCRIPT))
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, layout="lds")
    tr1 = {k: v.cpu().numpy() for k, v in sa.steps(K1, trace=True).items()}
    tr2 = {k: v.cpu().numpy() for k, v in sa.steps(K2, trace=True).items()}
    tr = {k: np.concatenate([tr1[k], tr2[k]]) for k in tr1}
    conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
    for r in (0, 63):
        o = fast.sa_loop(graphs[r], p, c, seeds[r], max_steps=K1 + K2, trace=True)
        L = len(o["trace"]["i"])
        assert L == t[r] == K1 + K2, r
        for key in ("i", "accept", "sum_end", "dE"):
            assert np.array_equal(tr[key][:L, r], o["trace"][key]), (r, key)
        assert np.array_equal(conf[r], o["conf"]), r
    # the schedule really anneals here: both accepts and rejects occur
    acc = tr["accept"][:, [0, 63]]
    assert (acc == 0).any() and (acc == 1).any()


def test_script_size_global_stream_window(mjx_mod):
    """SA_RRG.py literally at its size: ONE numpy stream seeded once, N_stat
    replicas back to back on it, each on a fresh graph (code/SA_RRG.py:58-88),
    the whole-CU kernel on one replica at a time (R = 1), 5000 proposals per
    replica (sa_run's chunks 256, 512, ... make the calls ragged).  Equal to
    the C oracle continued on one MT19937 stream: conf, num_steps,
    mag_reached, and the second replica starts where the first left the
    stream."""
    d, n, p, c, seed, gs, K = D_SCRIPT, N_SCRIPT, 3, 1, 9, 8800, 5000
    res = mjx_mod.sa_run(d, n, p, c, N_stat=2, seed=seed, graph_seed=gs, stream="global", max_steps=K)
    st = np.random.RandomState(seed).get_state()
    state = (st[1], st[2])
    for k in range(2):
        g = mjx_mod.random_regular_graph(d, n, seed=gs + k)
        assert np.array_equal(res["graphs"][k], g)
        o = fast.sa_loop(g, p, c, seed, max_steps=K, mt_state=state)
        state = o["mt_state"]
        assert res["num_steps"][k] == o["num_steps"] == K, k
        assert np.array_equal(res["conf"][k], o["conf"]), k
        assert res["mag_reached"][k] == o["mag_reached"], k


def test_lds_opt_in_survives_a_smaller_call(mjx_mod):
    """One kernel instance at n = 1e4, then n = 1e3, then n = 1e4 again in one
    process (the dynamic-LDS opt-in is kept at its largest value
    per device and kernel, never lowered by a smaller launch); every run equals
    the oracle."""
    p, c, K = 3, 1, 300
    for n in (N_SCRIPT, 1000, N_SCRIPT):
        graphs = _graphs(mjx_mod, 4, 9100 + n, n=n)
        seeds = [11, 12, 13, 14]
        sa = mjx_mod.SAReplicas(graphs, p, c, seeds, layout="lds")
        sa.steps(K)
        conf, t = sa.conf().cpu().numpy(), sa.t.cpu().numpy()
        for r in (0, 3):
            o = fast.sa_loop(graphs[r], p, c, seeds[r], max_steps=K)
            assert o["num_steps"] == t[r] and np.array_equal(conf[r], o["conf"]), (n, r)
