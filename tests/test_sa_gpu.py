"""GPU parity of the simulated-annealing path (rows a5-a6 of SURVEY.md 8a).

Bar: bit-exact — the proposal sequence i_t, every accept decision, every
sum(s_endstate) and delta_H (float64, same operation order), the final conf,
num_steps and mag_reached equal the reference's (tests/golden/sa_*.npz were
produced by the reference's own SA code on numpy's seeded global stream).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import fast
from oracle import majority as orc

pytestmark = pytest.mark.gpu


def test_sa_init_draws_reference_s0(mjx_mod):
    z = load_golden("sa_d4_n200_p3c1.npz")
    seeds = [int(s) for s in z["seeds"]]
    sa = mjx_mod.SAReplicas(z["N"], 3, 1, seeds)
    conf = sa.conf().cpu().numpy()
    for r, sd in enumerate(seeds):
        assert np.array_equal(conf[r], z[f"seed{sd}_s0"])
    # s0 of many seeds against numpy directly (ragged R, n not multiple of 64)
    n = 777
    adj = mjx_mod.random_regular_graph(4, n, seed=1)
    seeds = list(range(1000, 1000 + 150))
    sa = mjx_mod.SAReplicas(adj, 1, 1, seeds)
    conf = sa.conf().cpu().numpy()
    for r, sd in enumerate(seeds):
        rs = np.random.RandomState(sd)
        assert np.array_equal(conf[r], 2 * rs.binomial(n=1, p=0.5, size=[n]) - 1)


def _sa(mjx_mod, N, p, c, seeds, mode):
    """mode: "lightcone" (HBM cone layout, default tape), "lightcone-notape"
    (draws inside the step kernel), "lightcone-tape7" (tape chunks of 7
    steps), "lightcone-lds" (graph, levels and stream in LDS, two proposals per
    step, eight at p+c-1 = 1; "-ldspair" two, "-ldssingle" one, "-ldsserial"
    the list-based step), "lightcone-rec"
    (the cone with the adjacency rows in its records), "rollout"."""
    tape = {"lightcone-notape": 0, "lightcone-tape7": 7}.get(mode, 1024)
    layout = {"lightcone-lds": "lds", "lightcone-ldsserial": "lds", "lightcone-ldssingle": "lds",
              "lightcone-ldspair": "lds", "lightcone-rec": "rec"}.get(mode, "cone")
    kernel = {"lightcone-ldsserial": {"lds_serial": True}, "lightcone-ldssingle": {"lds_single": True},
              "lightcone-ldspair": {"lds_pair": True}}.get(mode)
    return mjx_mod.SAReplicas(N, p, c, seeds, mode=mode.split("-")[0], tape=tape, layout=layout, kernel=kernel)


MODES = ["lightcone", "lightcone-notape", "lightcone-tape7", "lightcone-lds", "lightcone-ldsserial",
         "lightcone-ldssingle", "lightcone-ldspair", "lightcone-rec", "rollout"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name", ["sa_d4_n200_p3c1.npz", "sa_d3_n300_p2c1.npz", "sa_d4_n200_p1c1.npz",
                                  "sa_d4_n1000_p2c2.npz"])
def test_sa_trace_bit_exact(mjx_mod, name, mode):
    z = load_golden(name)
    N, p, c = z["N"], int(z["p"]), int(z["c"])
    seeds = [int(s) for s in z["seeds"]]
    sa = _sa(mjx_mod, N, p, c, seeds, mode)
    assert sa.mode == mode.split("-")[0]
    lens = [len(z[f"seed{sd}_i"]) for sd in seeds]
    steps = max(lens)
    done_at = 0
    chunk = 2000
    while done_at < steps:
        k = min(chunk, steps - done_at)
        tr = {key: v.cpu().numpy() for key, v in sa.steps(k, trace=True).items()}
        for r, sd in enumerate(seeds):
            L = lens[r]
            lo, hi = done_at, min(done_at + k, L)
            if hi > lo:
                sl = slice(0, hi - lo)
                assert np.array_equal(tr["i"][sl, r], z[f"seed{sd}_i"][lo:hi]), (sd, lo)
                assert np.array_equal(tr["accept"][sl, r], z[f"seed{sd}_accept"][lo:hi]), (sd, lo)
                assert np.array_equal(tr["sum_end"][sl, r], z[f"seed{sd}_sum_end"][lo:hi]), (sd, lo)
                assert np.array_equal(tr["dE"][sl, r], z[f"seed{sd}_dE"][lo:hi]), (sd, lo)
            if hi - lo < k and int(z[f"seed{sd}_converged"]):
                # replica finished inside this chunk: it must be frozen afterwards
                assert (tr["i"][hi - lo:, r] == -1).all()
                assert (tr["accept"][hi - lo:, r] == -1).all()
        done_at += k
    res = sa.results()
    for r, sd in enumerate(seeds):
        if int(z[f"seed{sd}_converged"]):
            assert res["done"][r] == 1
            assert res["num_steps"][r] == float(z[f"seed{sd}_num_steps"])
            assert np.array_equal(res["conf"][r], z[f"seed{sd}_conf"])
            assert res["mag_reached"][r] == float(z[f"seed{sd}_mag_reached"])
        else:
            assert np.array_equal(res["conf"][r], z[f"seed{sd}_conf"])
    assert int(res["near_ties"].sum()) == 0


@pytest.mark.parametrize("d,p,c", [(4, 2, 2), (3, 2, 1), (6, 2, 1), (5, 1, 2)])
def test_sa_lightcone_levels_stay_consistent(mjx_mod, d, p, c):
    """After many accepted flips the cached levels the light-cone kernel keeps
    up to date must equal fresh rollouts of the current configuration
    (d = 3, 4, 6: batched-load evaluation; d = 5: the generic one)."""
    n = 2000
    adj = mjx_mod.random_regular_graph(d, n, seed=9)
    sa = mjx_mod.SAReplicas(adj, p, c, list(range(130)), mode="lightcone", layout="cone")
    sa.steps(3000)
    W = sa.W
    g = mjx_mod.Graph.ell(adj)
    cur = sa.s
    for lvl in sa.levels:
        cur = mjx_mod.rollout(g, cur, 1, words=W)
        assert torch.equal(cur, lvl)
    assert torch.equal(sa.cone_level0(), sa.s)       # level 0 of the cone mirrors s
    cnt = torch.zeros(64 * W, dtype=torch.int64, device="cuda")
    mjx_mod.rollout(g, sa.s, p + c - 1, words=W, counts=cnt)
    assert torch.equal(2 * cnt[:sa.R] - n, sa.sum_end)


@pytest.mark.parametrize("d,p,c,kernel", [(3, 2, 1, "spec8"), (3, 2, 1, "spec16"), (3, 2, 1, "one_trip"),
                                          (3, 2, 1, "lightcone"), (3, 1, 1, "spec8"), (3, 1, 1, "spec16"),
                                          (4, 1, 1, "spec8"), (4, 1, 1, "spec16"), (4, 1, 1, "lightcone"),
                                          (4, 2, 2, ""), (5, 1, 2, ""), (3, 3, 4, "")])
@pytest.mark.parametrize("layout", ["cone", "rec"])
def test_sa_cone_layout_equals_separate_levels(mjx_mod, d, p, c, kernel, layout):
    """The cone layout (levels of one (node, word) side by side) gives the
    same proposals, accepts, sums and delta_H as separate level arrays, and
    the same final configuration and levels (LV = 2, 4 and 8 words).  At
    d=3, p+c-1=2 three kernels run on the cone: the speculative 8-proposal
    batches of 8 or 16 proposals (default; also d=3 and d=4 at p+c-1=1), the one-round-trip step
    (no_spec) and the general light-cone step (no_spec + no_cone2), chosen
    through the state's kernel options.  ``rec``: the same with every node's
    adjacency row in its records (d <= 4)."""
    if layout == "rec" and (d > 4 or p + c - 1 > 5):
        pytest.skip("record layout: d <= 4, p+c-1 <= 5")
    opts = {"spec16": {"spec_k": 16}, "spec8": {"spec_k": 8}, "one_trip": {"no_spec": True},
            "lightcone": {"no_spec": True, "no_cone2": True}}.get(kernel, {})
    n = 3000
    adj = mjx_mod.random_regular_graph(d, n, seed=4)
    R = 150
    a = mjx_mod.SAReplicas(adj, p, c, list(range(R)), mode="lightcone", layout=layout, kernel=opts)
    b = mjx_mod.SAReplicas(adj, p, c, list(range(R)), mode="lightcone", layout="levels")
    assert a.cone is not None and b.cone is None
    for k in (7, 600, 1500):
        ta, tb = a.steps(k, trace=True), b.steps(k, trace=True)
        for key in ("i", "accept", "sum_end", "dE"):
            assert torch.equal(ta[key], tb[key]), key
    assert torch.equal(a.s, b.s)
    for la, lb in zip(a.levels, b.levels):
        assert torch.equal(la, lb)
    for f in ("a", "b", "t", "sum_end", "done", "ties"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def _rec_neighbour_words_ok(rec, n, W):
    """The record layout's neighbour words (d = 3, p+c-1 = 2; include/mjx.h
    mjx_sa_rec_words): replica q's level-1 bit of row neighbour y at bit
    3*(q % 10) + y of 32-bit word q // 10 (words 0..5 in bytes 40..63, word 6
    in the row's pad int), recomputed here from the records' rows and levels."""
    r = rec.cpu().numpy().view(np.uint64).reshape(W, n, 8)
    rows = r[:, :, :2].copy().view(np.int32).reshape(W, n, 4)[:, :, :3].astype(np.int64)
    lev1 = r[:, :, 3]
    u32 = r[:, :, 5:8].copy().view(np.uint32).reshape(W, n, 6)
    pad = r[:, :, :2].copy().view(np.uint32).reshape(W, n, 4)[:, :, 3]
    got = np.concatenate([u32, pad[:, :, None]], axis=2)
    want = np.zeros_like(got)
    for w in range(W):
        L = lev1[w][rows[w]]                                  # (n, 3) neighbours' level-1 words
        for q in range(64):
            bits = ((L >> np.uint64(q)) & np.uint64(1)).astype(np.uint32)
            for y in range(3):
                want[w, :, q // 10] |= bits[:, y] << np.uint32(3 * (q % 10) + y)
    return np.array_equal(got, want)


def test_sa_rec_neighbour_words_across_kernels(mjx_mod):
    """d = 3, p+c-1 = 2 records carry their neighbours' level-1 bits for the
    speculative batches (round 6: no separate round trip for the children's
    other neighbours).  Calls alternate between the speculative kernel (keeps
    the words) and the general light-cone kernel (leaves them stale; the next
    speculative call rebuilds them): every call equals separate level arrays,
    and after speculative calls the words equal a recomputation from the
    records' rows and level-1 words."""
    n, d, p, c, R = 3000, 3, 2, 1, 150
    adj = mjx_mod.random_regular_graph(d, n, seed=11)
    a = mjx_mod.SAReplicas(adj, p, c, list(range(R)), mode="lightcone", layout="rec")
    b = mjx_mod.SAReplicas(adj, p, c, list(range(R)), mode="lightcone", layout="levels")
    assert _rec_neighbour_words_ok(a.cone, n, a.W)             # as packed
    general = mjx_mod._lib.MJX_SA_NO_SPEC | mjx_mod._lib.MJX_SA_NO_CONE2
    for k, flags in ((700, 0), (300, general), (900, 0), (5, general), (400, 0)):
        a._state.opt_flags = flags
        ta, tb = a.steps(k, trace=True), b.steps(k, trace=True)
        for key in ("i", "accept", "sum_end", "dE"):
            assert torch.equal(ta[key], tb[key]), (k, flags, key)
        assert a._state.rec_nb == (0 if flags else 1)
        if not flags:
            torch.cuda.synchronize()
            assert _rec_neighbour_words_ok(a.cone, n, a.W), k
    assert torch.equal(a.s, b.s)
    for la, lb in zip(a.levels, b.levels):
        assert torch.equal(la, lb)


def test_sa_run_matches_full_reference_script(mjx_mod):
    full = load_golden("sa_fullscript.npz")
    N = full["n200_d4_p3_graphs"][0]
    res = mjx_mod.sa_run(4, 200, 3, 1, N_stat=1, seeds=[0], N=N)
    assert res["num_steps"][0] == full["n200_d4_p3_num_steps"][0]
    assert np.array_equal(res["conf"][0], full["n200_d4_p3_conf"][0])
    assert res["mag_reached"][0] == full["n200_d4_p3_mag_reached"][0]
    assert np.array_equal(res["graphs"][0], N)


@pytest.mark.parametrize("mode", MODES)
def test_sa_many_replicas_vs_oracle(mjx_mod, mode):
    """R = 200 replicas (ragged: 4 words, 56 padding bits) on a fresh graph,
    600 steps, sampled replicas' accept sequences against the oracle."""
    n, d, p, c = 500, 3, 2, 1
    adj = mjx_mod.random_regular_graph(d, n, seed=42)
    seeds = list(range(200))
    sa = _sa(mjx_mod, adj, p, c, seeds, mode)
    tr = {k: v.cpu().numpy() for k, v in sa.steps(600, trace=True).items()}
    for r in (0, 1, 63, 64, 127, 199):
        o = orc.sa_loop(adj, p, c, seeds[r], max_steps=600, trace=True)["trace"]
        L = len(o["i"])
        assert np.array_equal(tr["i"][:L, r], o["i"])
        assert np.array_equal(tr["accept"][:L, r], o["accept"])
        assert np.array_equal(tr["sum_end"][:L, r], o["sum_end"])
        assert np.array_equal(tr["dE"][:L, r], o["dE"])


def test_E_delta_matches_oracle(mjx_mod):
    z = load_golden("rrg_dyn.npz")
    N, s0 = z["d4_n1000_N"], z["d4_n1000_s0"][0]
    for (a, b, p, c, i) in [(15.0, 10.0, 1, 1, 3), (150.3, 77.7, 2, 1, 999), (1.5, 4000.0, 3, 1, 0)]:
        assert mjx_mod.E_delta(N, s0, a, b, p, c, i) == orc.E_delta(N, s0, a, b, p, c, i)


@pytest.mark.parametrize("split", ["1", "4", "64"])
def test_sa_lightcone_wave_split_is_bit_exact(mjx_mod, split):
    """Waves per word column (1, 4, 64 replicas per wave ... 1) only change the
    schedule: the accept sequences equal the oracle's."""
    n, d, p, c = 400, 3, 2, 1
    adj = mjx_mod.random_regular_graph(d, n, seed=5)
    sa = mjx_mod.SAReplicas(adj, p, c, list(range(70)), mode="lightcone", layout="cone",
                            kernel={"split": int(split), "no_spec": True, "no_cone2": True})
    tr = {k: v.cpu().numpy() for k, v in sa.steps(300, trace=True).items()}
    for r in (0, 5, 63, 64, 69):
        o = orc.sa_loop(adj, p, c, r, max_steps=300, trace=True)["trace"]
        L = len(o["i"])
        assert np.array_equal(tr["accept"][:L, r], o["accept"])
        assert np.array_equal(tr["sum_end"][:L, r], o["sum_end"])


def _ref_sa_arrays(full, key):
    return {k: full[f"{key}_{k}"] for k in ("mag_reached", "num_steps", "conf", "graphs")}


@pytest.mark.parametrize("mode", ["lightcone", "rollout"])
def test_sa_run_global_stream_two_replicas_to_npz(mjx_mod, mode, tmp_path):
    """SA_RRG.py with N_stat = 2 end to end: one numpy stream seeded once and
    consumed by the replicas back to back, a graph per replica (:58-65), and
    the np.savez file (:92) equal to the one the reference script wrote
    (keys, dtypes, values)."""
    full = load_golden("sa_fullscript.npz")
    ref = _ref_sa_arrays(full, "n200_d4_p3_nstat2")
    res = mjx_mod.sa_run(4, 200, 3, 1, N_stat=2, seed=11, graphs=list(ref["graphs"]), stream="global", mode=mode)
    assert list(res["done"]) == [1, 1]
    path = tmp_path / "MCMC_p3_d4.npz"
    mjx_mod.save_sa_npz(path, res)
    with np.load(path) as z:
        assert sorted(z.files) == sorted(ref)
        for k in ref:
            assert z[k].dtype == ref[k].dtype, k
            assert np.array_equal(z[k], ref[k]), k


def test_sa_run_single_replica_to_npz(mjx_mod, tmp_path):
    full = load_golden("sa_fullscript.npz")
    ref = _ref_sa_arrays(full, "n200_d4_p3")
    res = mjx_mod.sa_run(4, 200, 3, 1, N_stat=1, seed=0, graphs=list(ref["graphs"]), stream="global")
    path = tmp_path / "sa.npz"
    mjx_mod.save_sa_npz(path, res)
    with np.load(path) as z:
        for k in ref:
            assert z[k].dtype == ref[k].dtype and np.array_equal(z[k], ref[k]), k


def test_sa_run_independent_per_replica_graphs(mjx_mod):
    """Independent streams, a fresh graph per replica: replica k equals the
    oracle run on its own graph with seed k (first 400 steps)."""
    res = mjx_mod.sa_run(3, 300, 2, 1, N_stat=3, seed=40, graph_seed=7, max_steps=400)
    g = res["graphs"]
    assert g.shape == (3, 300, 3) and not np.array_equal(g[0], g[1])
    for k in range(3):
        o = orc.sa_loop(g[k], 2, 1, 40 + k, max_steps=400)
        assert np.array_equal(res["conf"][k], o["conf"]), k
        assert res["num_steps"][k] == o["num_steps"], k


@pytest.mark.parametrize("d,p,c,kern", [(4, 3, 1, None), (4, 3, 1, "lds_serial"), (4, 3, 1, "lds_single"),
                                        (3, 2, 1, None), (4, 1, 1, None), (4, 1, 1, "lds_single"),
                                        (4, 1, 1, "lds_pair"), (3, 1, 1, None)])
def test_sa_lds_stream_position_in_ragged_calls(mjx_mod, d, p, c, kern):
    """The LDS-resident steps parse the numpy stream 64 words at a time
    (the paired step carries a leftover proposal into the next window) and
    hand back the index after the last proposal consumed: calls of
    ragged lengths (1, 2, 3, 5, 7, ... steps) give the oracle's trace, and the
    MT19937 state after them equals numpy's RandomState after the same draws
    (binomial s0, then randint(0, n) and rand() per proposal,
    code/SA_RRG.py:65,73,76) -- twists included."""
    n, R = 300, 3
    graphs = [mjx_mod.random_regular_graph(d, n, seed=70 + g) for g in range(R)]
    seeds = [17, 18, 19]
    kernel = {kern: True} if kern else None
    sa = mjx_mod.SAReplicas(graphs, p, c, seeds, layout="lds", kernel=kernel)
    got = {k: [] for k in ("i", "accept", "sum_end", "dE")}
    total = 0
    for k in [1, 2, 3, 5, 7, 11, 1, 64, 65, 129, 3, 200]:
        tr = sa.steps(k, trace=True)
        for key in got:
            got[key].append(tr[key].cpu().numpy())
        total += k
    got = {key: np.concatenate(v) for key, v in got.items()}
    mt, idx = sa.mt_state()
    for r in range(R):
        o = fast.sa_loop(graphs[r], p, c, seeds[r], max_steps=total, trace=True)
        L = len(o["trace"]["i"])
        for key in got:
            assert np.array_equal(got[key][:L, r], o["trace"][key]), (r, key)
        rs = np.random.RandomState(seeds[r])
        rs.binomial(n=1, p=0.5, size=[n])
        for _ in range(L):
            rs.randint(low=0, high=n)
            rs.rand()
        st = rs.get_state()
        assert np.array_equal(mt[r], st[1].astype(np.uint32)) and int(idx[r]) == st[2], r


def test_tape_side_stream_cache_with_a_fresh_stream_per_call(mjx_mod):
    """A caller that makes a fresh stream for every call: 70 calls of 200
    steps (the side-stream tape path, > 128 steps a call) on 70 new streams
    retire idle entries of the per-stream side-stream cache past 64 (no
    unbounded growth) and give the same traces as the same calls on one
    stream."""
    n, d, p, c, R = 3000, 3, 2, 1, 128
    adj = mjx_mod.random_regular_graph(d, n, seed=13)
    runs = []
    for fresh in (False, True):
        sa = mjx_mod.SAReplicas(adj, p, c, list(range(R)), mode="lightcone", layout="rec")
        torch.cuda.synchronize()
        trs = []
        for _ in range(70):
            if fresh:
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    tr = sa.steps(200, trace=True)
                torch.cuda.current_stream().wait_stream(st)
            else:
                tr = sa.steps(200, trace=True)
            trs.append({k: v.cpu().numpy() for k, v in tr.items()})
        runs.append((trs, sa.s.cpu().numpy()))
    (ta, sa_), (tb, sb_) = runs
    for x, y in zip(ta, tb):
        for k in x:
            assert np.array_equal(x[k], y[k]), k
    assert np.array_equal(sa_, sb_)
