"""Every BASELINE.json config exercised at its full size (C3 is
covered by tests/test_hpr_gpu.py::test_c3_size_sampled_rows).

  C1  SA_RRG.py on a d=4 RRG, N=1e4, p=c=1, 64 replicas, 1e4 proposals each:
      sampled replicas' (i, accept, sum_end, delta_H) traces and conf against
      the C restatement of code/SA_RRG.py:63-88 (oracle/orc_majority.c), in
      both SA modes; all 64 replicas identical across the modes.
  C2  d=3 RRG, N=1e6, p=2, c=1, 4096 replicas: light-cone (record layout,
      side-stream MT19937 tape) and full-rollout traces identical for every
      replica over one 3000-step call; sampled proposal columns equal
      np.random.RandomState replays; after 2000 further light-cone steps the
      cached levels equal fresh rollouts; 20 steps of two sampled replicas
      against the oracle; two callers on two streams equal sequential runs.
  C4  ER mean degree 5, N=1e7 (device generator), 4096 replicas, p+c-1 = 2:
      degree-class layout == CSR layout (words and per-replica counts); two
      sampled replicas against the oracle's s_endstate (nb:113-123).
  C5  d=6 RRG, N=1e9 on one GPU: the source-binned sweep (pieces 1 and 2)
      equals the gather sweep for 2 sweeps (words and counts); sampled nodes of
      both sweeps against the oracle's onestep_majority (code/SA_RRG.py:18-20).
"""
import functools

import numpy as np
import pytest
import torch

from oracle import fast
from oracle import majority as orc

pytestmark = pytest.mark.gpu


def _replica(bits, n, W, r):
    """+-1 int64 spins (n,) of replica r of a replica-packed array (host numpy)."""
    col = bits.view(n, W)[:, r >> 6]
    return (((col >> (r & 63)) & 1) * 2 - 1).cpu().numpy()


# ---------------------------------------------------------------- C1 --------
C1 = dict(n=10_000, d=4, p=1, c=1, R=64, K=10_000, graph_seed=1000)
C1_SAMPLED = (0, 21, 42, 63)


@functools.lru_cache(maxsize=None)
def _c1_graph():
    import mjx
    return mjx.random_regular_graph(C1["d"], C1["n"], seed=C1["graph_seed"])


@functools.lru_cache(maxsize=None)
def _c1_oracle(seed):
    return fast.sa_loop(_c1_graph(), C1["p"], C1["c"], seed, max_steps=C1["K"], trace=True)


@functools.lru_cache(maxsize=None)
def _c1_run(mode):
    import mjx
    sa = mjx.SAReplicas(_c1_graph(), C1["p"], C1["c"], list(range(C1["R"])), mode=mode)
    tr = {k: v.cpu().numpy() for k, v in sa.steps(C1["K"], trace=True).items()}
    return tr, sa.conf().cpu().numpy(), sa.t.cpu().numpy()


@pytest.mark.parametrize("mode", ["lightcone", "rollout"])
def test_c1_sa_full_size_vs_oracle(mjx_mod, mode):
    tr, conf, t = _c1_run(mode)
    assert tr["i"].shape == (C1["K"], C1["R"])
    for r in C1_SAMPLED:
        o = _c1_oracle(r)
        L = o["num_steps"]
        assert L == C1["K"] or o["done"] == 1
        ot = o["trace"]
        assert np.array_equal(tr["i"][:L, r], ot["i"]), r
        assert np.array_equal(tr["accept"][:L, r], ot["accept"]), r
        assert np.array_equal(tr["sum_end"][:L, r], ot["sum_end"]), r
        assert np.array_equal(tr["dE"][:L, r], ot["dE"]), r           # bit-exact float64
        assert np.array_equal(conf[r], o["conf"]), r
        assert int(t[r]) == L


def test_c1_modes_agree_on_every_replica(mjx_mod):
    a, ca, ta = _c1_run("lightcone")
    b, cb, tb = _c1_run("rollout")
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(ca, cb) and np.array_equal(ta, tb)


# ---------------------------------------------------------------- C2 --------
C2_K = 3000          # one call: tape chunks 128, 2048, 824 (ramp + a half reused)


def _numpy_proposals(seed, n, K):
    """The reference's draws for one replica (code/SA_RRG.py:65,73,76): s0 from
    binomial, then (randint, rand) per step, on np.random.RandomState(seed)."""
    rs = np.random.RandomState(seed)
    s0 = 2 * rs.binomial(n=1, p=0.5, size=[n]) - 1
    i = np.empty(K, dtype=np.int64)
    u = np.empty(K, dtype=np.float64)
    for t in range(K):
        i[t] = rs.randint(low=0, high=n)
        u[t] = rs.rand()
    return s0, i, u


def test_c2_sa_full_size(mjx_mod):
    """configs[1] at full size through the side-stream MT19937 tape: one
    3000-step traced call of the record layout (tape 4096: chunks drawn a chunk
    ahead on the caller stream's side stream, ramp 128 -> 2048, then the first
    half again) equals the full-rollout mode (proposals drawn in the step) on every
    replica; sampled replicas' proposal columns equal a RandomState replay."""
    n, d, p, c, R = 1_000_000, 3, 2, 1, 4096
    g = mjx_mod.random_regular_graph_device(d, n, seed=0)
    adj_h = g.adj.cpu().numpy()
    seeds = list(range(R))
    lc = mjx_mod.SAReplicas(g.adj, p, c, seeds, mode="lightcone")
    assert lc.layout == "rec" and lc.tape_cap == 4096
    ro = mjx_mod.SAReplicas(g.adj, p, c, seeds, mode="rollout")
    assert torch.equal(lc.s, ro.s)                                       # s0 draws
    W = lc.W
    sampled = (0, 1, 2047, R - 1)
    s0 = {r: _replica(lc.s, n, W, r) for r in sampled}
    K = C2_K
    ta = {k: v.cpu().numpy() for k, v in lc.steps(K, trace=True).items()}
    tb = {k: v.cpu().numpy() for k, v in ro.steps(K, trace=True).items()}
    assert ta["i"].shape == (K, R)
    for k in ta:                                                         # all 4096 replicas, every step
        assert np.array_equal(ta[k], tb[k]), k
    assert torch.equal(lc.s, ro.s) and torch.equal(lc.sum_end, ro.sum_end)
    assert torch.equal(lc.t, ro.t) and int(lc.t.min().item()) == K
    assert int(ta["accept"].sum()) > 0 and int((ta["accept"] == 0).sum()) > 0
    for r in sampled:
        want_s0, i, u = _numpy_proposals(seeds[r], n, K)
        assert np.array_equal(s0[r], want_s0), r
        assert np.array_equal(ta["i"][:, r], i), r
        # accept = rand() < min(1, exp(-delta_H)) on the traced delta_H (SA_RRG.py:74-77)
        acc = u < np.minimum(1.0, np.exp(-ta["dE"][:, r]))
        assert np.array_equal(ta["accept"][:, r].astype(bool), acc), r
    # two sampled replicas against the oracle (20 steps: 3 full rollouts each)
    for r in (0, R - 1):
        o = fast.sa_loop(adj_h, p, c, seeds[r], max_steps=20, trace=True)["trace"]
        assert np.array_equal(ta["i"][:20, r], o["i"]), r
        assert np.array_equal(ta["accept"][:20, r], o["accept"]), r
        assert np.array_equal(ta["sum_end"][:20, r], o["sum_end"]), r
        assert np.array_equal(ta["dE"][:20, r], o["dE"]), r
    del ro, ta, tb
    # 2000 more light-cone steps: the cached levels are still onestep^t(s)
    lc.steps(2000)
    cur = lc.s
    for lvl in lc.levels:
        cur = mjx_mod.rollout(g, cur, 1, words=W)
        assert torch.equal(cur, lvl)
    cnt = torch.zeros(64 * W, dtype=torch.int64, device="cuda")
    mjx_mod.rollout(g, lc.s, p + c - 1, words=W, counts=cnt)
    assert torch.equal(2 * cnt[:R] - n, lc.sum_end)
    assert int(lc.ties.sum().item()) == 0


def test_c2_two_callers_on_two_streams(mjx_mod):
    """Two independent SAReplicas (configs[1]'s graph, 1024 replicas each, the
    side-stream tape) driven in alternation on two torch streams, 600-step
    calls (past the one-stream limit of 128): every trace and final state equals
    the same runs made one after the other on the default stream.  Each caller
    stream has its own tape side stream (mjx_sa.hip tape_side_for)."""
    n, d, p, c, R = 1_000_000, 3, 2, 1, 1024
    g = mjx_mod.random_regular_graph_device(d, n, seed=0)
    sa_seeds = (list(range(R)), list(range(50_000, 50_000 + R)))
    chunks, K = 3, 600

    def run(concurrent):
        sas = [mjx_mod.SAReplicas(g.adj, p, c, sd, mode="lightcone") for sd in sa_seeds]
        torch.cuda.synchronize()
        trs = [[], []]
        if concurrent:
            streams = [torch.cuda.Stream(), torch.cuda.Stream()]
            for _ in range(chunks):
                for j in (0, 1):
                    with torch.cuda.stream(streams[j]):
                        trs[j].append(sas[j].steps(K, trace=True))
        else:
            for j in (0, 1):
                for _ in range(chunks):
                    trs[j].append(sas[j].steps(K, trace=True))
        torch.cuda.synchronize()
        out = []
        for j in (0, 1):
            tr = {k: torch.cat([t[k] for t in trs[j]]).cpu().numpy() for k in trs[j][0]}
            out.append((tr, sas[j].s.clone(), sas[j].sum_end.clone(), sas[j].t.clone()))
        return out

    seq = run(False)
    con = run(True)
    for j in (0, 1):
        ta, sa_, ea, ta_t = seq[j]
        tb, sb_, eb, tb_t = con[j]
        assert ta["i"].shape == (chunks * K, R)
        for k in ta:
            assert np.array_equal(ta[k], tb[k]), (j, k)
        assert torch.equal(sa_, sb_) and torch.equal(ea, eb) and torch.equal(ta_t, tb_t), j
    # and the first caller's proposals are its own seeds' numpy streams
    _, i, _ = _numpy_proposals(sa_seeds[0][5], n, chunks * K)
    assert np.array_equal(con[0][0]["i"][:, 5], i)


# ---------------------------------------------------------------- C4 --------
def test_c4_er_full_size(mjx_mod):
    n, R, T = 10_000_000, 4096, 2
    W = R // 64
    g = mjx_mod.erdos_renyi_device(n, 5.0 / (n - 1), seed=31)
    gen = torch.Generator(device="cuda").manual_seed(4)
    s0 = torch.randint(-2 ** 62, 2 ** 62, (n * W,), dtype=torch.int64, device="cuda", generator=gen)
    s0[: 64 * W] = -1                       # a few nodes all +1 and all -1 across replicas
    s0[64 * W: 128 * W] = 0
    ca = torch.zeros(64 * W, dtype=torch.int64, device="cuda")
    cb = torch.zeros_like(ca)
    g.rp_layout = "class"
    a = mjx_mod.rollout(g, s0, T, words=W, counts=ca)
    g.rp_layout = "csr"
    b = mjx_mod.rollout(g, s0, T, words=W, counts=cb)
    g.rp_layout = "class"
    assert torch.equal(a, b)
    assert torch.equal(ca, cb)
    del b
    rp, col = g.row_ptr.cpu().numpy(), g.col.cpu().numpy()
    for r in (0, R - 1):
        want = fast.s_endstate_er(rp, col, _replica(s0, n, W, r), T, 1)
        assert np.array_equal(_replica(a, n, W, r), want), r
        assert int(ca[r].item()) == int((want > 0).sum()), r


# ---------------------------------------------------------------- C5 --------
def _sampled_nodes_follow_the_rule(s_in, s_out, adj, n, k=4096, seed=0):
    """k random nodes of one sweep checked against the oracle's
    onestep_majority on their own neighbourhoods."""
    d = adj.shape[1]
    v = torch.from_numpy(np.random.default_rng(seed).integers(0, n, k)).cuda()
    rows = adj[v].long()                                            # (k, d)

    def bit(words, u):
        return ((words[u >> 6] >> (u & 63)) & 1).cpu().numpy().astype(np.int64)

    own = 2 * bit(s_in, v) - 1
    nb = 2 * bit(s_in, rows.reshape(-1)) - 1
    s_local = np.concatenate([own, nb])
    # local graph: node i < k is sampled node i, its neighbours are the nodes
    # k + d*i ... ; the neighbour nodes' own rows are irrelevant (row 0)
    N_local = np.zeros((k + k * d, d), dtype=np.int64)
    N_local[:k] = k + np.arange(k * d).reshape(k, d)
    want = orc.onestep_majority(N_local, s_local)[:k]
    got = 2 * bit(s_out, v) - 1
    assert np.array_equal(got, want)


def test_c5_giant_binned_equals_gather(mjx_mod):
    n, d, seed = 1_000_000_000, 6, 12345
    words = (n + 63) // 64
    sh = mjx_mod.ShardedRRG(d, n, seed=seed, mode="gather", pieces=1)
    gen = torch.Generator(device="cuda").manual_seed(99)
    init = torch.randint(-2 ** 62, 2 ** 62, (words,), dtype=torch.int64, device="cuda", generator=gen)
    sh.buf[sh.cur][:words].copy_(init)
    states, sums = [], []
    for k in range(2):
        before = sh.state_words[:words].clone()
        sh.sweep(count=True)
        _sampled_nodes_follow_the_rule(before, sh.state_words, sh.adj[0], n, seed=k)
        states.append(sh.state_words[:words].clone())
        sums.append(int(sh.cnt.item()))
        del before
    del sh
    torch.cuda.empty_cache()
    for pieces in (1, 2):
        bs = mjx_mod.ShardedRRG(d, n, seed=seed, mode="binned", pieces=pieces)
        bs.drop_adjacency()
        torch.cuda.empty_cache()
        bs.buf[bs.cur].zero_()
        bs.buf[bs.cur][:words].copy_(init)
        for k in range(2):
            bs.sweep(count=True)
            assert torch.equal(bs.state_words[:words], states[k]), (pieces, k)
            assert int(bs.cnt.item()) == sums[k], (pieces, k)
        del bs
        torch.cuda.empty_cache()
