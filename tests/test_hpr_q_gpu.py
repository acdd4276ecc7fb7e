"""The decay-split layout of the HPR loop state (mjx_hpr_impl.h, HPRState
layout="q"): entries with an invalid sender trajectory are kept as chi_0 and
read with the scale (1-damp)^t, because HPr_dp only damps them
(code/HPR_pytorch_RRG.py:215 with chi_mat2 = 0 there).

Bar: one step from the reference's own state matches the reference's next
state within the fp32 tolerance (1e-5 row-normalised), marginals
within 1e-5; the layout permutation round-trips exactly; at configs[2] size one
q-layout step equals one reference-layout step within 1e-6; hipGraph batches
equal eager steps bit for bit.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

Q_CASES = ["hpr_d4_n64_p2c2.npz", "hpr_d3_n40_p3c1.npz"]


def rownorm_err(got, ref):
    got = np.asarray(got, dtype=np.float64)
    return float(np.max(np.abs(got - ref) / np.max(np.abs(ref), axis=1, keepdims=True)))


@pytest.mark.parametrize("attr", [1, -1])
def test_qlayout_round_trip(mjx_mod, attr):
    lib = mjx_mod.load_library()
    st = torch.cuda.current_stream().cuda_stream
    for p, c in ((2, 2), (1, 2), (3, 2)):
        nc = 4 ** (p + c)
        x = torch.rand((37, nc), dtype=torch.float32, device="cuda")
        q = torch.empty_like(x)
        back = torch.empty_like(x)
        assert lib.mjx_hpr_qlayout(mjx_mod._lib.MJX_F32, x.data_ptr(), q.data_ptr(), 37, p, c, attr, 1, 1.0, st) == 0
        assert lib.mjx_hpr_qlayout(mjx_mod._lib.MJX_F32, q.data_ptr(), back.data_ptr(), 37, p, c, attr, 0, 1.0, st) == 0
        assert torch.equal(back, x)
        assert not torch.equal(q, x)
        # scale: only the invalid-sender entries (x_s[T-1] != attr) are scaled
        assert lib.mjx_hpr_qlayout(mjx_mod._lib.MJX_F32, q.data_ptr(), back.data_ptr(), 37, p, c, attr, 0, 0.5, st) == 0
        X = 2 ** (p + c)
        xs = np.repeat(np.arange(X), X)
        invalid = (xs & 1) != (0 if attr > 0 else 1)
        want = x.cpu().numpy().copy()
        want[:, invalid] *= np.float32(0.5)
        assert np.array_equal(back.cpu().numpy(), want)


@pytest.mark.parametrize("name", Q_CASES)
def test_q_step_vs_reference(mjx_mod, name):
    """Every step from the reference's own state (fp32): messages() after one
    q-layout step vs the reference's next chi; the marginals the step computes
    vs the reference's."""
    z = load_golden(name)
    n, d, p, c = (int(z[k]) for k in ("n", "d", "p", "c"))
    assert p + c == 4 and d <= 4
    plan = mjx_mod.HPRPlan(z["edges"], n, d, z["N_nodes"])
    for k in range(int(z["chain"])):
        chi = z["chi0"] if k == 0 else z[f"it{k - 1}_chi"]
        b = z["biases0"] if k == 0 else z[f"it{k - 1}_biases"]
        st = mjx_mod.HPRState(plan, p, c, chi, b, dtype=torch.float32, damppar=float(z["damppar"]),
                              attr_value=int(z["attr_value"]), lmbd_in=int(z["lmbd_in"]), pie=float(z["pie"]),
                              gamma=float(z["gamma"]))
        assert st.layout == "q"
        st.t = k                       # the reference's t (threshold); the decay restarts at this state
        st._t0 = k
        st.step(u=z[f"it{k}_u"])
        # messages() scales by (1-damp)^(updates since construction) = one
        got = st.messages().cpu().numpy()
        assert rownorm_err(got, z[f"it{k}_chi"]) <= 1e-5, k
        assert float(np.max(np.abs(st.marg.cpu().double().numpy() - z[f"it{k}_marg"]))) <= 1e-5, k
        assert np.array_equal(st.s.cpu().numpy(), z[f"it{k}_s"]), k


def _pair(mjx_mod, n, d, p, c, seed=0):
    edges = mjx_mod.random_regular_edges(d, n, seed=seed)
    plan = mjx_mod.HPRPlan(edges, n, d)
    g = torch.Generator().manual_seed(seed)
    nc = 4 ** (p + c)
    chi0 = torch.rand((2 * plan.E, nc), dtype=torch.float64, generator=g)
    chi0 /= chi0.sum(1, keepdim=True)
    b0 = torch.rand((n, 2), dtype=torch.float64, generator=g)
    b0 /= b0.sum(1, keepdim=True)
    mk = lambda layout: mjx_mod.HPRState(plan, p, c, chi0, b0, dtype=torch.float32, layout=layout)  # noqa: E731
    return plan, mk


def test_q_equals_ref_layout_at_c3_size(mjx_mod):
    """configs[2] (d=4, N=1e5, p=c=2, fp32): three steps in both layouts from
    the same state and uniforms give the same messages (1e-6 row-normalised)
    and marginals."""
    n, d, p, c = 100_000, 4, 2, 2
    plan, mk = _pair(mjx_mod, n, d, p, c, seed=4)
    a, b = mk("q"), mk("ref")
    rng = np.random.default_rng(0)
    for k in range(3):
        u = rng.random(n)
        sa, sb = a.step(u=u), b.step(u=u)
        assert rownorm_err(a.messages().cpu().numpy(), b.messages().cpu().double().numpy()) <= 1e-6, k
        assert float((a.marg - b.marg).abs().max()) <= 1e-6, k
        assert sa == sb, k


def test_q_graph_batches_equal_eager(mjx_mod):
    """hipGraph-replayed batches of the q layout (node step fused into one
    launch) equal the eager steps bit for bit."""
    n, d, p, c = 2000, 3, 3, 1
    plan, mk = _pair(mjx_mod, n, d, p, c, seed=7)
    a, b = mk("q"), mk("q")
    ga, gb = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    for _ in range(3):                          # eager, capture, replay
        sums, _, _ = a.steps_batched(4, ga, graph=True)
    want = [b.step(generator=gb) for _ in range(12)]
    assert a.t == b.t == 12
    assert torch.equal(a.messages(), b.messages())
    # the batches' fused node step (mjx_hpr_node_step) vs marginals + new_biases_i
    assert torch.equal(a.biases, b.biases) and torch.equal(a.marg, b.marg) and torch.equal(a.s, b.s)
    assert int(sums[-1]) == want[-1]


def test_q_batches_track_ref_layout(mjx_mod):
    """Batched (hipGraph) iterations of the loop in both layouts (fp32, d=4,
    p=c=2) from one state and one random stream: the same trial
    configurations over 16 iterations and messages within 1e-5; hpr_run in
    the q layout ends with the reference's output keys (a whole run is not
    compared: fp32 rounding of the two layouts differs by ulps, and the
    reinforcement is chaotic over hundreds of iterations)."""
    n, d, p, c = 400, 4, 2, 2
    plan, mk = _pair(mjx_mod, n, d, p, c, seed=2)
    a, b = mk("q"), mk("ref")
    ga, gb = torch.Generator().manual_seed(5), torch.Generator().manual_seed(5)
    for _ in range(2):
        sa, ha, _ = a.steps_batched(8, ga)
        ha = ha.clone()
        sb, hb, _ = b.steps_batched(8, gb)
        assert np.array_equal(sa, sb)
        assert torch.equal(ha, hb)
    assert rownorm_err(a.messages().cpu().numpy(), b.messages().cpu().double().numpy()) <= 1e-5
    edges = mjx_mod.random_regular_edges(d, n, seed=2)
    res = mjx_mod.hpr_run(d, n, p, c, TT=60, edges=edges, seed=5, dtype=torch.float32, layout="q")
    assert set(res) == {"mag_reached", "num_steps", "conf", "graphs"}
    assert res["conf"].shape == (1, n) and 1 <= res["num_steps"][0] <= 61


def test_marginals_q_precomputed_ii_equals_full_read(mjx_mod):
    """The II x II sums precomputed once (mjx_hpr_q_ii) give the marginals of
    the full read (ii = NULL) and of the reference layout, at a decayed
    scale, within 1e-6 (fp32)."""
    lib = mjx_mod.load_library()
    F32 = mjx_mod._lib.MJX_F32
    n, d, p, c = 20_000, 4, 2, 2
    plan, mk = _pair(mjx_mod, n, d, p, c, seed=9)
    a = mk("q")
    st = torch.cuda.current_stream().cuda_stream
    sc = torch.tensor([0.6 ** 3], dtype=torch.float32, device="cuda")
    z = torch.empty(4 * plan.E, dtype=torch.float32, device="cuda")
    m_ii = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    m_full = torch.empty_like(m_ii)
    for ii, out in ((a._ii.data_ptr(), m_ii), (None, m_full)):
        assert lib.mjx_hpr_marginals_q(F32, a.chi.data_ptr(), plan.out_row.data_ptr(), n, d, p, c, 1e-15,
                                       sc.data_ptr(), ii, z.data_ptr(), out.data_ptr(), st) == 0
    assert float((m_ii - m_full).abs().max()) <= 1e-6
    ref = torch.empty(a.chi.shape, dtype=torch.float32, device="cuda")
    assert lib.mjx_hpr_qlayout(F32, a.chi.data_ptr(), ref.data_ptr(), a.chi.shape[0], p, c, 1, 0, 0.6 ** 3, st) == 0
    m_ref = mjx_mod.marginals_comp(ref, plan, p, c)
    assert float((m_ii - m_ref).abs().max()) <= 1e-6


@pytest.mark.parametrize("pre,n,k", [(0, 1000, 3), (3, 4097, 2), (1000, 313, 5), (311, 624, 4)])
def test_device_refresh_masks_equal_torch_cpu_stream(mjx_mod, pre, n, k):
    """mjx_hpr_refresh_masks continues torch's CPU generator on the device: the
    masks equal torch.rand(n) < thresh drawn on the CPU (code/HPR_pytorch_RRG.py:
    142), from a fresh generator and from positions mid-block (odd word
    counts), and the state handed back is the CPU generator's."""
    plan, mk = _pair(mjx_mod, 64, 4, 2, 2, seed=1)
    st = mk("q")
    g = torch.Generator().manual_seed(7)
    if pre:
        torch.rand(pre, dtype=torch.float64, generator=g)
    h = torch.Generator()
    h.set_state(g.get_state())
    st.rng_attach(g)
    thr = [0.1 * (j + 1) for j in range(k)]
    lib = mjx_mod.load_library()
    mask = torch.empty((k, n), dtype=torch.uint8, device="cuda")
    th = torch.tensor(thr, dtype=torch.float64, device="cuda")
    assert lib.mjx_hpr_refresh_masks(st._mt.data_ptr(), st._ln.data_ptr(), n, k, th.data_ptr(), mask.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream) == 0
    want = torch.stack([torch.rand(n, dtype=torch.float64, generator=h) < thr[j] for j in range(k)])
    assert torch.equal(mask.cpu().bool(), want)
    g2 = torch.Generator()
    g2.set_state(st.rng_state_bytes())
    assert torch.equal(torch.rand(9, dtype=torch.float64, generator=g2), torch.rand(9, dtype=torch.float64, generator=h))


@pytest.mark.parametrize("pre,n,k,G", [(0, 1000, 3, 256), (3, 4097, 2, 7), (1000, 313, 5, 2), (311, 624, 4, 256),
                                       (0, 100, 1, 256), (623, 100_000, 16, 256)])
def test_jump_refresh_masks_equal_torch_cpu_stream(mjx_mod, pre, n, k, G):
    """mjx_hpr_refresh_masks_jump (G workgroups, each jumping the batch-start
    state ahead by z^(jL-1) mod P): the same masks as torch.rand(n) < thresh
    drawn on the CPU (code/HPR_pytorch_RRG.py:142) and the CPU generator's
    state handed back, from fresh and mid-block stream positions, down to a
    single chunk and up to the C3 batch (n = 1e5, 16 iterations)."""
    import numpy as np
    plan, mk = _pair(mjx_mod, 64, 4, 2, 2, seed=1)
    st = mk("q")
    g = torch.Generator().manual_seed(9)
    if pre:
        torch.rand(pre, dtype=torch.float64, generator=g)
    h = torch.Generator()
    h.set_state(g.get_state())
    st.rng_attach(g)
    thr = [0.05 + 0.9 * j / k for j in range(k)]
    lib = mjx_mod.load_library()
    words = lib.mjx_mt_jump_table_words(n, k, G)
    assert words >= 0
    table = None
    if words:
        host = np.zeros(words, dtype=np.uint64)
        assert lib.mjx_mt_jump_table(n, k, G, host.ctypes.data) == 0
        table = torch.from_numpy(host.view(np.int64)).cuda()
    mask = torch.empty((k, n), dtype=torch.uint8, device="cuda")
    th = torch.tensor(thr, dtype=torch.float64, device="cuda")
    mt_out, ln_out = torch.empty_like(st._mt), torch.empty_like(st._ln)
    assert lib.mjx_hpr_refresh_masks_jump(st._mt.data_ptr(), st._ln.data_ptr(), mt_out.data_ptr(), ln_out.data_ptr(),
                                          n, k, G, table.data_ptr() if table is not None else None, th.data_ptr(),
                                          mask.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    want = torch.stack([torch.rand(n, dtype=torch.float64, generator=h) < thr[j] for j in range(k)])
    assert torch.equal(mask.cpu().bool(), want)
    st._mt.copy_(mt_out)
    st._ln.copy_(ln_out)
    g2 = torch.Generator()
    g2.set_state(st.rng_state_bytes())
    assert torch.equal(torch.rand(9, dtype=torch.float64, generator=g2), torch.rand(9, dtype=torch.float64, generator=h))


def test_hpr_run_device_rng_equals_host_rng(mjx_mod):
    """hpr_run with the stream continued on the device and with host draws:
    same stop iteration, configuration and generator position afterwards."""
    n, d, p, c = 300, 4, 2, 2
    edges = mjx_mod.random_regular_edges(d, n, seed=6)
    out = []
    for rng in ("device", "host"):
        g = torch.Generator().manual_seed(11)
        res = mjx_mod.hpr_run(d, n, p, c, TT=100, edges=edges, dtype=torch.float64, generator=g, rng=rng, batch=8)
        out.append((res, torch.rand(5, dtype=torch.float64, generator=g)))
    assert out[0][0]["num_steps"][0] == out[1][0]["num_steps"][0]
    assert np.array_equal(out[0][0]["conf"], out[1][0]["conf"])
    assert torch.equal(out[0][1], out[1][1])


def test_hpr_run_initial_state_from_the_cuda_generator(mjx_mod):
    """The reference draws chi0 and the biases with device=device
    (code/HPR_pytorch_RRG.py:102,334): on a GPU box torch's CUDA generator,
    chi0 first.  hpr_run(init_generator=cuda generator) makes those draws in
    that order: same run as the explicitly drawn initial state, and the CUDA
    generator left at the same offset."""
    n, d, p, c = 200, 4, 1, 1
    edges = mjx_mod.random_regular_edges(d, n, seed=3)
    E = n * d // 2
    gi = torch.Generator("cuda").manual_seed(21)
    res = mjx_mod.hpr_run(d, n, p, c, TT=60, edges=edges, dtype=torch.float64,
                          generator=torch.Generator().manual_seed(4), init_generator=gi)
    gj = torch.Generator("cuda").manual_seed(21)
    chi = torch.rand((2 * E, 4 ** (p + c)), dtype=torch.float64, device="cuda", generator=gj)
    chi = chi / torch.sum(chi, axis=1, keepdims=True)
    b = torch.rand((n, 2), dtype=torch.float64, device="cuda", generator=gj)
    b = b / torch.sum(b, axis=1, keepdims=True)
    ref = mjx_mod.hpr_run(d, n, p, c, TT=60, edges=edges, dtype=torch.float64,
                          generator=torch.Generator().manual_seed(4), chi0=chi, biases0=b)
    assert res["num_steps"][0] == ref["num_steps"][0]
    assert np.array_equal(res["conf"], ref["conf"])
    assert torch.equal(torch.rand(7, device="cuda", generator=gi), torch.rand(7, device="cuda", generator=gj))
