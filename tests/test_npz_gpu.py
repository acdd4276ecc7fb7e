"""End-to-end result files: a run on the device written
by the package's npz writers equals, in keys, dtypes, shapes and values, the
file the reference writes (code/HPR_pytorch_RRG.py:377; the notebook's
np.savez of nb:515).  The SA file is covered by
tests/test_sa_gpu.py::test_sa_run_global_stream_two_replicas_to_npz."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_hpr_run_to_npz_equals_reference_file(mjx_mod, tmp_path):
    full = load_golden("hpr_fullscript.npz")
    key = "n40_d4_p1c1"
    n, d, p, c, TT, tseed = (int(x) for x in full[f"{key}_params"])
    ref = {k: full[f"{key}_{k}"] for k in ("mag_reached", "conf", "num_steps", "graphs")}
    res = mjx_mod.hpr_run(d, n, p, c, TT=TT, edges=full[f"{key}_edges"], nbrs=ref["graphs"][0].astype(np.int64),
                          seed=tseed, dtype=torch.float64)
    path = tmp_path / "hpr_d4_p1.npz"
    mjx_mod.save_hpr_npz(path, res, time=2.5)
    with np.load(path) as z:
        assert sorted(z.files) == sorted(list(ref) + ["time"])
        for k in ref:
            assert z[k].dtype == ref[k].dtype and z[k].shape == ref[k].shape, k
            assert np.array_equal(z[k], ref[k]), k
        assert z["time"].dtype == np.float64 and float(z["time"]) == 2.5


def test_bdcm_er_run_to_npz_has_the_notebook_layout(mjx_mod, tmp_path):
    """bdcm_er_run -> save_bdcm_npz: the keys of nb:515's np.savez, with the
    shapes and dtypes the notebook's own arrays have (nb:456-492: float64
    (deg, num_rep, lambdas) curves, float64 (deg, num_rep) graph statistics,
    deg/prob float64 vectors, T_max/num_rep Python ints), values as returned;
    the lambda = 0 point of every curve is a physical m_init in (0, 1] with
    ent1 = phi + 0 * m_init = ent at lambda = 0 (nb:436-437)."""
    deg, num_rep, a, dl, T_max = (1.0, 2.0), 2, 0.3, 0.1, 60
    res = mjx_mod.bdcm_er_run(n=300, deg=deg, num_rep=num_rep, a=a, dl=dl, T_max=T_max, seed=3)
    path = tmp_path / "ER_p1.npz"
    mjx_mod.save_bdcm_npz(path, res)
    nl = int(a / dl + 1)
    want_shape = {"m_init": (2, num_rep, nl), "ent1": (2, num_rep, nl), "ent": (2, num_rep, nl),
                  "nodes_numbers": (2, num_rep), "mean_degrees": (2, num_rep), "max_degrees": (2, num_rep),
                  "nodes_isolated": (2, num_rep), "mean_degrees_total": (2, num_rep), "deg": (2,), "prob": (2,),
                  "T_max": (), "num_rep": ()}
    with np.load(path) as z:
        assert sorted(z.files) == sorted(want_shape)
        for k, shp in want_shape.items():
            assert z[k].shape == shp, k
            want_dtype = np.asarray(T_max).dtype if k in ("T_max", "num_rep") else np.float64
            assert z[k].dtype == want_dtype, k
            assert np.array_equal(z[k], np.asarray(res[k])), k
        m0 = z["m_init"][:, :, 0]
        assert np.all((m0 > 0) & (m0 <= 1))
        np.testing.assert_allclose(z["ent1"][:, :, 0], z["ent"][:, :, 0], rtol=0, atol=1e-12)
        assert np.array_equal(z["prob"], np.asarray(deg) / 299)


def test_graphs_from_result_file_run_the_dynamics(mjx_mod, tmp_path):
    """A graph read back from a reference result file drives the device
    dynamics exactly like the neighbour array the script used."""
    from oracle import majority as orc
    full = load_golden("sa_fullscript.npz")
    adj = full["n200_d4_p3_graphs"]
    path = tmp_path / "g.npz"
    np.savez(path, graphs=adj)
    graphs = mjx_mod.graphs_from_npz(path)
    s0 = 2 * np.random.default_rng(3).integers(0, 2, (8, adj.shape[1])).astype(np.int64) - 1
    for g, a in zip(graphs, adj):
        got = mjx_mod.s_endstate(g, s0, 3, 1)
        assert np.array_equal(got, orc.s_endstate_batch(a.astype(np.int64), s0, 3, 1))
