"""python -m mjx sa|hpr|bdcm on the device: each front writes the reference's
np.savez keys (code/SA_RRG.py:92, code/HPR_pytorch_RRG.py:377,
code/ER_BDCM_entropy.ipynb nb:515), and the SA front's file equals sa_run's
result (the global-stream run pinned to the C oracle by
tests/test_sa_multi_gpu.py::test_sa_run_global_stream_to_consensus)."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_sa_front_writes_the_script_file(mjx_mod, tmp_path):
    cli = importlib.import_module("mjx.cli")
    out = tmp_path / "MCMC_p3_d4.npz"
    cli.main(["sa", "--n", "1000", "--N_stat", "2", "--seed", "5", "--graph-seed", "70", "--out", str(out)])
    ref = mjx_mod.sa_run(4, 1000, 3, 1, N_stat=2, seed=5, graph_seed=70, stream="global")
    with np.load(out, allow_pickle=False) as z:
        assert sorted(z.files) == ["conf", "graphs", "mag_reached", "num_steps"]
        assert z["graphs"].shape == (2, 1000, 4) and z["conf"].shape == (2, 1000)
        for k in ("mag_reached", "num_steps", "conf", "graphs"):
            assert np.array_equal(z[k], np.asarray(ref[k]).astype(z[k].dtype)), k
    assert np.all(ref["done"] == 1)


def test_sa_front_independent_streams(mjx_mod, tmp_path):
    cli = importlib.import_module("mjx.cli")
    out = tmp_path / "sa_ind.npz"
    cli.main(["sa", "--n", "500", "--p", "1", "--N_stat", "3", "--stream", "independent", "--max-steps", "400",
              "--out", str(out)])
    ref = mjx_mod.sa_run(4, 500, 1, 1, N_stat=3, seed=0, graph_seed=0, stream="independent", max_steps=400)
    with np.load(out, allow_pickle=False) as z:
        for k in ("mag_reached", "num_steps", "conf"):
            assert np.array_equal(z[k], ref[k]), k


def test_hpr_and_bdcm_fronts_write_the_reference_keys(mjx_mod, tmp_path):
    cli = importlib.import_module("mjx.cli")
    out = tmp_path / "hpr.npz"
    cli.main(["hpr", "--n", "60", "--d", "3", "--TT", "40", "--out", str(out)])
    with np.load(out, allow_pickle=False) as z:
        assert sorted(z.files) == ["conf", "graphs", "mag_reached", "num_steps", "time"]
        assert z["conf"].shape == (1, 60) and z["graphs"].shape == (1, 60, 3)
    out = tmp_path / "ER_p1.npz"
    cli.main(["bdcm", "--n", "200", "--deg", "1.5", "--num_rep", "1", "--a", "0.2", "--out", str(out)])
    with np.load(out, allow_pickle=False) as z:
        assert {"m_init", "ent1", "ent", "deg", "prob", "T_max", "num_rep"} <= set(z.files)
        assert z["m_init"].shape == (1, 1, 3)
