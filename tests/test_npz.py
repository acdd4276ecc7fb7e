"""Result files keep the reference's keys and dtypes,
checked against the files the reference scripts themselves wrote
(tests/golden/sa_fullscript.npz, hpr_fullscript.npz hold their np.savez output)."""
import numpy as np

from conftest import load_golden


def _ref_arrays(full, key):
    pre = key + "_"
    names = ("mag_reached", "num_steps", "conf", "graphs")
    return {k[len(pre):]: v for k, v in full.items() if k.startswith(pre) and k[len(pre):] in names}


def test_sa_npz_matches_reference_file(mjx_mod, tmp_path):
    full = load_golden("sa_fullscript.npz")
    ref = _ref_arrays(full, "n200_d4_p3")
    res = {"mag_reached": ref["mag_reached"], "num_steps": ref["num_steps"],
           "conf": ref["conf"].astype(np.int64), "graphs": ref["graphs"].astype(np.int32)}
    path = tmp_path / "sa.npz"
    mjx_mod.save_sa_npz(path, res)
    with np.load(path) as z:
        assert sorted(z.files) == sorted(ref)
        for k in ref:
            assert z[k].dtype == ref[k].dtype, k
            assert np.array_equal(z[k], ref[k]), k


def test_hpr_npz_matches_reference_file(mjx_mod, tmp_path):
    full = load_golden("hpr_fullscript.npz")
    ref = _ref_arrays(full, "n40_d4_p1c1")
    res = {"mag_reached": ref["mag_reached"], "num_steps": ref["num_steps"], "conf": ref["conf"].astype(np.int32),
           "graphs": ref["graphs"]}
    path = tmp_path / "hpr.npz"
    mjx_mod.save_hpr_npz(path, res, time=1.5)
    with np.load(path) as z:
        assert sorted(z.files) == sorted(list(ref) + ["time"])
        for k in ref:
            assert z[k].dtype == ref[k].dtype, k
            assert np.array_equal(z[k], ref[k]), k
        assert float(z["time"]) == 1.5


def test_graphs_round_trip_through_result_files(mjx_mod, tmp_path):
    """The `graphs` of the reference's own result files (int from SA_RRG.py,
    float64 from HPR_pytorch_RRG.py) come back as (n, d) int32 neighbour
    arrays equal to the arrays the scripts used, and survive a write."""
    for name, key in (("sa_fullscript.npz", "n200_d4_p3"), ("hpr_fullscript.npz", "n40_d4_p1c1")):
        ref = _ref_arrays(load_golden(name), key)
        got = mjx_mod.neighbour_arrays({"graphs": ref["graphs"]})
        assert len(got) == ref["graphs"].shape[0]
        for a, b in zip(got, ref["graphs"]):
            assert a.dtype == np.int32 and np.array_equal(a, b)
        path = tmp_path / f"{key}.npz"
        np.savez(path, graphs=ref["graphs"])
        again = mjx_mod.neighbour_arrays(path)
        assert all(np.array_equal(a, b) for a, b in zip(again, got))
    bad = {"graphs": np.array([[[0.5, 1.0]]])}
    try:
        mjx_mod.neighbour_arrays(bad)
    except ValueError:
        pass
    else:
        raise AssertionError("non-integral node ids accepted")
