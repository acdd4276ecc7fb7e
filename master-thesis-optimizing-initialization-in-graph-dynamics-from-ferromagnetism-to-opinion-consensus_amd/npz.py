"""Result files with the reference's keys and dtypes.

  save_sa_npz    code/SA_RRG.py:53-56,86-92  mag_reached, num_steps, conf (float64), graphs (int)
  save_hpr_npz   code/HPR_pytorch_RRG.py:252-255,359-377  mag_reached, conf, num_steps, graphs (float64), time
  save_bdcm_npz  nb:485-515 (the cell's commented np.savez)  m_init, ent1, ent, nodes_numbers, ...
  neighbour_arrays / graphs_from_npz   the `graphs` key of those files back as (n, d)
                 neighbour arrays (the reference's N / N_nodes, SA_RRG.py:9-16,
                 HPR_pytorch_RRG.py:110-118) and device graphs

These are host-side format writers (numpy), not compute.
"""
import numpy as np

SA_KEYS = ("mag_reached", "num_steps", "conf", "graphs")
HPR_KEYS = ("mag_reached", "conf", "num_steps", "graphs", "time")
BDCM_KEYS = ("m_init", "ent1", "ent", "nodes_numbers", "mean_degrees", "max_degrees", "deg", "prob",
             "mean_degrees_total", "nodes_isolated", "T_max", "num_rep")


def sa_arrays(res):
    """The arrays SA_RRG.py saves: zeros-initialised float64 buffers filled per
    replica (:53-56, 86-88) and graphs.astype(int) (:90)."""
    return {
        "mag_reached": np.asarray(res["mag_reached"], dtype=np.float64),
        "num_steps": np.asarray(res["num_steps"], dtype=np.float64),
        "conf": np.asarray(res["conf"], dtype=np.float64),
        "graphs": np.asarray(res["graphs"]).astype(int),
    }


def save_sa_npz(path, res):
    np.savez(path, **sa_arrays(res))


def hpr_arrays(res, time=None):
    """HPR_pytorch_RRG.py's arrays: float64 torch buffers moved to numpy (:252-255, 366-375)."""
    out = {k: np.asarray(res[k], dtype=np.float64) for k in ("mag_reached", "conf", "num_steps", "graphs")}
    out["time"] = np.float64(0.0 if time is None else time)
    return out


def save_hpr_npz(path, res, time=None):
    np.savez(path, **hpr_arrays(res, time))


def save_bdcm_npz(path, res):
    """bdcm_er_run's dict with the notebook's keys (nb:515)."""
    np.savez(path, **{k: np.asarray(res[k]) for k in BDCM_KEYS})


def neighbour_arrays(src):
    """The (n, d) int32 neighbour arrays stored under `graphs` in a result file
    (a path or a loaded mapping): SA_RRG.py saves them as int (n_stat, n, d)
    (:90), HPR_pytorch_RRG.py as float64 (:255, 362).  Rows must hold integral
    node ids in [0, n)."""
    if isinstance(src, (str, bytes)) or hasattr(src, "__fspath__"):
        with np.load(src, allow_pickle=False) as z:
            g = np.asarray(z["graphs"])
    else:
        g = np.asarray(src["graphs"])
    if g.ndim == 2:
        g = g[None]
    if g.ndim != 3:
        raise ValueError(f"graphs must be (n_rep, n, d), got {g.shape}")
    out = []
    for a in g:
        ai = a.astype(np.int64)
        if not np.array_equal(ai, a) or ai.min() < 0 or ai.max() >= a.shape[0]:
            raise ValueError("graphs rows must hold node ids in [0, n)")
        out.append(ai.astype(np.int32))
    return out


def graphs_from_npz(src):
    """Device ELL graphs (mjx.Graph) of every replica's graph in a result file."""
    from .graph import Graph
    return [Graph.ell(a) for a in neighbour_arrays(src)]
