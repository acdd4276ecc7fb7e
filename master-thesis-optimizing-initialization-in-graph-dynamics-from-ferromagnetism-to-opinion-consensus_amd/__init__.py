"""mjx — MI355X-native engine for majority-rule (zero-temperature Ising,
always-stay) dynamics on random regular and Erdos-Renyi graphs, the
data-parallel hot path of the thesis code.

Every compute entry point calls hand-written HIP kernels (libmjx.so, gfx950)
through the C ABI in include/mjx.h.  There is no CPU fallback.
"""
from . import _lib
from ._lib import MjxError, lib_path
from .graph import (Graph, neighbours, csr_from_networkx, random_regular_graph, random_regular_edges,
                    erdos_renyi, erdos_renyi_edges, csr_from_edges, remove_isolated,
                    random_regular_rows_device, random_regular_graph_device, erdos_renyi_device, check_ell)
from .partition import BinnedPlan, NodeRange, ShardedRRG, pack_host, unpack_host
from .npz import (save_sa_npz, save_hpr_npz, save_bdcm_npz, sa_arrays, hpr_arrays, neighbour_arrays,
                  graphs_from_npz)
from .dynamics import onestep_majority, s_endstate, m, pack, unpack, rollout, popcount, as_graph
from .sa import SAReplicas, E_delta, sa_run, schedule_constants
from .hpr import HPRPlan, HPRState, HPr_dp, marginals_comp, new_biases_i, hpr_run
from .hpr_er import HPRERPlan, HPr_dp_er, marginals_comp_er, hpr_er_plan, hpr_er_run
from .bdcm import (BDCMPlan, bdcm_er_plan, BDCM_ER, bdcm_leaf_reset, Zij, Zi_ER, phi_BP_GENERAL_ER,
                   avg_m_init_GENERAL_ER, BDCM_entropy_procedure_GENERAL_ER, bdcm_er_run)
from .bdcm import converge as bdcm_converge
from . import drop_in  # reference-signature HPR drop-ins (code/HPR_pytorch_RRG.py)

__all__ = [
    "MjxError", "lib_path", "BinnedPlan", "neighbour_arrays", "graphs_from_npz", "Graph", "neighbours", "csr_from_networkx", "random_regular_graph",
    "random_regular_edges", "erdos_renyi", "erdos_renyi_device", "erdos_renyi_edges", "csr_from_edges", "remove_isolated",
    "onestep_majority", "s_endstate", "m", "pack", "unpack", "rollout", "popcount", "as_graph",
    "SAReplicas", "E_delta", "sa_run", "schedule_constants",
    "HPRPlan", "HPRState", "HPr_dp", "marginals_comp", "new_biases_i", "hpr_run",
    "HPRERPlan", "HPr_dp_er", "marginals_comp_er", "hpr_er_plan", "hpr_er_run",
    "BDCMPlan", "bdcm_er_plan", "BDCM_ER", "bdcm_converge", "bdcm_leaf_reset", "Zij", "Zi_ER", "phi_BP_GENERAL_ER",
    "avg_m_init_GENERAL_ER", "BDCM_entropy_procedure_GENERAL_ER", "bdcm_er_run", "drop_in",
]


def load_library():
    """Load libmjx.so (raises MjxError if it has not been built)."""
    return _lib.load()
