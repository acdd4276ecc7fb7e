"""ctypes binding of libmjx.so — the C ABI declared in include/mjx.h.

This is exactly the binding a maintainer of the reference would add
(INTEGRATION.md): plain pointers, sizes and a hipStream_t.  There is no CPU
fallback: if the library or a GPU is missing every compute entry point raises.
"""
import ctypes
import os

from . import _build

_LIB = None

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
c_vp = ctypes.c_void_p
c_u64 = ctypes.c_uint64

# name -> argtypes (restype is c_int unless listed in _RESTYPES)
SIGNATURES = {
    "mjx_abi_version": [],
    "mjx_build_id": [],
    "mjx_strerror": [c_int],
    "mjx_last_hip_error": [],
    "mjx_pack_np": [c_vp, c_int, c_i64, c_vp, c_vp],
    "mjx_unpack_np": [c_vp, c_i64, c_vp, c_int, c_vp],
    "mjx_pack_rp": [c_vp, c_int, c_i64, c_i64, c_vp, c_vp],
    "mjx_unpack_rp": [c_vp, c_i64, c_i64, c_vp, c_int, c_vp],
    "mjx_rollout_ell_np": [c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_rollout_ell_rp": [c_vp, c_i64, c_int, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_rollout_ell_rp_multi": [c_vp, c_i64, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_rollout_ell_rp_sliced": [c_vp, c_i64, c_int, c_i64, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp],
    "mjx_rollout_csr_rp_ordered": [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_rollout_csr_np": [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_rollout_csr_rp": [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_class_ell_fill": [c_vp, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp],
    "mjx_rollout_class_rp": [c_vp, c_vp, c_vp, c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    "mjx_gather_floor_class": [c_vp, c_vp, c_vp, c_int, c_i64, c_i64, c_vp, c_vp, c_vp],
    "mjx_popcount_np": [c_vp, c_i64, c_vp, c_vp],
    "mjx_popcount_rp": [c_vp, c_i64, c_i64, c_vp, c_vp],
    "mjx_sa_init": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_dbl, c_dbl,
                    c_vp, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_init_mt": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_dbl, c_dbl,
                       c_vp, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_steps": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp,
                     c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_i64, c_vp],
    "mjx_sa_lightcone_lds": [c_int, c_int, c_int],
    "mjx_sa_lightcone_prepare": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_lightcone_steps": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp,
                               c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_i64, c_vp],
    "mjx_sa_lds_bytes": [c_i64, c_int, c_int, c_int],
    "mjx_sa_lds_plan": [c_i64, c_int, c_int, c_int, ctypes.c_uint32, c_int, c_vp],
    "mjx_selftest_devmemo": [],
    "mjx_sa_lds_steps": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_i64, c_dbl, c_dbl, c_dbl, c_dbl,
                         c_i64, c_vp],
    "mjx_sa_cone_words": [c_int, c_int],
    "mjx_sa_cone_pack": [c_i64, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_cone_unpack": [c_i64, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_cone_steps": [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp,
                          c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_i64, c_vp],
    "mjx_sa_rec_words": [c_int, c_int, c_int],
    "mjx_sa_state_bytes": [],
    "mjx_sa_rec_pack": [c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_rec_unpack": [c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp],
    "mjx_sa_rec_steps": [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp,
                         c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_i64, c_vp],
    "mjx_hpr_update": [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int,
                       c_dbl, c_dbl, c_dbl, c_vp],
    "mjx_hpr_marginals": [c_int, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_dbl, c_vp, c_vp, c_vp],
    "mjx_hpr_new_biases": [c_int, c_vp, c_vp, c_vp, c_dbl, c_dbl, c_i64, c_vp, c_vp],
    "mjx_hpr_new_biases_mask": [c_int, c_vp, c_vp, c_vp, c_dbl, c_i64, c_vp, c_vp],
    "mjx_hpr_node_step": [c_int, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_dbl, c_vp, c_vp, c_vp],
    "mjx_hpr_refresh_masks": [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp],
    "mjx_mt_jump_geometry": [c_i64, c_int, c_int, c_vp, c_vp],
    "mjx_mt_jump_table_words": [c_i64, c_int, c_int],
    "mjx_mt_jump_table": [c_i64, c_int, c_int, c_vp],
    "mjx_hpr_refresh_masks_jump": [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp],
    "mjx_hpr_edge_z": [c_int, c_vp, c_i64, c_int, c_int, c_dbl, c_vp, c_vp],
    "mjx_hpr_node_biases": [c_int, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp],
    "mjx_hpr_q_supported": [c_int, c_int, c_int, c_int],
    "mjx_hpr_qlayout": [c_int, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int, c_dbl, c_vp],
    "mjx_hpr_update_q": [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int,
                         c_dbl, c_dbl, c_dbl, c_vp, c_vp],
    "mjx_hpr_marginals_q": [c_int, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp],
    "mjx_hpr_q_ii": [c_int, c_vp, c_i64, c_int, c_int, c_vp, c_vp],
    "mjx_hpr_er_scratch_bytes": [c_int, c_int, c_int, c_int],
    "mjx_hpr_er_update_class": [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int,
                                c_dbl, c_dbl, c_dbl, c_vp, c_i64, c_vp],
    "mjx_hpr_node_marg_csr": [c_int, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp],
    "mjx_sweep_ell_np_range": [c_vp, c_i64, c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp],
    "mjx_rrg_generate": [c_i64, c_int, c_u64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp],
    "mjx_rrg_partner_host": [c_i64, c_int, c_u64, c_i64],
    "mjx_graph_check_ell": [c_vp, c_i64, c_int, c_vp, c_vp],
    "mjx_er_work_bytes": [c_i64],
    "mjx_er_generate": [c_i64, c_dbl, c_u64, c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp],
    "mjx_binned_plan_shape": [c_i64, c_int, c_i64, c_i64, c_vp],
    "mjx_binned_build": [c_vp, c_i64, c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    "mjx_sweep_binned": [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_vp],
    "mjx_bdcm_lds_bytes": [c_int, c_int, c_int],
    "mjx_bdcm_scratch_bytes": [c_int, c_int, c_int],
    "mjx_bdcm_update_class": [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_vp,
                              c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    "mjx_bdcm_iter_begin": [c_vp, c_vp],
    "mjx_bdcm_iter_end": [c_vp, c_dbl, c_i64, c_vp],
    "mjx_bdcm_node_z": [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int, c_dbl, c_dbl, c_vp, c_vp, c_i64,
                        c_vp],
    "mjx_bdcm_edge_obs": [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_dbl, c_vp, c_vp, c_vp],
    "mjx_sum_f64": [c_vp, c_i64, c_int, c_vp, c_vp, c_vp],
}
_RESTYPES = {"mjx_strerror": ctypes.c_char_p, "mjx_build_id": ctypes.c_char_p, "mjx_last_hip_error": ctypes.c_char_p,
             "mjx_sa_lightcone_lds": c_i64, "mjx_sa_lds_bytes": c_i64, "mjx_sa_lds_plan": c_i64, "mjx_bdcm_lds_bytes": c_i64, "mjx_bdcm_scratch_bytes": c_i64,
             "mjx_rrg_partner_host": c_i64, "mjx_er_work_bytes": c_i64, "mjx_hpr_er_scratch_bytes": c_i64,
             "mjx_mt_jump_table_words": c_i64}

MJX_OK, MJX_EINVAL, MJX_EHIP, MJX_ERANGE = 0, 1, 2, 3      # status codes (include/mjx.h)
MJX_I8, MJX_I32, MJX_I64 = 1, 4, 8
MJX_F32, MJX_F64 = 104, 108


class MjxSaState(ctypes.Structure):
    """Mirror of ``mjx_sa_state`` in include/mjx.h (field order matters)."""
    _fields_ = [
        ("mt", c_vp), ("mt_idx", c_vp), ("a", c_vp), ("b", c_vp), ("t", c_vp),
        ("sum_end", c_vp), ("done", c_vp), ("prop_i", c_vp), ("prop_s", c_vp),
        ("prop_u", c_vp), ("cnt", c_vp),
        ("tr_i", c_vp), ("tr_acc", c_vp), ("tr_sum", c_vp), ("tr_dE", c_vp), ("tr_tie", c_vp),
        ("tape_i", c_vp), ("tape_u", c_vp), ("tape_cap", c_i64),
        ("rep_graph", c_vp), ("opt_split", ctypes.c_int32), ("opt_spec_k", ctypes.c_int32),
        ("opt_flags", ctypes.c_uint32), ("philox_key", c_vp), ("rec_nb", ctypes.c_int32),
    ]


MJX_SA_NO_SPEC, MJX_SA_NO_CONE2, MJX_SA_LDS_SERIAL, MJX_SA_LDS_SINGLE, MJX_SA_LDS_PAIR = 1, 2, 4, 8, 16  # opt_flags (include/mjx.h)
MJX_SA_LDS_WAVE = 32
MJX_SA_LDS_CU = 64


class MjxError(RuntimeError):
    pass


def lib_path():
    return _build.LIB


def verify_build_id(lib, csrc=None, include=None):
    """Raise MjxError unless the library's mjx_build_id() is the content hash
    of the source tree (default: the csrc/ and include/ next to this file)."""
    got = lib.mjx_build_id().decode()
    want = _build.source_hash(csrc or _build.CSRC, include or _build.INCLUDE)
    if got != want:
        raise MjxError(f"libmjx.so was built from other sources (build id {got}, source tree {want}): "
                       "rebuild it with __graft_entry__.build()")


def open_library(path, verify=True):
    """dlopen a build of libmjx.so and declare every entry point; with
    ``verify`` the build id must match the source tree (verify_build_id).
    Unverified (an A/B build of older sources, tools/ab_lib.py) an entry point
    the build lacks is left undeclared."""
    lib = ctypes.CDLL(path)
    for name, argtypes in SIGNATURES.items():
        if not verify and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, c_int)
    if verify:
        verify_build_id(lib)
    return lib


def load(build_if_missing=False):
    """Load the in-tree libmjx.so (its build id checked against the sources)
    and declare every entry point.  Raises if it is absent or stale."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = _build.LIB
    if not os.path.exists(path):
        if build_if_missing:
            _build.build()
        else:
            raise MjxError(f"libmjx.so not found at {path}: run __graft_entry__.build() "
                           "(there is no CPU fallback for the majority-dynamics kernels)")
    _LIB = open_library(path)
    return _LIB


def check(rc, what):
    if rc != 0:
        lib = load()
        msg = lib.mjx_strerror(rc).decode()
        hip = lib.mjx_last_hip_error().decode()
        raise MjxError(f"{what} failed: {msg} (status {rc}){'; ' + hip if hip else ''}")


def call(name, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)
