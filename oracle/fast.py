"""ORACLE (test infrastructure only): ctypes front of the C restatement
(oracle/orc_majority.c) with the numpy oracle's signatures and return
values, for checks at the BASELINE configs' sizes.

  s_endstate(N, s0, p, c)               code/SA_RRG.py:23-26
  s_endstate_er(row_ptr, col, s0, p, c) code/ER_BDCM_entropy.ipynb raw lines 120-123
  sa_loop(N, p, c, seed, ...)           code/SA_RRG.py:63-88 (same dict as
                                        oracle.majority.sa_loop)
  sa_loop_philox(N, p, c, seed, ...)    the same loop on the library's non-parity
                                        Philox-4x32-10 proposal stream
  philox4x32_10(ctr, key)               Random123's philox4x32_10 block
"""
import ctypes
import os

import numpy as np

from . import build_oracle

_LIB = None
_P = ctypes.c_void_p
_I64 = ctypes.c_int64


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(build_oracle.LIB):
            build_oracle.build(verbose=False)
        lib = ctypes.CDLL(build_oracle.LIB)
        lib.orc_s_endstate_ell.argtypes = [_P, _I64, ctypes.c_int, _P, ctypes.c_int, _P, _P]
        lib.orc_s_endstate_ell.restype = _I64
        lib.orc_s_endstate_csr.argtypes = [_P, _P, _I64, _P, ctypes.c_int, _P, _P]
        lib.orc_s_endstate_csr.restype = _I64
        lib.orc_sa_loop.argtypes = [_P, _I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                    ctypes.c_double, ctypes.c_double, _I64, _P, _P, _P, _P, _P, _P, _P, _P]
        lib.orc_sa_loop.restype = _I64
        lib.orc_sa_loop_philox.argtypes = [_P, _I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                           ctypes.c_uint64, ctypes.c_double, ctypes.c_double, _I64, _P, _P, _P, _P,
                                           _P, _P]
        lib.orc_sa_loop_philox.restype = _I64
        lib.orc_philox4x32_10.argtypes = [_P, _P, _P]
        _LIB = lib
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _spins(s0):
    return np.ascontiguousarray(np.asarray(s0), dtype=np.int8)


def s_endstate(N, s0, p, c):
    N = np.ascontiguousarray(N, dtype=np.int32)
    n, d = N.shape
    s = _spins(s0)
    out, tmp = np.empty(n, np.int8), np.empty(n, np.int8)
    _lib().orc_s_endstate_ell(_ptr(N), n, d, _ptr(s), int(p) + int(c) - 1, _ptr(out), _ptr(tmp))
    return out.astype(np.int64)


def s_endstate_er(row_ptr, col, s0, p, c):
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    n = rp.shape[0] - 1
    s = _spins(s0)
    out, tmp = np.empty(n, np.int8), np.empty(n, np.int8)
    _lib().orc_s_endstate_csr(_ptr(rp), _ptr(cl), n, _ptr(s), int(p) + int(c) - 1, _ptr(out), _ptr(tmp))
    return out.astype(np.int64)


def sa_loop(N, p, c, seed, par_a=1.0005, par_b=1.0005, max_steps=None, trace=False, mt_state=None):
    """``mt_state`` = (mt uint32 (624,), idx): continue that stream instead of
    seeding; the returned dict then holds the stream's final "mt_state"."""
    N = np.ascontiguousarray(N, dtype=np.int32)
    n, d = N.shape
    if max_steps is None and trace:
        raise ValueError("trace needs max_steps (the trace buffers are preallocated)")
    cap = -1 if max_steps is None else int(max_steps)
    L = max(cap, 1)
    tr = None
    if trace:
        tr = {"i": np.zeros(L, np.int32), "accept": np.zeros(L, np.int8), "sum_end": np.zeros(L, np.int64),
              "dE": np.zeros(L, np.float64)}
    conf = np.empty(n, np.int8)
    done = ctypes.c_int32(0)
    mt = idx = None
    if mt_state is not None:
        mt = np.ascontiguousarray(np.asarray(mt_state[0], dtype=np.uint32).reshape(624)).copy()
        idx = ctypes.c_int32(int(mt_state[1]))
    t = _lib().orc_sa_loop(_ptr(N), n, d, int(p), int(c), int(seed) & 0xFFFFFFFF, float(par_a), float(par_b), cap,
                           _ptr(tr["i"]) if tr else None, _ptr(tr["accept"]) if tr else None,
                           _ptr(tr["sum_end"]) if tr else None, _ptr(tr["dE"]) if tr else None, _ptr(conf),
                           ctypes.byref(done), _ptr(mt) if mt is not None else None,
                           ctypes.byref(idx) if idx is not None else None)
    conf = conf.astype(np.int64)
    out = {"conf": conf, "num_steps": int(t), "mag_reached": np.sum(conf) / n, "done": int(done.value)}
    if mt is not None:
        out["mt_state"] = (mt, int(idx.value))
    if trace:
        out["trace"] = {"i": tr["i"][:t].astype(np.int64), "accept": tr["accept"][:t],
                        "sum_end": tr["sum_end"][:t], "dE": tr["dE"][:t]}
    return out


def philox4x32_10(ctr, key):
    """Random123's philox4x32_10 of counter (4 uint32) and key (2 uint32)."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    _lib().orc_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def sa_loop_philox(N, p, c, seed, par_a=1.0005, par_b=1.0005, max_steps=None, trace=False, key=None):
    """sa_loop with proposal t drawn from Philox-4x32-10 (key = the seed unless
    given): the initial configuration from np.random.seed(seed) as in sa_loop."""
    N = np.ascontiguousarray(N, dtype=np.int32)
    n, d = N.shape
    if max_steps is None and trace:
        raise ValueError("trace needs max_steps (the trace buffers are preallocated)")
    cap = -1 if max_steps is None else int(max_steps)
    L = max(cap, 1)
    tr = None
    if trace:
        tr = {"i": np.zeros(L, np.int32), "accept": np.zeros(L, np.int8), "sum_end": np.zeros(L, np.int64),
              "dE": np.zeros(L, np.float64)}
    conf = np.empty(n, np.int8)
    done = ctypes.c_int32(0)
    k = int(seed) if key is None else int(key)
    t = _lib().orc_sa_loop_philox(_ptr(N), n, d, int(p), int(c), int(seed) & 0xFFFFFFFF, k & 0xFFFFFFFFFFFFFFFF,
                                  float(par_a), float(par_b), cap, _ptr(tr["i"]) if tr else None,
                                  _ptr(tr["accept"]) if tr else None, _ptr(tr["sum_end"]) if tr else None,
                                  _ptr(tr["dE"]) if tr else None, _ptr(conf), ctypes.byref(done))
    conf = conf.astype(np.int64)
    out = {"conf": conf, "num_steps": int(t), "mag_reached": np.sum(conf) / n, "done": int(done.value)}
    if trace:
        out["trace"] = {"i": tr["i"][:t].astype(np.int64), "accept": tr["accept"][:t],
                        "sum_end": tr["sum_end"][:t], "dE": tr["dE"][:t]}
    return out
