"""ORACLE (test infrastructure only): torch-CPU restatement of HPr_dp
(code/HPR_pytorch_RRG.py:183-218) — the same vectorised DP as oracle/hpr.py,
written with torch ops so that the bench's CPU baseline runs it the way the
reference runs, on torch's CPU backend with every host core
(torch.set_num_threads), float64 (the reference's default dtype, :11).
Used only by bench.py's cpu_baseline leg; checked against oracle/hpr.py in
tests/test_hpr_oracle.py."""
import itertools

import numpy as np
import torch

from .hpr import A_factor, traj_table

_A_CACHE = {}


def HPr_dp(chi, biases, in_rows, src, n, d, p, c, attr_value, lmbd_in, damppar, rows):
    """Rows ``rows`` of one HPR message update; chi (2E, 4^T), biases (n, 2)
    float64 torch CPU tensors; in_rows (2E, d-1), src (2E,) numpy."""
    T = p + c
    X = 2 ** T
    rows = torch.as_tensor(np.asarray(rows), dtype=torch.int64)
    tr = traj_table(T)
    plus0 = torch.from_numpy(tr[:, 0] == 1)
    inr = torch.as_tensor(np.asarray(in_rows), dtype=torch.int64)[rows]           # (R, d-1)
    srct = torch.as_tensor(np.asarray(src), dtype=torch.int64)
    cm = chi.view(-1, X, X)
    M = cm[inr]                                                                     # (R, d-1, X, X)
    bsrc = biases[srct[inr]]                                                        # (R, d-1, 2)
    bs = torch.where(plus0[None, None, :], bsrc[..., 0:1], bsrc[..., 1:2])          # (R, d-1, X)
    M = M * bs[..., None]
    nb = d ** T
    digits = torch.from_numpy(np.array(list(itertools.product(range(d), repeat=T)), dtype=np.int64))
    pw = torch.from_numpy(d ** np.arange(T - 1, -1, -1))
    x01 = torch.from_numpy((tr == 1).astype(np.int64))
    R = rows.numel()
    LL = torch.zeros((R, X, nb), dtype=chi.dtype)
    for ik in range(X):
        LL[:, :, int(x01[ik] @ pw)] += M[:, 0, ik, :]
    for m in range(1, d - 1):
        L = torch.zeros_like(LL)
        for ik in range(X):
            off = int(x01[ik] @ pw)
            srcs = torch.nonzero(torch.all(digits + x01[ik] < d, dim=1)).flatten()
            L[:, :, srcs + off] += LL[:, :, srcs] * M[:, m, ik, :][:, :, None]
        LL = L
    key = (T, p, c, d, attr_value)
    if key not in _A_CACHE:
        _A_CACHE[key] = torch.from_numpy(A_factor(T, p, c, d, attr_value))
    A = _A_CACHE[key]
    w = torch.exp(-lmbd_in * torch.from_numpy(tr[:, 0]).to(chi.dtype) / n)
    new = torch.einsum("raq,abq->rab", LL, A) * w[None, :, None]
    new = new.reshape(R, X * X)
    return damppar * new / new.sum(dim=1, keepdim=True) + (1 - damppar) * chi[rows]
