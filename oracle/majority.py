"""ORACLE (test infrastructure only): numpy restatement of the majority path.

Follows, function by function (paths relative to the reference repository):
  onestep_majority      code/SA_RRG.py:18-20  (and code/HPR_pytorch_RRG.py:169-171)
  s_endstate            code/SA_RRG.py:23-26
  m                     code/SA_RRG.py:39-40
  E_delta               code/SA_RRG.py:32-37
  sa_loop               code/SA_RRG.py:63-88
  onestep_majority_er   code/ER_BDCM_entropy.ipynb raw JSON lines 113-117 (sign(2S+s))
  s_endstate_er         same notebook, lines 120-123
"""
import numpy as np


def onestep_majority(N, s0):
    """S = sum of neighbour spins; new = sign(S), or s0 where S == 0.
    int64 throughout like the reference's numpy path (code/SA_RRG.py:19-20)."""
    s0 = np.asarray(s0, dtype=np.int64)
    S = np.sum(s0[np.asarray(N)], axis=-1)
    sg = np.sign(S)
    return (1 - np.abs(sg)) * s0 + sg


def s_endstate(N, s0, p, c):
    s = np.asarray(s0, dtype=np.int64)
    for _ in range(p + c - 1):
        s = onestep_majority(N, s)
    return s


def m(s, n=None):
    s = np.asarray(s)
    n = s.shape[-1] if n is None else n
    return np.sum(s, axis=-1) / n


def onestep_majority_batch(N, S0):
    """(R, n) batch version: every row is an independent replica."""
    S0 = np.asarray(S0, dtype=np.int64)
    tot = S0[:, np.asarray(N)].sum(axis=-1)
    sg = np.sign(tot)
    return (1 - np.abs(sg)) * S0 + sg


def s_endstate_batch(N, S0, p, c):
    S = np.asarray(S0, dtype=np.int64)
    for _ in range(p + c - 1):
        S = onestep_majority_batch(N, S)
    return S


# ---- Erdos-Renyi (CSR neighbour lists) ------------------------------------
def onestep_majority_er(row_ptr, col, s):
    """sign(2*S + s) with S the neighbour sum (nb:113-117); a degree-0 node
    keeps its spin."""
    s = np.asarray(s, dtype=np.int64)
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n = row_ptr.shape[0] - 1
    vals = s[..., np.asarray(col, dtype=np.int64)]
    csum = np.concatenate([np.zeros(s.shape[:-1] + (1,), np.int64), np.cumsum(vals, axis=-1)], axis=-1)
    S = csum[..., row_ptr[1:]] - csum[..., row_ptr[:-1]]
    assert S.shape[-1] == n
    return np.sign(2 * S + s)


def s_endstate_er(row_ptr, col, s, p, c):
    s = np.asarray(s, dtype=np.int64)
    for _ in range(p + c - 1):
        s = onestep_majority_er(row_ptr, col, s)
    return s


# ---- simulated annealing ----------------------------------------------------
def E_delta(N, s0, a, b, p, c, i, n=None):
    """(-2*a*s0[i] + b*(sum(s_end1) - sum(s_end2)))/n  (code/SA_RRG.py:32-37)."""
    n = len(s0) if n is None else n
    s_end1 = s_endstate(N, s0, p, c)
    s0_copy = np.array(s0, copy=True)
    s0_copy[i] = -s0[i]
    s_end2 = s_endstate(N, s0_copy, p, c)
    return (-2 * a * s0[i] + b * (np.sum(s_end1) - np.sum(s_end2))) / n


def sa_loop(N, p, c, seed, par_a=1.0005, par_b=1.0005, max_steps=None, trace=False):
    """One replica of the SA experiment with numpy's legacy MT19937 seeded by
    ``seed`` (the reference's global stream after np.random.seed(seed)).

    Returns dict(conf, num_steps, mag_reached, done[, trace]) where done is
    1 (consensus), 2 (t cap) or 0 (stopped by max_steps)."""
    N = np.asarray(N)
    n = N.shape[0]
    rs = np.random.RandomState(seed)
    s = 2 * rs.binomial(n=1, p=0.5, size=[n]) - 1            # code/SA_RRG.py:65
    a = 0.015 * n                                              # :67
    b = 0.01 * n                                               # :68
    t = 0
    tr_i, tr_acc, tr_sum, tr_dE = [], [], [], []
    sum_end = int(np.sum(s_endstate(N, s, p, c)))
    m_final = sum_end / n                                      # :71
    done = 0
    while m_final < 1:                                         # :72
        if max_steps is not None and t >= max_steps:
            break
        i = rs.randint(low=0, high=n)                          # :73
        delta_H = E_delta(N, s, a, b, p, c, i, n)              # :74
        prob_accept = min([1, np.exp(-delta_H)])               # :75
        acc = rs.rand() < prob_accept                          # :76
        if acc:
            s[i] = -s[i]                                       # :77
        if a < 4.5 * n:                                        # :80
            a = par_a * a
        if b < 5 * n:                                          # :81
            b = par_b * b
        t += 1                                                 # :82
        if t > (2 * n ** 3):                                   # :84
            m_final = 2
            done = 2
        else:
            sum_end = int(np.sum(s_endstate(N, s, p, c)))      # :85
            m_final = sum_end / n
            if m_final >= 1:
                done = 1
        if trace:
            tr_i.append(i)
            tr_acc.append(int(acc))
            tr_sum.append(sum_end)
            tr_dE.append(delta_H)
    if m_final >= 1 and done == 0:
        done = 1
    out = {"conf": s, "num_steps": t, "mag_reached": m(s, n), "done": done}
    if trace:
        out["trace"] = {"i": np.asarray(tr_i, np.int64), "accept": np.asarray(tr_acc, np.int8),
                        "sum_end": np.asarray(tr_sum, np.int64), "dE": np.asarray(tr_dE, np.float64)}
    return out
