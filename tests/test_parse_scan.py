"""The lane-parallel stream parse (csrc/mjx_mt.h mt_window_starts, used by the
tape kernel and the whole-CU LDS kernels) restated in Python and checked
against the serial walk it replaced, on random windows: numpy's proposals
(code/SA_RRG.py:73,76) start at the first word randint's masked rejection
accepts at or after the previous proposal's end, then rand() takes two words.
The device form is pinned by the SA GPU tests (bit-exact streams); this pins
the algorithm: a 3-state automaton scanned by composing transition functions
(4 row shifts, 2 row broadcasts, as the DPP steps do), and the MT twist's
three-phase batching.  CPU only."""
import random

import numpy as np


def walk(ok, lim, room):
    """The serial walk: the starts whose two rand() words fit the window, at most room."""
    okm = sum(1 << i for i in range(64) if ok[i])
    stm, pos, got = 0, 0, 0
    while pos < 64 and got < room:
        m = okm >> pos
        if not m:
            break
        f = pos + (m & -m).bit_length() - 1
        if f + 2 >= lim:
            break
        stm |= 1 << f
        got += 1
        pos = f + 3
    return stm, (pos if got else 0)


def compose(g, h):                     # x -> g(h(x)), maps packed as three 2-bit fields
    return ((g >> (2 * (h & 3))) & 3) | (((g >> (2 * ((h >> 2) & 3))) & 3) << 2) | \
           (((g >> (2 * ((h >> 4) & 3))) & 3) << 4)


TOK, TNO = 1 | (2 << 2), 2 << 2       # acceptable word: 0->1, 1->2, 2->0; else 0->0, 1->2, 2->0


def scan(ok, lim, room):
    f = [TOK if ok[lane] else TNO for lane in range(64)]
    for d in (1, 2, 4, 8):             # row_shr:d inside 16-lane rows (no source: identity)
        f = [compose(f[lane], f[lane - d]) if lane % 16 >= d else f[lane] for lane in range(64)]
    g = list(f)                        # row_bcast:15 into rows 1 and 3
    for lane in range(64):
        if lane // 16 in (1, 3):
            g[lane] = compose(f[lane], f[16 * (lane // 16) - 1])
    f, g = g, list(g)                  # row_bcast:31 into rows 2 and 3
    for lane in range(64):
        if lane // 16 in (2, 3):
            g[lane] = compose(f[lane], f[31])
    starts = sum(1 << lane for lane in range(64) if (g[lane] & 3) == 1)
    stm = starts & (((1 << (lim - 2)) - 1) if lim >= 2 else 0)
    while bin(stm).count("1") > room:
        stm &= ~(1 << (stm.bit_length() - 1))
    got = bin(stm).count("1")
    return stm, (stm.bit_length() + 2 if got else 0)


def test_scan_equals_walk_on_random_windows():
    rnd = random.Random(1)
    for _ in range(5000):
        p = rnd.random()
        lim = rnd.choice([64] * 5 + list(range(1, 65)))
        ok = [(rnd.random() < p) and i < lim for i in range(64)]
        room = rnd.choice([64, 63, 17, 5, 1, 0])
        assert walk(ok, lim, room) == scan(ok, lim, room)


def test_twist_phase_batching_equals_the_recurrence():
    from oracle.mt19937 import MT19937
    N, M = 624, 397

    def mix(cur, nxt, far):
        y = (cur & 0x80000000) | (nxt & 0x7FFFFFFF)
        return far ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)

    def batched(buf):                  # csrc/mjx_mt.h lds_twist: reads of a phase before its writes
        buf = list(buf)
        P1 = N - M
        for lo, hi, far in ((0, P1, M), (P1, 2 * P1, -P1), (2 * P1, N - 1, -P1)):
            new = {k: mix(buf[k], buf[k + 1], buf[k + far]) for k in range(lo, hi)}
            for k, v in new.items():
                buf[k] = v
        buf[N - 1] = mix(buf[N - 1], buf[0], buf[M - 1])
        return buf

    for seed in (0, 5, 4095):
        m = MT19937(seed)
        state = [int(x) for x in m.mt]
        rs = np.random.RandomState(seed)
        ref = [int(x) for x in rs.get_state()[1]]
        assert state == ref                                   # the oracle's seeding is numpy's
        rs.random_sample()                                    # forces numpy's first twist
        twisted = [int(x) for x in rs.get_state()[1]]
        assert batched(state) == twisted
