"""ORACLE (test infrastructure only): pure-Python MT19937 and the numpy legacy
distributions the SA uses.

Third-party algorithm restated: numpy 2.2.6 ``RandomState`` (legacy seeding
``mt19937_seed``, ``random_standard_uniform`` 53-bit doubles,
``legacy binomial`` inversion path, masked-rejection ``randint``), called by
the reference at code/SA_RRG.py:65,73,76.  Checked against numpy itself in
tests/test_oracle_golden.py.
"""

MT_N, MT_M = 624, 397


class MT19937:
    def __init__(self, seed):
        seed &= 0xFFFFFFFF
        mt = [0] * MT_N
        mt[0] = seed
        for i in range(1, MT_N):
            mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.mt, self.idx = mt, MT_N

    def _twist(self):
        mt = self.mt
        for k in range(MT_N):
            y = (mt[k] & 0x80000000) | (mt[(k + 1) % MT_N] & 0x7FFFFFFF)
            mt[k] = mt[(k + MT_M) % MT_N] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.idx = 0

    def u32(self):
        if self.idx >= MT_N:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y

    def random_double(self):
        a = self.u32() >> 5
        b = self.u32() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0

    def binomial_half(self):
        """binomial(n=1, p=0.5): one double U, returns U > 0.5 (inversion)."""
        return 1 if self.random_double() > 0.5 else 0

    def randint(self, n):
        """randint(low=0, high=n) for 1 <= n <= 2**32."""
        rng = n - 1
        if rng == 0:
            return 0
        mask = rng
        for sh in (1, 2, 4, 8, 16):
            mask |= mask >> sh
        while True:
            v = self.u32() & mask
            if v <= rng:
                return v
