/* ORACLE — test infrastructure only (never linked into libmjx.so, never on the
 * product path).  Plain-C restatement of the reference's majority path, used by
 * tests/ as a fast checker at the BASELINE configs' sizes (where the numpy
 * restatement in oracle/majority.py takes minutes per SA replica).
 *
 * Follows, function by function (paths relative to the reference repository):
 *   orc_onestep_ell     code/SA_RRG.py:18-20   (1-|sign S|)*s + sign S
 *   orc_s_endstate_ell  code/SA_RRG.py:23-26   p+c-1 steps
 *   orc_onestep_csr     code/ER_BDCM_entropy.ipynb raw lines 113-117  sign(2S+s)
 *   orc_s_endstate_csr  same notebook, lines 120-123
 *   orc_sa_loop         code/SA_RRG.py:63-88 (E_delta :32-37, m :39-40), with
 *                       numpy's legacy global MT19937 stream (np.random.seed,
 *                       binomial(1,.5), randint(0,n), rand) restated as in
 *                       oracle/mt19937.py.
 *   orc_sa_loop_philox  the same loop with the library's NON-parity proposal
 *                       stream: proposal t of a replica from
 *                       Philox-4x32-10 keyed by its seed (orc_philox4x32_10);
 *                       the initial configuration still from the seeded MT.
 * It does exactly what the reference does per proposal (three full rollouts:
 * s_endstate(s), s_endstate(s with s_i flipped), s_endstate(s) after the
 * step); no light-cone shortcut.  Pinned against the numpy oracle and the
 * reference-generated fixtures in tests/test_oracle_c.py.
 *
 * Build: oracle/build_oracle.py (gcc -O2 -ffp-contract=off -shared).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- MT19937 + numpy legacy distributions (oracle/mt19937.py) ------------ */
typedef struct {
    uint32_t mt[624];
    int idx;
} orc_mt;

static void mt_seed(orc_mt* s, uint32_t seed)
{
    s->mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = 624;
}

static uint32_t mt_u32(orc_mt* s)
{
    if (s->idx >= 624) {
        for (int k = 0; k < 624; ++k) {
            uint32_t y = (s->mt[k] & 0x80000000u) | (s->mt[(k + 1) % 624] & 0x7FFFFFFFu);
            s->mt[k] = s->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
        }
        s->idx = 0;
    }
    uint32_t y = s->mt[s->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
}

static double mt_double(orc_mt* s)
{
    uint32_t a = mt_u32(s) >> 5, b = mt_u32(s) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

static int64_t mt_randint(orc_mt* s, int64_t n)
{
    uint32_t rng = (uint32_t)(n - 1);
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    for (;;) {
        uint32_t v = mt_u32(s) & mask;
        if (v <= rng) return v;
    }
}

/* ---- Philox-4x32-10 ---------------------------------------------------------
 * Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3"
 * (SC'11), Random123's philox4x32_10: ten rounds of two 32x32->64 multiplies
 * (M0 = 0xD2511F53, M1 = 0xCD9E8D57) with the key bumped by the Weyl constants
 * (0x9E3779B9, 0xBB67AE85) between rounds.  Not the reference's generator: the
 * library's counter-based mode for runs that do not replay numpy's stream.
 * Pinned by Random123's known-answer vectors (tests/test_oracle_c.py). */
void orc_philox4x32_10(const uint32_t* ctr, const uint32_t* key, uint32_t* out)
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* proposal t (the replica's step count before it) keyed by the replica's seed:
 * counter (t_lo, t_hi, 0, 0), key (seed_lo, seed_hi); i = the high 64 bits of
 * (x0 | x1 << 32) * n, u = numpy rand()'s 53-bit double of (x2, x3) */
static void philox_prop(uint64_t seed, int64_t t, int64_t n, int64_t* i, double* u)
{
    const uint32_t ctr[4] = {(uint32_t)t, (uint32_t)((uint64_t)t >> 32), 0u, 0u};
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t x[4];
    orc_philox4x32_10(ctr, key, x);
    const uint64_t w = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
    *i = (int64_t)(((unsigned __int128)w * (uint64_t)n) >> 64);
    *u = ((double)(x[2] >> 5) * 67108864.0 + (double)(x[3] >> 6)) / 9007199254740992.0;
}

/* ---- dynamics -------------------------------------------------------------- */
void orc_onestep_ell(const int32_t* adj, int64_t n, int d, const int8_t* s, int8_t* out)
{
    for (int64_t i = 0; i < n; ++i) {
        int S = 0;
        for (int k = 0; k < d; ++k) S += s[adj[i * d + k]];
        out[i] = S > 0 ? 1 : (S < 0 ? -1 : s[i]);
    }
}

/* s_endstate: `steps` sweeps from s0 into out; returns sum(out). */
int64_t orc_s_endstate_ell(const int32_t* adj, int64_t n, int d, const int8_t* s0, int steps, int8_t* out,
                           int8_t* tmp)
{
    const int8_t* cur = s0;
    for (int t = 0; t < steps; ++t) {
        int8_t* dst = ((steps - 1 - t) % 2 == 0) ? out : tmp;
        orc_onestep_ell(adj, n, d, cur, dst);
        cur = dst;
    }
    if (steps == 0) memcpy(out, s0, (size_t)n);
    int64_t sum = 0;
    for (int64_t i = 0; i < n; ++i) sum += out[i];
    return sum;
}

void orc_onestep_csr(const int64_t* row_ptr, const int32_t* col, int64_t n, const int8_t* s, int8_t* out)
{
    for (int64_t i = 0; i < n; ++i) {
        int64_t S = 0;
        for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) S += s[col[k]];
        int64_t x = 2 * S + s[i];
        out[i] = x > 0 ? 1 : (x < 0 ? -1 : 0);
    }
}

int64_t orc_s_endstate_csr(const int64_t* row_ptr, const int32_t* col, int64_t n, const int8_t* s0, int steps,
                           int8_t* out, int8_t* tmp)
{
    const int8_t* cur = s0;
    for (int t = 0; t < steps; ++t) {
        int8_t* dst = ((steps - 1 - t) % 2 == 0) ? out : tmp;
        orc_onestep_csr(row_ptr, col, n, cur, dst);
        cur = dst;
    }
    if (steps == 0) memcpy(out, s0, (size_t)n);
    int64_t sum = 0;
    for (int64_t i = 0; i < n; ++i) sum += out[i];
    return sum;
}

/* ---- SA loop (code/SA_RRG.py:63-88) ----------------------------------------
 * One replica on numpy's stream after np.random.seed(seed).  Stops at
 * consensus, at the t > 2n^3 cap, or after max_steps (< 0: no limit).
 * Per-step traces (length >= max_steps when given): proposal i, accept,
 * sum(s_endstate) after the step, delta_H.  conf receives the final s.
 * Returns the number of steps taken; *done = 1 consensus, 2 cap, 0 stopped.
 * mt_io/idx_io (optional): the stream to continue instead of seeding, and
 * where the stream stands on return. */
static int64_t sa_loop(const int32_t* adj, int64_t n, int d, int p, int c, uint32_t seed, double par_a,
                       double par_b, int64_t max_steps, int32_t* tr_i, int8_t* tr_acc, int64_t* tr_sum,
                       double* tr_dE, int8_t* conf, int32_t* done, uint32_t* mt_io, int32_t* idx_io, int philox,
                       uint64_t key)
{
    int T = p + c - 1;
    int8_t* s = (int8_t*)malloc((size_t)n);
    int8_t* s2 = (int8_t*)malloc((size_t)n);
    int8_t* e1 = (int8_t*)malloc((size_t)n);
    int8_t* tmp = (int8_t*)malloc((size_t)n);
    orc_mt rs;
    if (mt_io) {            /* continue the given stream (numpy's ONE global stream, :58-65) */
        memcpy(rs.mt, mt_io, sizeof(rs.mt));
        rs.idx = *idx_io;
    } else {
        mt_seed(&rs, seed);
    }
    for (int64_t i = 0; i < n; ++i) s[i] = mt_double(&rs) > 0.5 ? 1 : -1;      /* :65 */
    double a = 0.015 * (double)n, b = 0.01 * (double)n;                        /* :67-68 */
    double a_cap = 4.5 * (double)n, b_cap = 5.0 * (double)n;                   /* :80-81 */
    /* 2*n**3 (:84) in Python integers; n <= 2^21 keeps it inside int64 */
    int64_t t_cap = 2 * n * n * n;
    int64_t t = 0;
    int64_t sum_end = orc_s_endstate_ell(adj, n, d, s, T, e1, tmp);            /* :71 */
    *done = 0;
    while (sum_end < n) {                                                      /* :72, m < 1 */
        if (max_steps >= 0 && t >= max_steps) break;
        int64_t i;
        double u;
        if (philox) philox_prop(key, t, n, &i, &u);
        else i = mt_randint(&rs, n);                                           /* :73 */
        /* E_delta (:32-37): two rollouts, the flipped one on a copy */
        int64_t sum1 = orc_s_endstate_ell(adj, n, d, s, T, e1, tmp);
        memcpy(s2, s, (size_t)n);
        s2[i] = (int8_t)-s2[i];
        int64_t sum2 = orc_s_endstate_ell(adj, n, d, s2, T, e1, tmp);
        volatile double m2a = -2.0 * a;                   /* (-2*a)*s0[i] + b*(diff), then /n */
        volatile double x1 = m2a * (double)s[i];
        volatile double x2 = b * (double)(sum1 - sum2);
        volatile double x3 = x1 + x2;
        double dH = x3 / (double)n;
        double prob = exp(-dH);                                                /* :75 min([1, exp]) */
        if (prob > 1.0) prob = 1.0;
        if (!philox) u = mt_double(&rs);                                       /* :76 */
        int acc = u < prob;
        if (acc) s[i] = (int8_t)-s[i];                                         /* :77 */
        if (a < a_cap) a = par_a * a;                                          /* :80 */
        if (b < b_cap) b = par_b * b;                                          /* :81 */
        t += 1;                                                                /* :82 */
        if (t > t_cap) {                                                       /* :84 */
            *done = 2;
        } else {
            sum_end = orc_s_endstate_ell(adj, n, d, s, T, e1, tmp);            /* :85 */
            if (sum_end >= n) *done = 1;
        }
        if (tr_i) {
            tr_i[t - 1] = (int32_t)i;
            tr_acc[t - 1] = (int8_t)acc;
            tr_sum[t - 1] = sum_end;
            tr_dE[t - 1] = dH;
        }
        if (*done == 2) break;
    }
    if (sum_end >= n) *done = 1;
    memcpy(conf, s, (size_t)n);
    if (mt_io) {
        memcpy(mt_io, rs.mt, sizeof(rs.mt));
        *idx_io = rs.idx;
    }
    free(s); free(s2); free(e1); free(tmp);
    return t;
}

int64_t orc_sa_loop(const int32_t* adj, int64_t n, int d, int p, int c, uint32_t seed, double par_a, double par_b,
                    int64_t max_steps, int32_t* tr_i, int8_t* tr_acc, int64_t* tr_sum, double* tr_dE, int8_t* conf,
                    int32_t* done, uint32_t* mt_io, int32_t* idx_io)
{
    return sa_loop(adj, n, d, p, c, seed, par_a, par_b, max_steps, tr_i, tr_acc, tr_sum, tr_dE, conf, done, mt_io,
                   idx_io, 0, 0);
}

/* key: the replica's 64-bit Philox key (the library uses its seed) */
int64_t orc_sa_loop_philox(const int32_t* adj, int64_t n, int d, int p, int c, uint32_t seed, uint64_t key,
                           double par_a, double par_b, int64_t max_steps, int32_t* tr_i, int8_t* tr_acc,
                           int64_t* tr_sum, double* tr_dE, int8_t* conf, int32_t* done)
{
    return sa_loop(adj, n, d, p, c, seed, par_a, par_b, max_steps, tr_i, tr_acc, tr_sum, tr_dE, conf, done, NULL,
                   NULL, 1, key);
}
