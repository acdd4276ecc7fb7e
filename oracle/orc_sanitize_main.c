/* ORACLE (test infrastructure only): a host driver that runs the C
 * restatement (orc_majority.c, included below) under AddressSanitizer and
 * UndefinedBehaviorSanitizer (tests/test_oracle_sanitize.py builds it with
 * -fsanitize=address,undefined).  Random adjacency arrays (ELL and CSR with
 * isolated and high-degree nodes), rollouts checked against iterated single
 * steps, and SA loops (code/SA_RRG.py:63-88) at several (d, p, c) whose last
 * traced sum(s_end) must equal a fresh rollout of the returned conf.  Any
 * out-of-bounds access or undefined operation aborts the run. */
#include "orc_majority.c"
#include <stdio.h>

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

static int check_ell(int64_t n, int d) {
    int32_t* adj = malloc(sizeof(int32_t) * n * d);
    int8_t *s = malloc(n), *a = malloc(n), *b = malloc(n), *e = malloc(n), *tmp = malloc(n);
    for (int64_t i = 0; i < n * d; ++i) adj[i] = (int32_t)(rnd() % n);
    for (int64_t i = 0; i < n; ++i) s[i] = (rnd() & 1) ? 1 : -1;
    memcpy(a, s, n);
    for (int steps = 0; steps <= 4; ++steps) {
        int64_t sum = orc_s_endstate_ell(adj, n, d, s, steps, e, tmp);
        int64_t ref = 0;
        for (int64_t i = 0; i < n; ++i) ref += a[i];
        for (int64_t i = 0; i < n; ++i)
            if (e[i] != a[i]) { printf("ell n=%ld d=%d steps=%d: node %ld differs\n", (long)n, d, steps, (long)i); return 1; }
        if (sum != ref) { printf("ell sum differs\n"); return 1; }
        orc_onestep_ell(adj, n, d, a, b);
        memcpy(a, b, n);
    }
    free(adj); free(s); free(a); free(b); free(e); free(tmp);
    return 0;
}

static int check_csr(int64_t n) {
    int64_t* rp = malloc(sizeof(int64_t) * (n + 1));
    rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t k = rnd() % 16;
        rp[i + 1] = rp[i] + ((k < 3) ? 0 : (k < 14) ? (int64_t)(k - 2) : 40);   /* isolated, typical, hubs */
    }
    int32_t* col = malloc(sizeof(int32_t) * (rp[n] ? rp[n] : 1));
    for (int64_t j = 0; j < rp[n]; ++j) col[j] = (int32_t)(rnd() % n);
    int8_t *s = malloc(n), *a = malloc(n), *b = malloc(n), *e = malloc(n), *tmp = malloc(n);
    for (int64_t i = 0; i < n; ++i) s[i] = (rnd() & 1) ? 1 : -1;
    memcpy(a, s, n);
    for (int steps = 0; steps <= 3; ++steps) {
        orc_s_endstate_csr(rp, col, n, s, steps, e, tmp);
        for (int64_t i = 0; i < n; ++i)
            if (e[i] != a[i]) { printf("csr steps=%d: node %ld differs\n", steps, (long)i); return 1; }
        orc_onestep_csr(rp, col, n, a, b);
        memcpy(a, b, n);
    }
    free(rp); free(col); free(s); free(a); free(b); free(e); free(tmp);
    return 0;
}

static int check_sa(int64_t n, int d, int p, int c, int64_t K) {
    int32_t* adj = malloc(sizeof(int32_t) * n * d);
    for (int64_t i = 0; i < n * d; ++i) adj[i] = (int32_t)(rnd() % n);
    int32_t* ti = malloc(sizeof(int32_t) * K);
    int8_t* ta = malloc(K);
    int64_t* tsum = malloc(sizeof(int64_t) * K);
    double* tde = malloc(sizeof(double) * K);
    int8_t* conf = malloc(n);
    int8_t *e = malloc(n), *tmp = malloc(n);
    int32_t done = 0;
    uint32_t mt[624];
    int32_t idx = 624;
    orc_mt seeded;
    mt_seed(&seeded, 1234u);
    memcpy(mt, seeded.mt, sizeof(mt));
    idx = seeded.idx;
    const int64_t t = orc_sa_loop(adj, n, d, p, c, 0u, 1.0005, 1.0005, K, ti, ta, tsum, tde, conf, &done, mt, &idx);
    if (t < 1 || t > K) { printf("sa: %ld steps\n", (long)t); return 1; }
    const int64_t sum = orc_s_endstate_ell(adj, n, d, conf, p + c - 1, e, tmp);
    if (sum != tsum[t - 1]) { printf("sa n=%ld d=%d p=%d c=%d: sum_end %ld vs rollout %ld\n", (long)n, d, p, c,
                                     (long)tsum[t - 1], (long)sum); return 1; }
    for (int64_t k = 0; k < t; ++k)
        if (ti[k] < 0 || ti[k] >= n || (ta[k] != 0 && ta[k] != 1)) { printf("sa trace\n"); return 1; }
    if (idx < 0 || idx > 624) { printf("sa stream index %d\n", idx); return 1; }
    /* the Philox-stream loop on the same graph */
    const int64_t tp = orc_sa_loop_philox(adj, n, d, p, c, 7u, 7ull, 1.0005, 1.0005, K, ti, ta, tsum, tde, conf, &done);
    if (tp < 1 || tp > K) { printf("sa philox: %ld steps\n", (long)tp); return 1; }
    if (orc_s_endstate_ell(adj, n, d, conf, p + c - 1, e, tmp) != tsum[tp - 1]) { printf("sa philox sum\n"); return 1; }
    for (int64_t k = 0; k < tp; ++k)
        if (ti[k] < 0 || ti[k] >= n || (ta[k] != 0 && ta[k] != 1)) { printf("sa philox trace\n"); return 1; }
    free(adj); free(ti); free(ta); free(tsum); free(tde); free(conf); free(e); free(tmp);
    return 0;
}

int main(void) {
    int bad = 0;
    bad |= check_ell(1, 1);
    bad |= check_ell(64, 3);
    bad |= check_ell(1000, 4);
    bad |= check_ell(257, 6);
    bad |= check_csr(1);
    bad |= check_csr(777);
    bad |= check_sa(50, 3, 1, 1, 3000);
    bad |= check_sa(200, 4, 3, 1, 3000);
    bad |= check_sa(120, 4, 2, 2, 2000);
    bad |= check_sa(90, 6, 2, 1, 2000);
    if (bad) return 1;
    printf("ok\n");
    return 0;
}
