// Simulated annealing over bit-packed replicas (code/SA_RRG.py:44-92).
//
// Replica r replays numpy's legacy global MT19937 after np.random.seed(seed_r)
// (SURVEY.md 0.1 SA3):
//   * init_genrand(seed) state, 32-bit tempered outputs;
//   * binomial(1, .5) consumes one double U per node and returns U > 0.5
//     (code/SA_RRG.py:65, s0 = 2*binomial - 1);
//   * randint(0, n): masked rejection on 32-bit words (code/SA_RRG.py:73);
//   * rand(): ((w1>>5)*67108864 + (w2>>6)) / 2^53 (code/SA_RRG.py:76).
// The draw sequence does not depend on accept decisions, so each replica's
// (i_t, u_t) tape is a pure function of its seed.
//
// One proposal of every running replica per step, evaluated by a full
// rollout of the flipped configuration (one rollout instead of the
// reference's three: sum(s_endstate(s)) of the current state is cached from
// the previous step's consensus check, code/SA_RRG.py:85).
//
// This translation unit is compiled with -ffp-contract=off: delta_H must be
// evaluated as ((-2*a)*s_i + b*D)/n with separately rounded operations, as
// numpy does (code/SA_RRG.py:37).
#include "mjx_common.h"
#include <map>
#include <memory>
#include <mutex>
#include "mjx_mt.h"
#include <math.h>
#include <stdlib.h>
#include <algorithm>
#include <type_traits>

#pragma clang fp contract(off)

namespace mjx {

// ---------------------------------------------------------------------------
// init: 64 replicas per block (one wave); their MT states live in LDS laid out
// [k][lane] (conflict-free), every lane consumes exactly 2 words per node so
// the wave twists in lockstep.  Bits are packed by ballot: the wave's 64
// replicas are exactly one replica-packed word column.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_sa_init_draw(int64_t n, int64_t R, int64_t W,
                                                     const uint32_t* __restrict__ seeds,
                                                     u64* __restrict__ s, uint32_t* __restrict__ mt_out,
                                                     int32_t* __restrict__ idx_out,
                                                     const uint32_t* __restrict__ mt_in = nullptr,
                                                     const int32_t* __restrict__ idx_in = nullptr) {
    __shared__ uint32_t st[MT_N * 64];
    const int lane = threadIdx.x;
    const int64_t w = blockIdx.x;
    const int64_t r = w * 64 + lane;
    const bool live = r < R;
    int idx = MT_N;
    if (mt_in) {                           // continue a given stream (numpy's global state)
        for (int k = 0; k < MT_N; ++k) st[k * 64 + lane] = live ? mt_in[r * MT_N + k] : 0u;
        idx = live ? idx_in[r] : MT_N;
    } else {
        uint32_t x = live ? seeds[r] : 0u;
        for (int k = 0; k < MT_N; ++k) {   // init_genrand / numpy mt19937_seed
            st[k * 64 + lane] = x;
            x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(k + 1);
        }
    }
    auto next = [&]() -> uint32_t {
        if (idx >= MT_N) {
            for (int k = 0; k < MT_N - MT_M; ++k)
                st[k * 64 + lane] = mt_mix(st[k * 64 + lane], st[(k + 1) * 64 + lane], st[(k + MT_M) * 64 + lane]);
            for (int k = MT_N - MT_M; k < MT_N - 1; ++k)
                st[k * 64 + lane] = mt_mix(st[k * 64 + lane], st[(k + 1) * 64 + lane],
                                           st[(k + MT_M - MT_N) * 64 + lane]);
            st[(MT_N - 1) * 64 + lane] = mt_mix(st[(MT_N - 1) * 64 + lane], st[lane], st[(MT_M - 1) * 64 + lane]);
            idx = 0;
        }
        return mt_temper(st[(idx++) * 64 + lane]);
    };
    for (int64_t v = 0; v < n; ++v) {
        uint32_t a = next();
        uint32_t b = next();
        bool plus = live && (mt_double(a, b) > 0.5);
        u64 word = __ballot(plus);
        if (lane == 0) s[v * W + w] = word;
    }
    if (live) {
        for (int k = 0; k < MT_N; ++k) mt_out[r * MT_N + k] = st[k * 64 + lane];
        idx_out[r] = idx;
    }
}

// ---------------------------------------------------------------------------
// init, wave per replica: the replica's MT19937 state in LDS, twisted by the
// whole wave; the 312 node draws of each twist become node-packed bits of a
// per-replica scratch row (ballot per 64-node word), then a 64x64 bit
// transpose per (word column, node word) writes the replica-packed layout.
// Same stream, same spins as k_sa_init_draw, with 64x the parallelism.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_sa_init_np(int64_t n, int64_t R, int64_t r0, const uint32_t* __restrict__ seeds,
                                                   u64* __restrict__ np_bits, uint32_t* __restrict__ mt_out,
                                                   int32_t* __restrict__ idx_out) {
    __shared__ uint32_t st[MT_N];
    __shared__ uint32_t tw[MT_N];
    const int lane = threadIdx.x;
    const int64_t r = r0 + blockIdx.x;
    const int64_t nw = (n + 63) >> 6;
    u64* row = np_bits + (int64_t)blockIdx.x * nw;
    if (r >= R) {                                    // padding replica: spins -1
        for (int64_t w = lane; w < nw; w += 64) row[w] = 0;
        return;
    }
    if (lane == 0) {                                 // init_genrand / numpy mt19937_seed
        uint32_t x = seeds[r];
        for (int k = 0; k < MT_N; ++k) {
            st[k] = x;
            x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(k + 1);
        }
    }
    __syncthreads();
    u64 acc = 0;
    for (int64_t v = 0; v < n; v += MT_N / 2) {
        lds_twist(st, lane);
        for (int k = lane; k < MT_N; k += 64) tw[k] = mt_temper(st[k]);
        __syncthreads();
        const int64_t vend = (n - v < MT_N / 2) ? n : v + MT_N / 2;
        for (int64_t c0 = v; c0 < vend;) {
            const int64_t ws = c0 & ~63ll, we = ws + 64;
            const int64_t node = ws + lane;
            bool plus = false;
            if (node >= c0 && node < vend) {
                const int j = (int)(node - v);
                plus = mt_double(tw[2 * j], tw[2 * j + 1]) > 0.5;      // binomial(1, .5) (code/SA_RRG.py:65)
            }
            acc |= __ballot(plus);
            if (we <= vend || vend == n) {
                if (lane == 0) row[ws >> 6] = acc;
                acc = 0;
            }
            c0 = we < vend ? we : vend;
        }
        __syncthreads();
    }
    for (int k = lane; k < MT_N; k += 64) mt_out[r * MT_N + k] = st[k];
    if (lane == 0) idx_out[r] = (int32_t)(2 * n - (int64_t)MT_N * ((2 * n + MT_N - 1) / MT_N - 1));
}

// word column w (64 replicas) x node word c: 64x64 bit transpose by ballots
__global__ void __launch_bounds__(256) k_np_to_rp(const u64* __restrict__ np_bits, int64_t n, int64_t W,
                                                  int64_t w0, int64_t ncols, u64* __restrict__ s) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (n + 63) >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    if (wave >= ncols * nw) return;                  // whole wave exits together
    const int64_t wl = wave / nw, c = wave % nw;
    const u64 x = np_bits[(wl * 64 + lane) * nw + c];
    u64 out = 0;
    for (int j = 0; j < 64; ++j) {
        const u64 b = __ballot((x >> j) & 1ull);
        if (lane == j) out = b;
    }
    const int64_t node = c * 64 + lane;
    if (node < n) s[node * W + (w0 + wl)] = out;
}

__global__ void k_sa_init_state(int64_t n, int64_t R, double a0, double b0,
                                const unsigned long long* __restrict__ cnt, mjx_sa_state st) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    st.a[r] = a0;
    st.b[r] = b0;
    st.t[r] = 0;
    const int64_t sum = 2 * (int64_t)cnt[r] - n;
    st.sum_end[r] = sum;
    st.done[r] = (sum == n) ? 1 : 0;   // m(s_endstate(s0)) == 1: loop never runs
    if (st.tr_tie) st.tr_tie[r] = 0;
}

// ---------------------------------------------------------------------------
// step kernels: one thread per replica, MT state replica-major in global
// memory mt[r*624 + k].  A lane that runs out of words gets its state twisted
// cooperatively by its whole wave through a 624-word LDS buffer.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_nc(const uint32_t* p) {
    // bypass the CU's L1: the words may have been rewritten by this wave's
    // own cooperative twist earlier in this launch
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void coop_twist(uint32_t* __restrict__ g, uint32_t* buf, int lane) {
    for (int k = lane; k < MT_N; k += 64) buf[k] = ld_nc(g + k);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    lds_twist(buf, lane);
    for (int k = lane; k < MT_N; k += 64) g[k] = buf[k];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct WaveMT {
    uint32_t* mt;      // all replicas
    uint32_t* buf;     // this wave's LDS twist buffer
    int64_t r;
    int idx;
    int lane;
    // wave-uniform call: lanes with want == false still participate
    __device__ __forceinline__ uint32_t draw(bool want) {
        const bool tw = want && idx >= MT_N;
        u64 m = __ballot(tw);
        const int64_t base = r - lane;
        while (m) {
            const int l = __ffsll((unsigned long long)m) - 1;
            coop_twist(mt + (base + l) * MT_N, buf, lane);
            m &= m - 1;
        }
        if (tw) idx = 0;
        uint32_t y = 0;
        if (want) y = mt_temper(ld_nc(mt + r * MT_N + idx++));
        return y;
    }
};

__global__ void __launch_bounds__(kBlock) k_sa_propose(int64_t n, int64_t R, int64_t W, u64* __restrict__ s,
                                                       mjx_sa_state st, int64_t step) {
    __shared__ uint32_t twist_buf[kBlock / 64][MT_N];
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool live = r < R;
    const bool active = live && st.done[r] == 0;
    WaveMT g{st.mt, twist_buf[threadIdx.x >> 6], r, live ? st.mt_idx[r] : MT_N, lane};
    // randint(low=0, high=n): numpy legacy masked rejection
    const uint64_t rng = (uint64_t)(n - 1);
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    bool pending = active && rng > 0;
    uint32_t i = 0;
    while (__ballot(pending)) {
        uint32_t y = g.draw(pending);
        if (pending) {
            uint32_t v = y & mask;
            if (v <= (uint32_t)rng) { i = v; pending = false; }
        }
    }
    // rand()
    uint32_t w1 = g.draw(active);
    uint32_t w2 = g.draw(active);
    if (live) st.mt_idx[r] = g.idx;
    if (active) {
        const double u = mt_double(w1, w2);
        const u64 bit = 1ull << (r & 63);
        const u64 old = atomicXor((unsigned long long*)&s[(int64_t)i * W + (r >> 6)], (unsigned long long)bit);
        st.prop_i[r] = (int32_t)i;
        st.prop_s[r] = (old & bit) ? 1 : -1;   // s0[i] before the flip
        st.prop_u[r] = u;
    }
    if (live && st.tr_i) st.tr_i[step * R + r] = active ? (int32_t)i : -1;
}

__global__ void __launch_bounds__(kBlock) k_sa_accept(int64_t n, int64_t R, int64_t W, u64* __restrict__ s,
                                                      mjx_sa_state st, int64_t step, double par_a, double par_b,
                                                      double a_cap, double b_cap, int64_t t_cap) {
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (r >= R) return;
    if (st.done[r] != 0) {
        if (st.tr_acc) st.tr_acc[step * R + r] = -1;
        if (st.tr_sum) st.tr_sum[step * R + r] = st.sum_end[r];
        if (st.tr_dE) st.tr_dE[step * R + r] = 0.0;
        return;
    }
    const int64_t sum_new = 2 * (int64_t)st.cnt[r] - n;        // sum(s_endstate(s with i flipped))
    const int64_t sum_old = st.sum_end[r];                      // sum(s_endstate(s))
    const double a = st.a[r], b = st.b[r];
    const double si = (double)st.prop_s[r];
    // delta_H = (-2*a*s0[i] + b*(sum(s_end1) - sum(s_end2)))/n   (code/SA_RRG.py:37)
    const double t1 = (-2.0 * a) * si;
    const double t2 = b * (double)(sum_old - sum_new);
    const double dE = (t1 + t2) / (double)n;
    // prob_accept = min([1, np.exp(-delta_H)])                 (code/SA_RRG.py:75)
    const double e = exp(-dE);
    const double prob = (e < 1.0) ? e : 1.0;
    const double u = st.prop_u[r];
    const bool acc = u < prob;                                  // (code/SA_RRG.py:76)
    if (st.tr_tie && e < 1.0) {
        const double gap = fabs(u - e);
        if (gap <= 4.0 * (nextafter(e, 2.0) - e)) st.tr_tie[r] += 1;
    }
    int64_t sum_cur = sum_old;
    if (acc) {
        sum_cur = sum_new;
    } else {
        const int32_t i = st.prop_i[r];
        atomicXor((unsigned long long*)&s[(int64_t)i * W + (r >> 6)], (unsigned long long)(1ull << (r & 63)));
    }
    // annealing schedule (code/SA_RRG.py:80-81)
    double an = a, bn = b;
    if (a < a_cap) an = par_a * a;
    if (b < b_cap) bn = par_b * b;
    st.a[r] = an;
    st.b[r] = bn;
    const int64_t t = st.t[r] + 1;                               // (code/SA_RRG.py:82)
    st.t[r] = t;
    st.sum_end[r] = sum_cur;
    if (t > t_cap) st.done[r] = 2;                              // m_final = 2 (code/SA_RRG.py:84)
    else if (sum_cur == n) st.done[r] = 1;                      // m(s_endstate(s)) == 1
    if (st.tr_acc) st.tr_acc[step * R + r] = acc ? 1 : 0;
    if (st.tr_sum) st.tr_sum[step * R + r] = sum_cur;
    if (st.tr_dE) st.tr_dE[step * R + r] = dE;
}


// ---------------------------------------------------------------------------
// Light-cone SA.  sum(s_endstate(s with s_i flipped)) -
// sum(s_endstate(s)) is evaluated exactly from cached levels
// s_0 = s, s_t = onestep^t(s_0) (t = 1..T, T = p+c-1): a flip at i can change
// s_t only inside the radius-t ball around i, and only nodes whose level-(t-1)
// inputs changed need re-evaluation.  Per level the changed nodes are kept in a
// per-lane list (LDS, [slot][lane]), candidates are the changed nodes of the
// previous level and their neighbours.  The accept sequence is bit-identical
// to the full rollout (same integer sum, same float64 delta_H).
//
// One wave = the 64 replicas of one replica-packed word column, so no other
// wave ever touches these words; words are read with agent-scope (L1
// bypassing) loads because the wave's own accepted flips are atomics.
// ---------------------------------------------------------------------------
constexpr int LC_MAXT = 6;
constexpr int LC_MAXD = 16;

struct LcLevels {
    u64* s[LC_MAXT + 1];     // s[0] = current configuration, s[t] = onestep^t(s[0])
    // word (node v, column col) of level t at s[t] + v * ns + col * cs: ns = W,
    // cs = 1 for separate level arrays; ns = W * LV, cs = LV for the cone
    // layout, whose levels of one (node, column) share a 32-B sector
    int64_t ns;
    int64_t cs;
    u64* s0c;                // cone layout: the configuration's own array (level-0 flips mirrored), else null
    int lo;                  // record layout (cone with rows): a (node, column) record of ns words holds the
                             // node's adjacency row (int32 x4) in words 0..1 and level t at word lo + t
                             // (s[t] = record base + lo + t); 0 = the plain cone / separate levels
    int off[LC_MAXT + 2];    // list slot offset of level t; off[T+1] = candidate list
    int tab;                 // slot offset of the ball table (node ids | adjacency rows | candidate entries)
    int ball;                // table capacity: nodes of the radius-T ball (d-regular bound)
};

__device__ __forceinline__ u64 ld_word(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D>
__device__ __forceinline__ int lc_nbrs(const int32_t* __restrict__ adj, int d, int32_t v, int32_t* k) {
    if constexpr (D > 0) {
#pragma unroll
        for (int j = 0; j < D; ++j) k[j] = adj[(int64_t)v * D + j];
        return D;
    } else {
        for (int j = 0; j < d; ++j) k[j] = adj[(int64_t)v * d + j];
        return d;
    }
}

// value (0/1) of node k at level t-1 as seen by the proposal: the list entry
// if k changed at that level, else the cached word bit
__device__ __forceinline__ uint32_t lc_val(const uint32_t* prev, int np, int32_t k, const u64* lvl, int64_t W,
                                           int64_t col, u64 bit) {
    for (int q = 0; q < np; ++q) {
        const uint32_t e = prev[q * 64];
        if ((int32_t)(e & 0x7fffffffu) == k) return e >> 31;
    }
    return (ld_word(lvl + (int64_t)k * W + col) & bit) ? 1u : 0u;
}

__device__ __forceinline__ void lc_add_unique(uint32_t* U, int& nu, int32_t v) {
    for (int q = 0; q < nu; ++q)
        if ((int32_t)U[q * 64] == v) return;
    U[nu * 64] = (uint32_t)v;
    ++nu;
}

// Returns sum(s_end(flipped)) - sum(s_end); fills the per-level change lists
// (cnt[t] entries at lists + off[t]*64) and the old spin of i.
template <int D>
__device__ int64_t lc_delta(const int32_t* __restrict__ adj, int d, int64_t W, int64_t col, u64 bit, int T,
                            const LcLevels& L, uint32_t* lists, int32_t i, int* cnt, int* old_i) {
    const u64 w0 = ld_word(L.s[0] + (int64_t)i * W + col);
    *old_i = (w0 & bit) ? 1 : 0;
    lists[L.off[0] * 64] = (uint32_t)i | ((w0 & bit) ? 0u : 0x80000000u);
    cnt[0] = 1;
    int t = 1;
    for (; t <= T; ++t) {
        const uint32_t* prev = lists + L.off[t - 1] * 64;
        uint32_t* U = lists + L.off[T + 1] * 64;
        uint32_t* cur = lists + L.off[t] * 64;
        const int np = cnt[t - 1];
        int nu = 0;
        for (int q = 0; q < np; ++q) {
            const int32_t v = (int32_t)(prev[q * 64] & 0x7fffffffu);
            int32_t k[D > 0 ? D : LC_MAXD];
            const int dd = lc_nbrs<D>(adj, d, v, k);
            lc_add_unique(U, nu, v);
            for (int j = 0; j < dd; ++j) lc_add_unique(U, nu, k[j]);
        }
        int nc = 0;
        for (int q = 0; q < nu; ++q) {
            const int32_t j = (int32_t)U[q * 64];
            int32_t k[D > 0 ? D : LC_MAXD];
            const int dd = lc_nbrs<D>(adj, d, j, k);
            int ones = 0;
            for (int m = 0; m < dd; ++m) ones += (int)lc_val(prev, np, k[m], L.s[t - 1], W, col, bit);
            const uint32_t own = lc_val(prev, np, j, L.s[t - 1], W, col, bit);
            // always-stay majority (code/SA_RRG.py:19-20)
            const uint32_t nb = (2 * ones > dd) ? 1u : ((2 * ones < dd) ? 0u : own);
            const uint32_t ob = (ld_word(L.s[t] + (int64_t)j * W + col) & bit) ? 1u : 0u;
            if (nb != ob) {
                cur[nc * 64] = (uint32_t)j | (nb << 31);
                ++nc;
            }
        }
        cnt[t] = nc;
        if (nc == 0) break;          // nothing propagates further
    }
    for (int u = t + 1; u <= T; ++u) cnt[u] = 0;
    if (t <= T) return 0;
    int64_t ds = 0;
    const uint32_t* last = lists + L.off[T] * 64;
    for (int q = 0; q < cnt[T]; ++q) ds += (last[q * 64] >> 31) ? 2 : -2;
    return ds;
}

// The same result as lc_delta, with the loads of a level issued together: the
// ball's nodes and adjacency rows are kept in a per-lane LDS table (entries in
// BFS order), the rows of the entries a level adds are loaded in one batch,
// and the level words of up to CH candidates (own, D neighbours, cached next
// level) in one batch, so a level costs two dependent memory round trips
// instead of one per load.
template <int D>
struct LcChunk {
    static constexpr int CH = (D <= 4) ? 16 : 8;
};

__device__ __forceinline__ int tab_find(const uint32_t* tnode, int nt, int32_t v) {
    for (int e = 0; e < nt; ++e)
        if ((int32_t)tnode[e * 64] == v) return e;
    return -1;
}

// 128-bit membership filter of node ids kept in two registers: a clear bit
// proves absence, so most table / change-list lookups skip their LDS scan
struct Bloom {
    u64 lo = 0, hi = 0;
    __device__ __forceinline__ static uint32_t slot(int32_t v) { return ((uint32_t)v * 0x9E3779B1u) >> 25; }
    __device__ __forceinline__ void add(int32_t v) {
        const uint32_t b = slot(v);
        if (b < 64) lo |= 1ull << b; else hi |= 1ull << (b - 64);
    }
    __device__ __forceinline__ bool maybe(int32_t v) const {
        const uint32_t b = slot(v);
        return ((b < 64 ? lo >> b : hi >> (b - 64)) & 1ull) != 0;
    }
};

// PRE: the rows of i (p0) and of its neighbours (p1) were loaded during the
// previous step (tape lookahead), so level 1 starts with its word batch and
// the word of i joins that batch.
template <int D, bool PRE>
__device__ int64_t lc_delta_mlp(const int32_t* __restrict__ adj, int64_t W, int64_t col, u64 bit, int T,
                                const LcLevels& L, uint32_t* lists, int32_t i, int* cnt, int* old_i,
                                const int32_t (&p0)[D], const int32_t (&p1)[D][D]) {
    constexpr int CH = LcChunk<D>::CH;
    const int B = L.ball;
    uint32_t* tnode = lists + L.tab * 64;                                // [B] node id
    int32_t* tadj = (int32_t*)(lists + (L.tab + B) * 64);                // [B][D] adjacency row
    uint32_t* ul = lists + (L.tab + B * (1 + D)) * 64;                   // [B] candidates of this level
    int32_t* tmark = (int32_t*)(lists + (L.tab + B * (2 + D)) * 64);     // [B] level it was last a candidate
    int32_t* tval = (int32_t*)(lists + (L.tab + B * (3 + D)) * 64);      // [B] (level << 1 | value) if changed
    uint32_t* cind = lists + (L.tab + B * (4 + D)) * 64;                 // entry of every change-list slot
    Bloom tab;
    int nt = 1, nadj = 1;
    tnode[0] = (uint32_t)i;
    tmark[0] = 0;
    tab.add(i);
    cind[L.off[0] * 64] = 0;
    cnt[0] = 1;
    if constexpr (PRE) {
        // entries 0..D: i and its neighbours, rows known; the word of i and
        // the level-0 list entry are completed inside level 1's batch
#pragma unroll
        for (int m = 0; m < D; ++m) {
            tadj[m * 64] = p0[m];
            tnode[(1 + m) * 64] = (uint32_t)p0[m];
            tmark[(1 + m) * 64] = 0;
            tval[(1 + m) * 64] = -2;
            tab.add(p0[m]);
#pragma unroll
            for (int q = 0; q < D; ++q) tadj[((1 + m) * D + q) * 64] = p1[m][q];
        }
        nt = nadj = 1 + D;
        lists[L.off[0] * 64] = (uint32_t)i;
    } else {
        // level 0: the flipped node, its row and its word, in one round trip
        int32_t r0[D];
#pragma unroll
        for (int m = 0; m < D; ++m) r0[m] = adj[(int64_t)i * D + m];
        const u64 w0 = ld_word(L.s[0] + (int64_t)i * W + col);
#pragma unroll
        for (int m = 0; m < D; ++m) tadj[m * 64] = r0[m];
        const uint32_t flipped = (w0 & bit) ? 0u : 1u;
        tval[0] = (int32_t)flipped;                       // level 0, new value
        *old_i = (w0 & bit) ? 1 : 0;
        lists[L.off[0] * 64] = (uint32_t)i | (flipped << 31);
    }
    int t = 1;
    for (; t <= T; ++t) {
        const uint32_t* prev = lists + L.off[t - 1] * 64;
        const uint32_t* pind = cind + L.off[t - 1] * 64;
        uint32_t* cur = lists + L.off[t] * 64;
        uint32_t* cdst = cind + L.off[t] * 64;
        const int np = cnt[t - 1];
        Bloom pb;                                      // the changed nodes of level t-1
        // candidates: the changed nodes of level t-1 and their neighbours
        int nu = 0;
        for (int q = 0; q < np; ++q) {
            const int e = (int)pind[q * 64];
            pb.add((int32_t)tnode[e * 64]);
            if (tmark[e * 64] != t) {
                tmark[e * 64] = t;
                ul[(nu++) * 64] = (uint32_t)e;
            }
            for (int m = 0; m < D; ++m) {
                const int32_t k = tadj[(e * D + m) * 64];
                int ek = tab.maybe(k) ? tab_find(tnode, nt, k) : -1;
                if (ek < 0) {
                    ek = nt++;
                    tnode[ek * 64] = (uint32_t)k;
                    tmark[ek * 64] = 0;
                    tval[ek * 64] = -2;
                    tab.add(k);
                }
                if (tmark[ek * 64] != t) {
                    tmark[ek * 64] = t;
                    ul[(nu++) * 64] = (uint32_t)ek;
                }
            }
        }
        // adjacency rows of the entries this level added, one batch per CH
        for (int base = nadj; base < nt; base += CH) {
            int32_t rr[CH][D];
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                if (base + e < nt) {
                    const int64_t node = (int64_t)tnode[(base + e) * 64];
#pragma unroll
                    for (int m = 0; m < D; ++m) rr[e][m] = adj[node * D + m];
                }
            }
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                if (base + e < nt) {
#pragma unroll
                    for (int m = 0; m < D; ++m) tadj[((base + e) * D + m) * 64] = rr[e][m];
                }
            }
        }
        nadj = nt;
        // level words of the candidates, one batch per CH, then the rule
        int nc = 0;
        const u64* lp = L.s[t - 1];
        const u64* lt = L.s[t];
        u64 wi = 0;
        if (PRE && t == 1) wi = ld_word(L.s[0] + (int64_t)i * W + col);
        for (int base = 0; base < nu; base += CH) {
            u64 wn[CH][D], wo[CH], wc[CH];
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                if (base + e < nu) {
                    const int ent = (int)ul[(base + e) * 64];
                    const int64_t node = (int64_t)tnode[ent * 64];
                    wo[e] = ld_word(lp + node * W + col);
                    wc[e] = ld_word(lt + node * W + col);
#pragma unroll
                    for (int m = 0; m < D; ++m) wn[e][m] = ld_word(lp + (int64_t)tadj[(ent * D + m) * 64] * W + col);
                }
            }
            if (PRE && t == 1 && base == 0) {     // the level-0 entry, now that the word of i is in
                const uint32_t flipped = (wi & bit) ? 0u : 1u;
                tval[0] = (int32_t)flipped;
                *old_i = (wi & bit) ? 1 : 0;
                lists[L.off[0] * 64] = (uint32_t)i | (flipped << 31);
            }
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                if (base + e < nu) {
                    const int ent = (int)ul[(base + e) * 64];
                    const int32_t j = (int32_t)tnode[ent * 64];
                    int ones = 0;
#pragma unroll
                    for (int m = 0; m < D; ++m) {
                        const int32_t k = tadj[(ent * D + m) * 64];
                        uint32_t v = (wn[e][m] & bit) ? 1u : 0u;
                        if (pb.maybe(k)) {
                            for (int q = 0; q < np; ++q) {
                                const uint32_t pe = prev[q * 64];
                                if ((int32_t)(pe & 0x7fffffffu) == k) v = pe >> 31;
                            }
                        }
                        ones += (int)v;
                    }
                    const int32_t tv = tval[ent * 64];
                    const uint32_t own = ((tv >> 1) == t - 1) ? (uint32_t)(tv & 1) : ((wo[e] & bit) ? 1u : 0u);
                    // always-stay majority (code/SA_RRG.py:19-20)
                    const uint32_t nb = (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
                    const uint32_t ob = (wc[e] & bit) ? 1u : 0u;
                    if (nb != ob) {
                        cur[nc * 64] = (uint32_t)j | (nb << 31);
                        cdst[nc * 64] = (uint32_t)ent;
                        tval[ent * 64] = (t << 1) | (int32_t)nb;
                        ++nc;
                    }
                }
            }
        }
        cnt[t] = nc;
        if (nc == 0) break;          // nothing propagates further
    }
    for (int u = t + 1; u <= T; ++u) cnt[u] = 0;
    if (t <= T) return 0;
    int64_t ds = 0;
    const uint32_t* last = lists + L.off[T] * 64;
    for (int q = 0; q < cnt[T]; ++q) ds += (last[q * 64] >> 31) ? 2 : -2;
    return ds;
}

// Radius-2 ball as a tree in registers (T <= 2, D <= 4): when i, its D
// neighbours a_m and their D(D-1) other neighbours (the children) are all
// distinct -- every ball of a random regular graph except the few that hold a
// short cycle -- the positions of the ball's nodes are fixed by the adjacency
// rows, so candidate sets are bit tests and every value is read from a
// register: no table, no scans.  Level 1 is one batch of words (level-0 words
// of i, the a_m and the row entries of every a_m; level-1 words of i and the
// a_m), level 2 two batches (rows and words of the children whose parent
// changed, level-2 words of the candidates; then the level-1 words of those
// children's neighbours).  Same change lists and sum as lc_delta.  Returns
// false (nothing written) when the ball is not such a tree.
template <int D>
__device__ bool lc_tree2(const int32_t* __restrict__ adj, int64_t W, int64_t col, u64 bit, int T,
                         const LcLevels& L, uint32_t* lists, int32_t i, int* cnt, int* old_i,
                         const int32_t (&r0)[D], const int32_t (&r1)[D][D], int64_t& ds) {
    // shape: i once in every a_m's row, all 1 + D + D(D-1) nodes distinct
    bool ok = true;
#pragma unroll
    for (int m = 0; m < D; ++m) {
        int ci = 0;
#pragma unroll
        for (int x = 0; x < D; ++x) ci += (r1[m][x] == i);
        ok &= (ci == 1) && (r0[m] != i);
#pragma unroll
        for (int m2 = m + 1; m2 < D; ++m2) ok &= r0[m] != r0[m2];
    }
    if (!ok) return false;
#pragma unroll
    for (int m = 0; m < D; ++m)
#pragma unroll
        for (int x = 0; x < D; ++x) {
            const int32_t c = r1[m][x];
            if (c == i) continue;
#pragma unroll
            for (int m2 = 0; m2 < D; ++m2) ok &= (c != r0[m2]);
#pragma unroll
            for (int m2 = m; m2 < D; ++m2)
#pragma unroll
                for (int x2 = 0; x2 < D; ++x2)
                    if (m2 > m || x2 > x) ok &= (r1[m2][x2] == i) || (r1[m2][x2] != c);
        }
    if (!ok) return false;
    const u64* s0 = L.s[0];
    const u64* s1 = L.s[1];
    auto w = [&](const u64* lv, int32_t v) { return ld_word(lv + (int64_t)v * W + col); };
    auto b = [&](u64 x) -> uint32_t { return (x & bit) ? 1u : 0u; };
    auto maj = [&](int ones, uint32_t own) -> uint32_t { return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own); };
    // level 1: one batch
    u64 wi0 = w(s0, i), wi1 = w(s1, i), wa0[D], wa1[D], wr0[D][D];
#pragma unroll
    for (int m = 0; m < D; ++m) {
        wa0[m] = w(s0, r0[m]);
        wa1[m] = w(s1, r0[m]);
#pragma unroll
        for (int x = 0; x < D; ++x) wr0[m][x] = w(s0, r1[m][x]);
    }
    const uint32_t f = b(wi0) ^ 1u;                  // flipped spin of i
    *old_i = (int)b(wi0);
    lists[L.off[0] * 64] = (uint32_t)i | (f << 31);
    cnt[0] = 1;
    uint32_t ch1 = 0, nv1 = 0;                       // bit e: entry e (0 = i, 1+m = a_m) changed / new value
    {
        int ones = 0;
#pragma unroll
        for (int m = 0; m < D; ++m) ones += (int)b(wa0[m]);
        const uint32_t nb = maj(ones, f);
        if (nb != b(wi1)) { ch1 |= 1u; nv1 |= nb; }
    }
#pragma unroll
    for (int m = 0; m < D; ++m) {
        int ones = 0;
#pragma unroll
        for (int x = 0; x < D; ++x) ones += (int)((r1[m][x] == i) ? f : b(wr0[m][x]));
        const uint32_t nb = maj(ones, b(wa0[m]));
        if (nb != b(wa1[m])) { ch1 |= 2u << m; nv1 |= nb << (1 + m); }
    }
    int n1 = 0;
    uint32_t* l1 = lists + L.off[1] * 64;
    if (ch1 & 1u) l1[(n1++) * 64] = (uint32_t)i | ((nv1 & 1u) << 31);
#pragma unroll
    for (int m = 0; m < D; ++m)
        if ((ch1 >> (1 + m)) & 1u) l1[(n1++) * 64] = (uint32_t)r0[m] | (((nv1 >> (1 + m)) & 1u) << 31);
    cnt[1] = n1;
    if (T == 1 || n1 == 0) {
        if (T >= 2) cnt[2] = 0;
        ds = 0;
        if (T == 1) {
            for (int q = 0; q < n1; ++q) ds += (l1[q * 64] >> 31) ? 2 : -2;
        }
        return true;
    }
    // level 2
    const u64* s2 = L.s[2];
    const bool c0 = ch1 & 1u;
    const bool u0 = ch1 != 0;                        // i is a candidate if it or any a_m changed
    u64 wi2 = 0, wa2[D], wc1[D][D], wc2[D][D];
    int32_t cr[D][D][D];
    if (u0) wi2 = w(s2, i);
#pragma unroll
    for (int m = 0; m < D; ++m) {
        const bool cm = (ch1 >> (1 + m)) & 1u;
        wa2[m] = 0;
        if (c0 || cm) wa2[m] = w(s2, r0[m]);
#pragma unroll
        for (int x = 0; x < D; ++x) {
            wc1[m][x] = 0;
            wc2[m][x] = 0;
            if (r1[m][x] == i) continue;
            if (c0 || cm) wc1[m][x] = w(s1, r1[m][x]);        // neighbour value of a_m
            if (cm) {
                wc2[m][x] = w(s2, r1[m][x]);
#pragma unroll
                for (int y = 0; y < D; ++y) cr[m][x][y] = adj[(int64_t)r1[m][x] * D + y];
            }
        }
    }
    u64 wg[D][D][D];
#pragma unroll
    for (int m = 0; m < D; ++m) {
        const bool cm = (ch1 >> (1 + m)) & 1u;
#pragma unroll
        for (int x = 0; x < D; ++x)
#pragma unroll
            for (int y = 0; y < D; ++y) {
                wg[m][x][y] = 0;
                if (cm && r1[m][x] != i && cr[m][x][y] != r0[m]) wg[m][x][y] = w(s1, cr[m][x][y]);
            }
    }
    int n2 = 0;
    int64_t acc = 0;
    uint32_t* l2 = lists + L.off[2] * 64;
    auto emit = [&](int32_t node, uint32_t nb) {
        l2[(n2++) * 64] = (uint32_t)node | (nb << 31);
        acc += nb ? 2 : -2;
    };
    const uint32_t vi1 = c0 ? (nv1 & 1u) : b(wi1);   // level-1 value of i
    if (u0) {
        int ones = 0;
#pragma unroll
        for (int m = 0; m < D; ++m) ones += (int)(((ch1 >> (1 + m)) & 1u) ? ((nv1 >> (1 + m)) & 1u) : b(wa1[m]));
        const uint32_t nb = maj(ones, vi1);
        if (nb != b(wi2)) emit(i, nb);
    }
#pragma unroll
    for (int m = 0; m < D; ++m) {
        const bool cm = (ch1 >> (1 + m)) & 1u;
        const uint32_t va1 = cm ? ((nv1 >> (1 + m)) & 1u) : b(wa1[m]);
        if (c0 || cm) {
            int ones = 0;
#pragma unroll
            for (int x = 0; x < D; ++x) ones += (int)((r1[m][x] == i) ? vi1 : b(wc1[m][x]));
            const uint32_t nb = maj(ones, va1);
            if (nb != b(wa2[m])) emit(r0[m], nb);
        }
        if (cm) {
#pragma unroll
            for (int x = 0; x < D; ++x) {
                if (r1[m][x] == i) continue;
                int ones = 0;
#pragma unroll
                for (int y = 0; y < D; ++y) ones += (int)((cr[m][x][y] == r0[m]) ? va1 : b(wg[m][x][y]));
                const uint32_t nb = maj(ones, b(wc1[m][x]));
                if (nb != b(wc2[m][x])) emit(r1[m][x], nb);
            }
        }
    }
    cnt[2] = n2;
    ds = (n2 == 0) ? 0 : acc;
    return true;
}

// (i_t, u_t) tape of K proposals per running replica (code/SA_RRG.py:73,76):
// wave per replica, its MT19937 state twisted in LDS.  The stream does not
// depend on accept decisions, so the tape can run ahead of the steps; a replica
// that finishes inside the tape leaves its tail unused.  The draws are parsed
// a 64-word window at a time, lane-parallel (as the whole-CU LDS kernels parse
// them): every lane tempers one word and tests randint's masked rejection; a
// scalar walk over the ballot finds the proposal starts (the first acceptable
// word at or after the previous proposal's end, then rand()'s two words); the
// start lanes write their proposals' tape entries.  A proposal whose words
// cross the end of the state is drawn serially across the twist, as numpy does.
__global__ void __launch_bounds__(64) k_sa_tape(int64_t n, int64_t R, int64_t K, mjx_sa_state st,
                                                int32_t* __restrict__ tape_i, double* __restrict__ tape_u) {
    __shared__ uint32_t buf[MT_N];
    const int64_t r = blockIdx.x;
    const int lane = threadIdx.x;
    const u64 ltmask = (1ull << lane) - 1ull;
    if (st.done[r]) return;
    const int64_t ts = st.tape_cap;                  // the tape's rows per replica (replica-major)
    uint32_t* g = st.mt + r * MT_N;
    for (int k = lane; k < MT_N; k += 64) buf[k] = ld_nc(g + k);
    int idx = st.mt_idx[r];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint64_t rng = (uint64_t)(n - 1);
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    auto twist_if_end = [&]() {
        if (idx >= MT_N) {
            lds_twist(buf, lane);
            idx = 0;
        }
    };
    int64_t k = 0;
    if (rng == 0) {
        // n = 1: randint(0, 1) draws nothing; rand() two words a proposal
        for (; k < K; ++k) {
            twist_if_end();
            const uint32_t w1 = mt_temper(buf[idx++]);
            twist_if_end();
            const uint32_t w2 = mt_temper(buf[idx++]);
            if (lane == 0) {
                tape_i[r * ts + k] = 0;
                tape_u[r * ts + k] = mt_double(w1, w2);
            }
        }
    }
    while (k < K) {
        twist_if_end();
        const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
        uint32_t tw = 0, y = 0;
        bool ok = false;
        if (lane < lim) {
            tw = mt_temper(buf[idx + lane]);
            y = tw & mask;
            ok = y <= (uint32_t)rng;
        }
        const u64 okm = __ballot(ok);
        // the proposal starts whose rand() words fit the window, at most K - k of them
        u64 stm = mt_window_starts(ok) & ((lim >= 2) ? ((1ull << (lim - 2)) - 1ull) : 0ull);
        while ((int64_t)__popcll(stm) > K - k) stm &= ~(1ull << (63 - __clzll(stm)));
        const int64_t got = __popcll(stm);
        const int pos = got ? 66 - __clzll(stm) : 0;          // after the last start's two words
        if (got > 0) {
            const uint32_t x1 = mt_next_lane(tw);
            const uint32_t x2 = mt_next_lane(x1);
            if ((stm >> lane) & 1ull) {
                const int64_t j = k + __popcll(stm & ltmask);
                tape_i[r * ts + j] = (int32_t)y;
                tape_u[r * ts + j] = mt_double(x1, x2);
            }
            k += got;
            idx += pos;
            continue;
        }
        if (!okm) { idx += lim; continue; }
        const int f = __ffsll((unsigned long long)okm) - 1;
        if (f > 0) { idx += f; continue; }
        // i is the window's first word and rand()'s two words cross the end of
        // the state: the serial draw twists between them
        const int32_t iv = __builtin_amdgcn_readlane((int)y, 0);
        idx += 1;
        twist_if_end();
        const uint32_t w1 = mt_temper(buf[idx++]);
        twist_if_end();
        const uint32_t w2 = mt_temper(buf[idx++]);
        if (lane == 0) {
            tape_i[r * ts + k] = iv;
            tape_u[r * ts + k] = mt_double(w1, w2);
        }
        ++k;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int q = lane; q < MT_N; q += 64) g[q] = buf[q];
    if (lane == 0) st.mt_idx[r] = idx;
}

// Philox-4x32-10 (Salmon et al., SC'11; Random123's philox4x32_10): the
// NON-parity proposal stream (mjx_sa_state.philox_key).  Ten
// rounds of two 32x32->64 multiplies, the key bumped by the Weyl constants
// between rounds; oracle/orc_majority.c's orc_philox4x32_10 is the checker.
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t (&x)[4]) {
#pragma unroll
    for (int q = 0; q < 10; ++q) {
        if (q > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    x[0] = c0; x[1] = c1; x[2] = c2; x[3] = c3;
}

// the Philox tape: entry (k, r) = the proposal of step t_r + k of replica r
// (counter (t lo, t hi, 0, 0), key = philox_key[r]): i = the high 64 bits of
// (x0 | x1 << 32) * n, u = numpy rand()'s 53-bit double of (x2, x3).  One
// thread an entry, replica-major: entry (k, r) at r * tape_cap + k (the
// layout include/mjx.h documents; replica r's proposals contiguous), no state
// to carry (the step count is the counter).
__global__ void __launch_bounds__(256) k_sa_tape_philox(int64_t n, int64_t R, int64_t K, mjx_sa_state st,
                                                        int32_t* __restrict__ tape_i, double* __restrict__ tape_u) {
    const int64_t total = K * R, ts = st.tape_cap;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / K, k = e - r * K;
        if (st.done[r]) continue;
        const uint64_t t = (uint64_t)(st.t[r] + k), key = st.philox_key[r];
        uint32_t x[4];
        philox4x32_10((uint32_t)t, (uint32_t)(t >> 32), 0u, 0u, (uint32_t)key, (uint32_t)(key >> 32), x);
        const uint64_t w = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
        tape_i[r * ts + k] = (int32_t)__umul64hi(w, (uint64_t)n);
        tape_u[r * ts + k] = mt_double(x[2], x[3]);
    }
}

template <int D, bool TAPE>
__global__ void __launch_bounds__(64) k_sa_lightcone(const int32_t* __restrict__ adj, int d, int64_t n, int64_t R,
                                                     int64_t W, LcLevels L, int T, mjx_sa_state st, int64_t nsteps,
                                                     double par_a, double par_b, double a_cap, double b_cap,
                                                     int64_t t_cap, const int32_t* __restrict__ tape_i,
                                                     const double* __restrict__ tape_u, int split,
                                                     const int32_t* __restrict__ rep_graph) {
    extern __shared__ uint32_t lc_lists[];
    __shared__ uint32_t twist_buf[MT_N];
    // `split` waves share one 64-replica word column, each taking 64/split
    // replicas (the rest of its lanes idle): the step is bound by one wave's
    // latency, so more, thinner waves carry more replicas per unit of time
    const int lane = threadIdx.x;
    const int per = 64 / split;
    const int64_t col = blockIdx.x % W;                       // a column's waves on one XCD when W % 8 == 0
    const int rl = (int)(blockIdx.x / W) * per + lane;        // bit of this lane's replica in the column
    const int64_t r = col * 64 + rl;
    const bool live = lane < per && r < R;
    const u64 bit = 1ull << (rl & 63);
    const int64_t NS = L.ns, colo = col * L.cs;     // level word addressing (separate arrays or cone)
    if (rep_graph && live) adj += (int64_t)rep_graph[r] * n * d;   // this replica's graph of the stack
    uint32_t* lists = lc_lists + lane;
    WaveMT g{st.mt, twist_buf, r, live ? st.mt_idx[r] : MT_N, lane};
    double a = live ? st.a[r] : 0.0, b = live ? st.b[r] : 0.0;
    int64_t t = live ? st.t[r] : 0, sum_end = live ? st.sum_end[r] : 0;
    int done = live ? st.done[r] : 1;
    int ties = 0;
    const uint64_t rng = (uint64_t)(n - 1);
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    // tape mode: proposals k+1 and k+2 are held in registers while step k runs
    // (tape rows come three steps ahead); with the batched evaluation the
    // adjacency rows of i_{k+1}'s neighbours and of i_{k+2} are loaded during
    // step k, so a step starts with its level-1 word batch
    constexpr int DD = (D > 0) ? D : 1;
    const bool pre = TAPE && D > 0 && L.tab >= 0 && live && done == 0;   // tape rows valid for this launch
    int32_t nx_i = 0, n1i = 0, n2i = 0;
    double nx_u = 0.0, n1u = 0.0, n2u = 0.0;
    int32_t A0[DD], A1[DD][DD], B0[DD];        // rows of i_k, of N(i_k), of i_{k+1}
    auto row = [&](int32_t v, int32_t (&o)[DD]) {
        const int64_t base = (int64_t)((uint32_t)v < (uint32_t)n ? v : 0) * DD;   // never out of bounds
#pragma unroll
        for (int m = 0; m < DD; ++m) o[m] = adj[base + m];
    };
    if constexpr (TAPE) {
        if (live && nsteps > 0) { nx_i = tape_i[r * st.tape_cap]; nx_u = tape_u[r * st.tape_cap]; }
        if (live && nsteps > 1) { n1i = tape_i[r * st.tape_cap + 1]; n1u = tape_u[r * st.tape_cap + 1]; }
        if (live && nsteps > 2) { n2i = tape_i[r * st.tape_cap + 2]; n2u = tape_u[r * st.tape_cap + 2]; }
        if (pre) {
            row(nx_i, A0);
#pragma unroll
            for (int m = 0; m < DD; ++m) row(A0[m], A1[m]);
            if (nsteps > 1) row(n1i, B0);
        }
    }
    for (int64_t step = 0; step < nsteps; ++step) {
        const bool active = live && done == 0;
        uint32_t i = 0;
        double u = 0.0;
        int32_t A1n[DD][DD], B0n[DD];
        if constexpr (TAPE) {
            i = (uint32_t)nx_i;
            u = nx_u;
            if (pre) {
                if (step + 1 < nsteps) {
#pragma unroll
                    for (int m = 0; m < DD; ++m) row(B0[m], A1n[m]);
                }
                if (step + 2 < nsteps) row(n2i, B0n);
            }
            nx_i = n1i; nx_u = n1u;
            n1i = n2i; n1u = n2u;
            if (live && step + 3 < nsteps) {
                n2i = tape_i[r * st.tape_cap + step + 3];
                n2u = tape_u[r * st.tape_cap + step + 3];
            }
        } else {
            // randint(low=0, high=n) (code/SA_RRG.py:73): numpy legacy masked rejection
            bool pending = active && rng > 0;
            while (__ballot(pending)) {
                const uint32_t y = g.draw(pending);
                if (pending) {
                    const uint32_t v = y & mask;
                    if (v <= (uint32_t)rng) { i = v; pending = false; }
                }
            }
            // rand() (code/SA_RRG.py:76)
            const uint32_t w1 = g.draw(active);
            const uint32_t w2 = g.draw(active);
            u = mt_double(w1, w2);
        }
        if (active) {
            int cnt[LC_MAXT + 1];
            int old_i = 0;
            int64_t ds = 0;
            if constexpr (D > 0) {
                // the prefetched entries assume i and its D neighbours are distinct
                // (a simple graph); a row with a loop or a repeated neighbour
                // takes the path that deduplicates through the table
                bool simple = true;
#pragma unroll
                for (int m = 0; m < DD; ++m) {
                    simple &= A0[m] != (int32_t)i;
#pragma unroll
                    for (int q = m + 1; q < DD; ++q) simple &= A0[m] != A0[q];
                }
                bool done_tree = false;
                if constexpr (D <= 4) {
                    if (pre && simple && T <= 2)
                        done_tree = lc_tree2<D>(adj, NS, colo, bit, T, L, lists, (int32_t)i, cnt, &old_i, A0, A1, ds);
                }
                if (done_tree) {
                } else if (pre && simple)
                    ds = lc_delta_mlp<D, true>(adj, NS, colo, bit, T, L, lists, (int32_t)i, cnt, &old_i, A0, A1);
                else if (L.tab >= 0)
                    ds = lc_delta_mlp<D, false>(adj, NS, colo, bit, T, L, lists, (int32_t)i, cnt, &old_i, A0, A1);
                else ds = lc_delta<D>(adj, d, NS, colo, bit, T, L, lists, (int32_t)i, cnt, &old_i);
            } else {
                ds = lc_delta<D>(adj, d, NS, colo, bit, T, L, lists, (int32_t)i, cnt, &old_i);
            }
            const int64_t sum_new = sum_end + ds;
            // delta_H (code/SA_RRG.py:37), same operation order, no contraction
            const double si = old_i ? 1.0 : -1.0;
            const double t1 = (-2.0 * a) * si;
            const double t2 = b * (double)(sum_end - sum_new);
            const double dE = (t1 + t2) / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;                 // (code/SA_RRG.py:75)
            const bool acc = u < prob;                               // (code/SA_RRG.py:76)
            if (e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e)) ++ties;
            if (acc) {                                               // (code/SA_RRG.py:77)
                for (int lv = 0; lv <= T; ++lv) {
                    const uint32_t* lst = lists + L.off[lv] * 64;
                    for (int q = 0; q < cnt[lv]; ++q) {
                        const int64_t j = (int64_t)(lst[q * 64] & 0x7fffffffu);
                        atomicXor((unsigned long long*)(L.s[lv] + j * NS + colo), (unsigned long long)bit);
                        if (lv == 0 && L.s0c)
                            atomicXor((unsigned long long*)(L.s0c + j * W + col), (unsigned long long)bit);
                    }
                }
                sum_end = sum_new;
            }
            if (a < a_cap) a = par_a * a;                            // (code/SA_RRG.py:80-81)
            if (b < b_cap) b = par_b * b;
            t += 1;                                                  // (code/SA_RRG.py:82)
            if (t > t_cap) done = 2;                                 // (code/SA_RRG.py:84)
            else if (sum_end == n) done = 1;                         // m(s_endstate(s)) == 1
            if (st.tr_i) st.tr_i[step * R + r] = (int32_t)i;
            if (st.tr_acc) st.tr_acc[step * R + r] = acc ? 1 : 0;
            if (st.tr_sum) st.tr_sum[step * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[step * R + r] = dE;
        } else if (live) {
            if (st.tr_i) st.tr_i[step * R + r] = -1;
            if (st.tr_acc) st.tr_acc[step * R + r] = -1;
            if (st.tr_sum) st.tr_sum[step * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[step * R + r] = 0.0;
        }
        // this wave's flips must land before its next reads of the same words
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (TAPE) {
            if (pre) {       // rotate the prefetched rows
#pragma unroll
                for (int m = 0; m < DD; ++m) {
                    A0[m] = B0[m];
                    B0[m] = B0n[m];
#pragma unroll
                    for (int q = 0; q < DD; ++q) A1[m][q] = A1n[m][q];
                }
            }
        }
    }
    if (live) {
        if constexpr (!TAPE) st.mt_idx[r] = g.idx;
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}

// list slots per lane: levels 0..T (ball bounds) + candidate list; with
// `table` also the ball table of lc_delta_mlp (node ids, rows, candidates)
// ---------------------------------------------------------------------------
// Light-cone step on the cone layout with one memory round trip per proposal
// (p+c-1 = 2, d = 3 and the proposal tape).  Adjacency rows are fetched in a
// pipeline down the tape -- at step k the row of i_{k+3}, the rows of the
// neighbours of i_{k+2} and the rows of the children of i_{k+1} -- so when step
// k starts every node of i_k's radius-3 tree is known, and ONE batch loads the
// level sectors (s_0, s_1, s_2) of i, its neighbours a_m and their children and
// the level-1 words of the grandchildren.  The evaluation is lc_tree2's with
// every value in a register, the change sets are bit masks over the tree's
// positions (flips straight from registers, no lists), and balls that are not
// trees fall back to lc_delta_mlp (lists in LDS).  Same accept sequence.
// ---------------------------------------------------------------------------
// Cone-word loads of the one-trip and speculative kernels: sc1 loads (served
// by L2, around the CU's vector L1) through a buffer descriptor over the wave's
// word-column slab.  A lane re-reads words that its own atomicXor flips have
// just changed; global atomics are performed in L2, and the gfx950 memory model
// gives no rule by which a line already held in this CU's L1 would see them, so
// plain (L1-cacheable) loads could return the lane's own bit stale.  sc1 loads
// cost 0-3 % against plain ones at 16 B (MI355X_MICROARCH.md, visibility
// table); the general kernels use agent-scope atomic loads (ld_word), the same
// sc1 instruction at 8 B.  The slab base is wave-uniform (the column comes from
// blockIdx), so the descriptor lives in SGPRs; offsets are 32-bit (the host
// checks n*LV*8 < 2^31).
typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));
typedef unsigned int v2u32_t __attribute__((ext_vector_type(2)));
constexpr int kSc1 = 16;        // buffer cache-policy bits: sc1

struct ConeRd {
    __amdgpu_buffer_rsrc_t rs;
    // the inputs are wave-uniform; readfirstlane makes that provable, so the
    // descriptor sits in SGPRs (no waterfall loop around each load)
    __device__ __forceinline__ static __amdgpu_buffer_rsrc_t make(const u64* slab, int64_t bytes) {
        const uint64_t a = (uint64_t)(uintptr_t)slab;
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
        const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
        return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0, nb,
                                                 0x00020000);
    }
    __device__ __forceinline__ ConeRd(const u64* slab, int64_t bytes) : rs(make(slab, bytes)) {}
    __device__ __forceinline__ u64 word(uint32_t idx) const {          // idx in 8-B words
        const v2u32_t x = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(idx * 8u), 0, kSc1);
        return (u64)x.x | ((u64)x.y << 32);
    }
    __device__ __forceinline__ void pair(uint32_t idx, u64& a, u64& b) const {   // 16-B aligned pair
        const v4u32_t x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(idx * 8u), 0, kSc1);
        a = (u64)x.x | ((u64)x.y << 32);
        b = (u64)x.z | ((u64)x.w << 32);
    }
    __device__ __forceinline__ int4 row(uint32_t idx) const {                    // 16-B adjacency row of a record
        const v4u32_t x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(idx * 8u), 0, kSc1);
        return make_int4((int)x.x, (int)x.y, (int)x.z, (int)x.w);
    }
    __device__ __forceinline__ uint32_t u32(uint32_t idx, uint32_t byte) const {  // 4 B at a byte offset of a record
        return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(idx * 8u + byte), 0, kSc1);
    }
};

// The neighbour words of a d = 3, p+c-1 = 2 record (64 B: row in bytes 0..11,
// levels 0..2 in bytes 16..39): level 1 of the node's three neighbours, 3 bits
// per replica of the column -- replica q's bits (neighbour y = 0..2 of the row)
// at bit 3*(q % 10) + y of the 32-bit word q / 10, words 0..5 in bytes 40..63
// and word 6 in the row's pad (bytes 12..15).  The speculative batch reads a
// child's record whole and so has its children's level-1 values with its own
// (no round trip of their own after level 1); every level-1 flip of a node
// XORs its bit into the records of its neighbours.
__host__ __device__ inline uint32_t nb_byte(int q) { return (q / 10 < 6) ? 40u + 4u * (uint32_t)(q / 10) : 12u; }
__host__ __device__ inline int nb_shift(int q) { return 3 * (q % 10); }
__device__ inline uint32_t nb_pack(const u64 (&L)[3], int j) {     // word j from the neighbours' level-1 words
    uint32_t x = 0;
    for (int qq = 0; qq < 10 && 10 * j + qq < 64; ++qq)
        for (int y = 0; y < 3; ++y) x |= (uint32_t)((L[y] >> (10 * j + qq)) & 1ull) << (3 * qq + y);
    return x;
}

// the neighbour words of every d = 3, p+c-1 = 2 record, from the records' own
// rows and level-1 words (after steps that did not keep them: every kernel but
// the speculative one)
__global__ void __launch_bounds__(kBlock) k_rec_nb_fill(u64* __restrict__ rec, int64_t n, int64_t W) {
    for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < n * W; w += (int64_t)gridDim.x * kBlock) {
        const int64_t col = w / n;                       // (record order: column-major)
        u64* dst = rec + w * 8;
        const int4 r = *reinterpret_cast<const int4*>(dst);
        const int32_t nbr[3] = {r.x, r.y, r.z};
        u64 L[3];
        for (int y = 0; y < 3; ++y) L[y] = rec[(col * n + nbr[y]) * 8 + 3];
        uint32_t nb[7];
        for (int j = 0; j < 7; ++j) nb[j] = nb_pack(L, j);
        reinterpret_cast<int32_t*>(dst)[3] = (int32_t)nb[6];
        dst[5] = (u64)nb[0] | ((u64)nb[1] << 32);
        dst[6] = (u64)nb[2] | ((u64)nb[3] << 32);
        dst[7] = (u64)nb[4] | ((u64)nb[5] << 32);
    }
}

template <int D>
__global__ void __launch_bounds__(64) k_sa_cone2(const int32_t* __restrict__ adj, const int4* __restrict__ adj_pad,
                                                 int64_t n, int64_t R, int64_t W,
                                                 LcLevels L, mjx_sa_state st, int64_t nsteps, double par_a,
                                                 double par_b, double a_cap, double b_cap, int64_t t_cap,
                                                 const int32_t* __restrict__ tape_i,
                                                 const double* __restrict__ tape_u, int split,
                                                 const int32_t* __restrict__ rep_graph) {
    extern __shared__ uint32_t lc_lists[];
    constexpr int T = 2;
    const int lane = threadIdx.x;
    const int per = 64 / split;
    const int64_t col = blockIdx.x % W;                       // a column's waves on one XCD when W % 8 == 0
    const int rl = (int)(blockIdx.x / W) * per + lane;
    const int64_t r = col * 64 + rl;
    const bool live = lane < per && r < R;
    const u64 bit = 1ull << (rl & 63);
    const int64_t NS = L.ns, colo = col * L.cs;
    const u64* cone = L.s[0];                                 // level t of (v, col) at cone + v*NS + colo + t
    uint32_t* lists = lc_lists + lane;
    double a = live ? st.a[r] : 0.0, b = live ? st.b[r] : 0.0;
    int64_t t = live ? st.t[r] : 0, sum_end = live ? st.sum_end[r] : 0;
    int done = live ? st.done[r] : 1;
    int ties = 0;
    const bool run = live && done == 0;
    static_assert(D == 3, "rows are read as one 16-B load from the padded adjacency");
    if (rep_graph && live) {                                  // this replica's graph of the stack
        const int64_t g = rep_graph[r];
        adj += g * n * D;
        adj_pad += g * n;
    }
    auto row = [&](int32_t v, int32_t (&o)[D]) {
        const int4 q = adj_pad[(uint32_t)v < (uint32_t)n ? v : 0];             // never out of bounds
        o[0] = q.x; o[1] = q.y; o[2] = q.z;
    };
    auto tape = [&](int64_t k, int32_t& iv, double& uv) {
        iv = 0; uv = 0.0;
        if (run && k < nsteps) { iv = tape_i[r * st.tape_cap + k]; uv = tape_u[r * st.tape_cap + k]; }
    };
    // pipeline registers: tape (i, u) of k+1..k+3; row of i_{k+1}, i_{k+2};
    // rows of N(i_{k+1}); current rows of i_k, N(i_k), children of i_k
    int32_t ti1, ti2, ti3, ti0;
    double tu1, tu2, tu3, tu0;
    int32_t Q1[D], Q2[D], N1[D][D], A0[D], A1[D][D], C[D][D][D];
    tape(0, ti0, tu0); tape(1, ti1, tu1); tape(2, ti2, tu2); tape(3, ti3, tu3);
    row(ti0, A0); row(ti1, Q1); row(ti2, Q2);
#pragma unroll
    for (int m = 0; m < D; ++m) { row(A0[m], A1[m]); row(Q1[m], N1[m]); }
#pragma unroll
    for (int m = 0; m < D; ++m)
#pragma unroll
        for (int x = 0; x < D; ++x) row(A1[m][x], C[m][x]);
    // sc1 loads (ConeRd): a lane's own bit of a word changes only by its own
    // atomics; other lanes' bits may be stale and are never used
    const ConeRd crd(cone + colo, n * NS * 8);
    auto w = [&](int32_t v, int lv) { return crd.word((uint32_t)v * (uint32_t)NS + (uint32_t)lv); };
    auto sector = [&](int32_t v, u64 (&o)[3]) {
        const uint32_t q = (uint32_t)v * (uint32_t)NS;
        crd.pair(q, o[0], o[1]);
        o[2] = crd.word(q + 2);
    };
    auto bv = [&](u64 x) -> uint32_t { return (x & bit) ? 1u : 0u; };
    auto maj = [&](int ones, uint32_t own) -> uint32_t { return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own); };
    for (int64_t step = 0; step < nsteps; ++step) {
        const bool active = run && done == 0;
        const int32_t i = ti0;
        const double u = tu0;
        // prefetch stage: tape k+4, row of i_{k+3}, rows of N(i_{k+2}), rows of the children of i_{k+1}
        int32_t ti4; double tu4;
        tape(step + 4, ti4, tu4);
        int32_t Q3[D], N2[D][D], Cn[D][D][D];
        row(ti3, Q3);
#pragma unroll
        for (int m = 0; m < D; ++m) row(Q2[m], N2[m]);
#pragma unroll
        for (int m = 0; m < D; ++m)
#pragma unroll
            for (int x = 0; x < D; ++x) row(N1[m][x], Cn[m][x]);
        if (active) {
            // the tree shape (lc_tree2): i, the a_m and their children all distinct
            bool ok = true;
#pragma unroll
            for (int m = 0; m < D; ++m) {
                int ci = 0;
#pragma unroll
                for (int x = 0; x < D; ++x) ci += (A1[m][x] == i);
                ok &= (ci == 1) && (A0[m] != i);
#pragma unroll
                for (int m2 = m + 1; m2 < D; ++m2) ok &= A0[m] != A0[m2];
            }
#pragma unroll
            for (int m = 0; m < D; ++m)
#pragma unroll
                for (int x = 0; x < D; ++x) {
                    const int32_t cc = A1[m][x];
                    if (cc == i) continue;
#pragma unroll
                    for (int m2 = 0; m2 < D; ++m2) ok &= (cc != A0[m2]);
#pragma unroll
                    for (int m2 = m; m2 < D; ++m2)
#pragma unroll
                        for (int x2 = 0; x2 < D; ++x2)
                            if (m2 > m || x2 > x) ok &= (A1[m2][x2] == i) || (A1[m2][x2] != cc);
                }
            int old_i = 0;
            int64_t ds = 0;
            uint32_t ch1 = 0, nv1 = 0, ch2 = 0;                 // positions: 0 = i, 1+m = a_m, 1+D+m*D+x = child
            if (ok) {
                // the one batch: sectors of i, a_m, children; level-1 words of the grandchildren
                u64 wi[3], wa[D][3], wc[D][D][3], wg[D][D][D];
                sector(i, wi);
#pragma unroll
                for (int m = 0; m < D; ++m) {
                    sector(A0[m], wa[m]);
#pragma unroll
                    for (int x = 0; x < D; ++x) {
                        const bool child = A1[m][x] != i;
                        wc[m][x][0] = wc[m][x][1] = wc[m][x][2] = 0ull;
                        if (child) sector(A1[m][x], wc[m][x]);
#pragma unroll
                        for (int y = 0; y < D; ++y)
                            wg[m][x][y] = (child && C[m][x][y] != A0[m]) ? w(C[m][x][y], 1) : 0ull;
                    }
                }
                // level 1 (lc_tree2)
                const uint32_t f = bv(wi[0]) ^ 1u;
                old_i = (int)bv(wi[0]);
                {
                    int ones = 0;
#pragma unroll
                    for (int m = 0; m < D; ++m) ones += (int)bv(wa[m][0]);
                    const uint32_t nb = maj(ones, f);
                    if (nb != bv(wi[1])) { ch1 |= 1u; nv1 |= nb; }
                }
#pragma unroll
                for (int m = 0; m < D; ++m) {
                    int ones = 0;
#pragma unroll
                    for (int x = 0; x < D; ++x) ones += (int)((A1[m][x] == i) ? f : bv(wc[m][x][0]));
                    const uint32_t nb = maj(ones, bv(wa[m][0]));
                    if (nb != bv(wa[m][1])) { ch1 |= 2u << m; nv1 |= nb << (1 + m); }
                }
                // level 2
                const bool c0 = ch1 & 1u;
                const uint32_t vi1 = c0 ? (nv1 & 1u) : bv(wi[1]);
                int64_t acc = 0;
                if (ch1 != 0) {
                    int ones = 0;
#pragma unroll
                    for (int m = 0; m < D; ++m) ones += (int)(((ch1 >> (1 + m)) & 1u) ? ((nv1 >> (1 + m)) & 1u) : bv(wa[m][1]));
                    const uint32_t nb = maj(ones, vi1);
                    if (nb != bv(wi[2])) { ch2 |= 1u; acc += nb ? 2 : -2; }
                }
#pragma unroll
                for (int m = 0; m < D; ++m) {
                    const bool cm = (ch1 >> (1 + m)) & 1u;
                    const uint32_t va1 = cm ? ((nv1 >> (1 + m)) & 1u) : bv(wa[m][1]);
                    if (c0 || cm) {
                        int ones = 0;
#pragma unroll
                        for (int x = 0; x < D; ++x) ones += (int)((A1[m][x] == i) ? vi1 : bv(wc[m][x][1]));
                        const uint32_t nb = maj(ones, va1);
                        if (nb != bv(wa[m][2])) { ch2 |= 2u << m; acc += nb ? 2 : -2; }
                    }
                    if (cm) {
#pragma unroll
                        for (int x = 0; x < D; ++x) {
                            if (A1[m][x] == i) continue;
                            int ones = 0;
#pragma unroll
                            for (int y = 0; y < D; ++y) ones += (int)((C[m][x][y] == A0[m]) ? va1 : bv(wg[m][x][y]));
                            const uint32_t nb = maj(ones, bv(wc[m][x][1]));
                            if (nb != bv(wc[m][x][2])) { ch2 |= 1u << (1 + D + m * D + x); acc += nb ? 2 : -2; }
                        }
                    }
                }
                ds = acc;
            } else {
                // not a tree: the batched table path (lc_delta_mlp), rows of i and
                // its neighbours taken from the pipeline when they are distinct
                bool simple = true;
#pragma unroll
                for (int m = 0; m < D; ++m) {
                    simple &= A0[m] != i;
#pragma unroll
                    for (int q = m + 1; q < D; ++q) simple &= A0[m] != A0[q];
                }
                int cnt[LC_MAXT + 1];
                if (simple) ds = lc_delta_mlp<D, true>(adj, NS, colo, bit, T, L, lists, i, cnt, &old_i, A0, A1);
                else ds = lc_delta_mlp<D, false>(adj, NS, colo, bit, T, L, lists, i, cnt, &old_i, A0, A1);
                ch1 = (uint32_t)cnt[1] | ((uint32_t)cnt[2] << 8) | 0x80000000u;   // list path marker
            }
            const int64_t sum_new = sum_end + ds;
            // delta_H (code/SA_RRG.py:37), same operation order, no contraction
            const double si = old_i ? 1.0 : -1.0;
            const double t1 = (-2.0 * a) * si;
            const double t2 = b * (double)(sum_end - sum_new);
            const double dE = (t1 + t2) / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;                 // (code/SA_RRG.py:75)
            const bool acc = u < prob;                               // (code/SA_RRG.py:76)
            if (e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e)) ++ties;
            if (acc) {                                               // (code/SA_RRG.py:77)
                auto flip = [&](int32_t v, int lv) {
                    atomicXor((unsigned long long*)(cone + (int64_t)v * NS + colo + lv), (unsigned long long)bit);
                };
                flip(i, 0);
                atomicXor((unsigned long long*)(L.s0c + (int64_t)i * W + col), (unsigned long long)bit);
                if (ch1 & 0x80000000u) {
                    const int c1 = (int)(ch1 & 0xffu), c2 = (int)((ch1 >> 8) & 0xffu);
                    for (int q = 0; q < c1; ++q) flip((int32_t)(lists[(L.off[1] + q) * 64] & 0x7fffffffu), 1);
                    for (int q = 0; q < c2; ++q) flip((int32_t)(lists[(L.off[2] + q) * 64] & 0x7fffffffu), 2);
                } else {
                    if (ch1 & 1u) flip(i, 1);
                    if (ch2 & 1u) flip(i, 2);
#pragma unroll
                    for (int m = 0; m < D; ++m) {
                        if ((ch1 >> (1 + m)) & 1u) flip(A0[m], 1);
                        if ((ch2 >> (1 + m)) & 1u) flip(A0[m], 2);
#pragma unroll
                        for (int x = 0; x < D; ++x)
                            if ((ch2 >> (1 + D + m * D + x)) & 1u) flip(A1[m][x], 2);
                    }
                }
                sum_end = sum_new;
            }
            if (a < a_cap) a = par_a * a;                            // (code/SA_RRG.py:80-81)
            if (b < b_cap) b = par_b * b;
            t += 1;                                                  // (code/SA_RRG.py:82)
            if (t > t_cap) done = 2;                                 // (code/SA_RRG.py:84)
            else if (sum_end == n) done = 1;                         // m(s_endstate(s)) == 1
            if (st.tr_i) st.tr_i[step * R + r] = i;
            if (st.tr_acc) st.tr_acc[step * R + r] = acc ? 1 : 0;
            if (st.tr_sum) st.tr_sum[step * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[step * R + r] = dE;
        } else if (live) {
            if (st.tr_i) st.tr_i[step * R + r] = -1;
            if (st.tr_acc) st.tr_acc[step * R + r] = -1;
            if (st.tr_sum) st.tr_sum[step * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[step * R + r] = 0.0;
        }
        // this wave's flips must land before its next reads of the same words
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // rotate the pipeline
        ti0 = ti1; tu0 = tu1; ti1 = ti2; tu1 = tu2; ti2 = ti3; tu2 = tu3; ti3 = ti4; tu3 = tu4;
#pragma unroll
        for (int m = 0; m < D; ++m) {
            A0[m] = Q1[m]; Q1[m] = Q2[m]; Q2[m] = Q3[m];
#pragma unroll
            for (int x = 0; x < D; ++x) {
                A1[m][x] = N1[m][x]; N1[m][x] = N2[m][x];
#pragma unroll
                for (int y = 0; y < D; ++y) C[m][x][y] = Cn[m][x][y];
            }
        }
    }
    if (live) {
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}

// ---------------------------------------------------------------------------
// Speculative batches (cone layout, proposal tape; d = 3 at p+c-1 <= 2, d = 4 at
// p+c-1 = 1): the K = 8 or 16 lanes of a lane group evaluate the next K
// proposals of ONE replica at once,
// all against the current configuration, and the batch is then resolved in
// proposal order.  Proposal j's evaluation reads the words of the nodes R_j of
// its radius-3 tree; it is the one a sequential run computes unless an earlier
// proposal of the batch may write one of those nodes, so every proposal's
// potential writes W_k (i and the positions whose level values it changes) go
// into a per-replica LDS filter, and j stands only while no node of R_j may be
// in an earlier W_k (a ball that is not a tree stands only as the first of a
// batch).  The filter is conservative, never exact-or-nothing: two tables of
// K-bit proposal masks, slot h1(v) of one and h2(v) of the other, both get
// proposal k's bit for every v of W_k (a non-returning LDS OR); node v of R_j
// is taken as written by an earlier proposal when the two slots' masks share a
// bit below j.  A node that is written is always found; a node that is not is
// found only when other keys of one earlier proposal cover both of its slots
// (h1, h2 together are the node's low 22 bits: ~|W_k|^2 / 2048^2), and such a
// false conflict only ends the batch early -- the proposals after it are
// evaluated again against the updated state, as after a real one.  (Round 6;
// before, an exact hash set of (node, min tag) keys: CAS inserts, probe loops
// on collisions, 20 % of the step and most of a launch's tail.)  The batch consumes the proposals before the
// first that does not stand and ends after the first that finishes the replica;
// the rest are drawn again as the next batch.  Acceptance needs no ordering
// (the schedule a, b depends on the step count only; delta_H on the proposal's
// own change), the stop needs a prefix sum of the accepted changes.  Two random
// proposals on a 1e6-node graph collide with probability ~1e-4, so batches
// almost always consume all K: the replica's serial chain moves K proposals per
// batch of round trips instead of one.  Same accept sequence as the serial step.
// (Two-hop adjacency records -- a node's row and its neighbours' rows in one
// line -- measured no faster: the 16 MB adjacency is served on-die.)
// ---------------------------------------------------------------------------
constexpr int SPEC_FS = 2048;          // filter slots per table per replica (two tables)
constexpr int SPEC_LDS = 64 * 2 * SPEC_FS / 8;   // bytes of filters per wave: 64/K replicas, K-bit slots

// Diagnostic build only (-DMJX_SA_PROF, tools/sa_prof.py): per-phase s_memtime
// cycles of k_sa_spec summed over waves; every stamp drains the wave's memory
// counters first, so a phase's exposed latency is charged to that phase.
#ifdef MJX_SA_PROF
__device__ unsigned long long mjx_sa_prof[8];
#define SA_STAMP(k) do { __builtin_amdgcn_sched_barrier(0); asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); const unsigned long long _c = __builtin_amdgcn_s_memtime(); _acc[k] += _c - _t0; _t0 = _c; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define SA_STAMP(k) do {} while (0)
#endif
template <int D, int TT, int K, bool NB>
__global__ void __launch_bounds__(64) k_sa_spec(const int32_t* __restrict__ adj, const int4* __restrict__ adj_pad,
                                                int64_t n, int64_t R, int64_t W, LcLevels L, mjx_sa_state st,
                                                int64_t nsteps, double par_a, double par_b, double a_cap,
                                                double b_cap, int64_t t_cap, const int32_t* __restrict__ tape_i,
                                                const double* __restrict__ tape_u, int hoff,
                                                const int32_t* __restrict__ rep_graph) {
    // rows as one 16-B load: the padded adjacency (d = 3) or the adjacency itself (d = 4)
    static_assert((D == 3 && (TT == 1 || TT == 2)) || (D == 4 && TT == 1), "speculative batches: d=3 T<=2, d=4 T=1");
    extern __shared__ uint32_t lc_lists[];
    static_assert(K == 8 || K == 16, "8 or 16 proposals per batch");
    // NB: records with neighbour words (nb_byte): the children's level-1
    // neighbours come with their records, and level-1 flips keep them
    static_assert(!NB || (D == 3 && TT == 2), "neighbour words: d = 3, p+c-1 = 2 records");
    constexpr int T = TT;
    constexpr int SPW = 32 / K;                              // filter slots per 32-bit word
    constexpr int FTW = SPEC_FS / SPW;                       // words per filter table
    constexpr u64 GM = (1ull << K) - 1;
    // the step chain is latency-bound: its waves issue first on a SIMD they
    // share with the next chunk's tape waves (drawn on a side stream)
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x;
    const int g = lane / K, k = lane % K;
    const int64_t col = blockIdx.x % W;                       // a column's waves on one XCD when W % 8 == 0
    const int rl = (int)(blockIdx.x / W) * (64 / K) + g;
    const int64_t r = col * 64 + rl;
    const bool live = r < R;
    const u64 bit = 1ull << (rl & 63);
    // words per (node, column): the NB records are 8 (a shift, not a multiply)
    const int64_t NS = NB ? 8 : L.ns, colo = col * L.cs;
    const u64* cone = L.s[0];
    uint32_t* lists = lc_lists + lane;
    uint32_t* ftab = lc_lists + hoff + g * 2 * FTW;           // this replica's two tables
    if (rep_graph && live) {                                  // this replica's graph of the stack
        const int64_t gi = rep_graph[r];
        adj += gi * n * D;
        adj_pad += gi * n;
    }
    // replica state, identical in the group's 8 lanes
    double a = live ? st.a[r] : 0.0, b = live ? st.b[r] : 0.0;
    int64_t t = live ? st.t[r] : 0, sum_end = live ? st.sum_end[r] : 0;
    int done = live ? st.done[r] : 1;
    int64_t pos = 0;                                          // proposals of this launch consumed
    int ties = 0;
    // sc1 loads: see ConeRd; over the record base (= the level-0 words unless
    // the records carry the adjacency rows, L.lo = 2)
    const uint32_t lo = (uint32_t)L.lo;
    const ConeRd crd(cone - lo + colo, n * NS * 8);
    auto row = [&](int32_t v, int32_t (&o)[D]) {
        const uint32_t vv = (uint32_t)v < (uint32_t)n ? (uint32_t)v : 0u;     // never out of bounds
        const int4 q = lo ? crd.row(vv * (uint32_t)NS) : adj_pad[vv];
        o[0] = q.x; o[1] = q.y; o[2] = q.z;
        if constexpr (D == 4) o[3] = q.w;
    };
    auto w = [&](int32_t v, int lv) { return crd.word((uint32_t)v * (uint32_t)NS + lo + (uint32_t)lv); };
    auto sector = [&](int32_t v, u64 (&o)[3]) {      // levels 0..T of v
        const uint32_t q = (uint32_t)v * (uint32_t)NS + lo;
        crd.pair(q, o[0], o[1]);
        o[2] = (TT == 2) ? crd.word(q + 2) : 0ull;
    };
    auto bv = [&](u64 x) -> uint32_t { return (x & bit) ? 1u : 0u; };
    const uint32_t nbo = nb_byte(rl & 63);                   // this replica's neighbour word and bits
    const int nbs = nb_shift(rl & 63);
    // XOR bits (neighbour slots) into v's neighbour word (records only)
    auto nbx = [&](int32_t v, uint32_t slots) {
        atomicXor((uint32_t*)(cone - lo + colo + (int64_t)v * NS) + nbo / 4, slots << nbs);
    };
    auto maj = [&](int ones, uint32_t own) -> uint32_t { return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own); };
    // the two slots of v: its low 11 bits, and bits 11..21 (node ids of a
    // random graph are random; ids past 2^22 only alias, never miss)
    auto fslot1 = [](int32_t v) { return (uint32_t)v & (uint32_t)(SPEC_FS - 1); };
    auto fslot2 = [](int32_t v) { return ((uint32_t)v >> 11) & (uint32_t)(SPEC_FS - 1); };
    const uint32_t kbit = 1u << k;
    const uint32_t below = kbit - 1u;                        // the earlier proposals' bits
    auto fword = [&](int tbl, uint32_t h) -> uint32_t* { return ftab + tbl * FTW + h / SPW; };
    auto fshift = [](uint32_t h) -> uint32_t { return (h % SPW) * K; };
    // lookups read the K-bit slots themselves (ds_read_u8 / _u16: no shifts)
    using FS = typename std::conditional<(K == 8), uint8_t, uint16_t>::type;
    const FS* fs1 = reinterpret_cast<const FS*>(ftab);
    const FS* fs2 = fs1 + SPEC_FS;
    auto fins = [&](int32_t v) {                             // proposal k may write v
        const uint32_t h1 = fslot1(v), h2 = fslot2(v);
        atomicOr(fword(0, h1), kbit << fshift(h1));
        atomicOr(fword(1, h2), kbit << fshift(h2));
    };
    // N nodes at once, branch-free (masked-off entries OR zero / test nothing)
    auto fins_n = [&](const int32_t* vv, const bool* mm, auto nn) {
        constexpr int N = decltype(nn)::value;
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t h1 = fslot1(vv[q]), h2 = fslot2(vv[q]);
            const uint32_t kb = mm[q] ? kbit : 0u;
            atomicOr(fword(0, h1), kb << fshift(h1));
            atomicOr(fword(1, h2), kb << fshift(h2));
        }
    };
    auto fearlier_n = [&](const int32_t* vv, const bool* mm, auto nn) -> bool {
        constexpr int N = decltype(nn)::value;
        uint32_t e1[N], e2[N];
#pragma unroll
        for (int q = 0; q < N; ++q) {
            e1[q] = fs1[fslot1(vv[q])];
            e2[q] = fs2[fslot2(vv[q])];
        }
        uint32_t hit = 0;
#pragma unroll
        for (int q = 0; q < N; ++q) hit |= mm[q] ? (e1[q] & e2[q]) : 0u;
        return (hit & below) != 0u;
    };
#ifdef MJX_SA_PROF
    unsigned long long _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _t0 = __builtin_amdgcn_s_memtime();
#endif
    // The proposal tape and the adjacency do not depend on accept decisions, so
    // the next batch's proposals (pos + K + k: every proposal of this batch
    // consumed, the usual case) and the rows of their balls are fetched while
    // this batch evaluates and resolves: the tape entry at its start, the row of
    // i behind this batch's first loads, the rows of i's neighbours after the
    // evaluation (each lands under a later phase of this batch).
    // A batch that consumed fewer than K (a conflict, a non-tree ball, a stop)
    // fetches its own afresh.  Three dependent round trips per batch fewer.
    int64_t pf_pos = -1;
    int32_t pf_i = 0, pf_A0[D], pf_A1[D][D];
    double pf_u = 0.0;
#pragma unroll
    for (int m = 0; m < D; ++m) {
        pf_A0[m] = 0;
#pragma unroll
        for (int x = 0; x < D; ++x) pf_A1[m][x] = 0;
    }
    for (;;) {
        const bool going = live && done == 0 && pos < nsteps;
        if (!__any(going)) break;
        // empty filters (32 KB per wave, 16-B stores); lanes then insert into
        // and read slots other lanes wrote: wave-scope fences at each hand-off
        for (int q = lane; q < SPEC_LDS / 16; q += 64)
            reinterpret_cast<uint4*>(lc_lists + hoff)[q] = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        SA_STAMP(5);
        const int64_t kk = pos + k;
        const bool mine = going && kk < nsteps;
        const bool fresh = pf_pos != pos;                     // (the whole lane group alike)
        int32_t i = 0;
        double u = 0.0;
        int32_t A0[D], A1[D][D], C[D][D][D];
        if (fresh) {
            // rows of i and of its neighbours (two round trips); the rows of the
            // children only where level 2 needs them (below)
            if (mine) { i = tape_i[r * st.tape_cap + kk]; u = tape_u[r * st.tape_cap + kk]; }
            row(i, A0);
#pragma unroll
            for (int m = 0; m < D; ++m) row(A0[m], A1[m]);
        } else {
            i = mine ? pf_i : 0;
            u = pf_u;
#pragma unroll
            for (int m = 0; m < D; ++m) {
                A0[m] = pf_A0[m];
#pragma unroll
                for (int x = 0; x < D; ++x) A1[m][x] = pf_A1[m][x];
            }
        }
        // the next batch's tape entry (proposal pos + K + k)
        const int64_t nk = pos + K + k;
        const bool pf = going && nk < nsteps;
        int32_t n_i = 0;
        double n_u = 0.0;
        if (pf) { n_i = tape_i[r * st.tape_cap + nk]; n_u = tape_u[r * st.tape_cap + nk]; }
        // tree shape (lc_tree2)
        bool ok = true, simple = true;
#pragma unroll
        for (int m = 0; m < D; ++m) {
            int ci = 0;
#pragma unroll
            for (int x = 0; x < D; ++x) ci += (A1[m][x] == i);
            ok &= (ci == 1) && (A0[m] != i);
            simple &= A0[m] != i;
#pragma unroll
            for (int m2 = m + 1; m2 < D; ++m2) { ok &= A0[m] != A0[m2]; simple &= A0[m] != A0[m2]; }
        }
#pragma unroll
        for (int m = 0; m < D; ++m)
#pragma unroll
            for (int x = 0; x < D; ++x) {
                const int32_t cc = A1[m][x];
                if (cc == i) continue;
#pragma unroll
                for (int m2 = 0; m2 < D; ++m2) ok &= (cc != A0[m2]);
#pragma unroll
                for (int m2 = m; m2 < D; ++m2)
#pragma unroll
                    for (int x2 = 0; x2 < D; ++x2)
                        if (m2 > m || x2 > x) ok &= (A1[m2][x2] == i) || (A1[m2][x2] != cc);
            }
        SA_STAMP(0);
        int old_i = 0;
        int64_t ds = 0;
        uint32_t ch1 = 0, nv1 = 0, ch2 = 0;      // positions: 0 = i, 1+m = a_m, 1+D+m*D+x = child
        bool listpath = false;
        int cnt[LC_MAXT + 1] = {0, 0, 0, 0, 0, 0, 0};
        u64 wi[3], wa[D][3], wc[D][D][3], wg[D][D][D];
        uint32_t wn[D][D];                       // NB: the children's neighbour words
        const bool tree = mine && ok;
        if (tree) {
            // rows of the children (T = 2) and the level sectors of i, the a_m and
            // the children in one batch
            if constexpr (TT == 2) {
#pragma unroll
                for (int m = 0; m < D; ++m)
#pragma unroll
                    for (int x = 0; x < D; ++x)
                        if (A1[m][x] != i) row(A1[m][x], C[m][x]);
            }
            sector(i, wi);
#pragma unroll
            for (int m = 0; m < D; ++m) {
                sector(A0[m], wa[m]);
#pragma unroll
                for (int x = 0; x < D; ++x) {
                    wc[m][x][0] = wc[m][x][1] = wc[m][x][2] = 0ull;
                    wn[m][x] = 0u;
                    if (A1[m][x] != i) {
                        sector(A1[m][x], wc[m][x]);
                        if constexpr (NB) wn[m][x] = crd.u32((uint32_t)A1[m][x] * (uint32_t)NS, nbo);
                    }
                }
            }
        }
        // the next batch: the row of its i (its tape entry landed with this
        // batch's first loads), in flight while this batch evaluates
        int32_t n_A0[D], n_A1[D][D];
        __builtin_amdgcn_sched_barrier(0);
        row(n_i, n_A0);
        __builtin_amdgcn_sched_barrier(0);
        if (tree) {
            const uint32_t f = bv(wi[0]) ^ 1u;
            old_i = (int)bv(wi[0]);
            {
                int ones = 0;
#pragma unroll
                for (int m = 0; m < D; ++m) ones += (int)bv(wa[m][0]);
                const uint32_t nb = maj(ones, f);
                if (nb != bv(wi[1])) { ch1 |= 1u; nv1 |= nb; }
            }
#pragma unroll
            for (int m = 0; m < D; ++m) {
                int ones = 0;
#pragma unroll
                for (int x = 0; x < D; ++x) ones += (int)((A1[m][x] == i) ? f : bv(wc[m][x][0]));
                const uint32_t nb = maj(ones, bv(wa[m][0]));
                if (nb != bv(wa[m][1])) { ch1 |= 2u << m; nv1 |= nb << (1 + m); }
            }
            SA_STAMP(1);
            if constexpr (TT == 1) {
                // T = 1: the sum over the level-1 changes (lc_tree2)
                int64_t acc = 0;
#pragma unroll
                for (int e = 0; e <= D; ++e)
                    if ((ch1 >> e) & 1u) acc += ((nv1 >> e) & 1u) ? 2 : -2;
                ds = acc;
            } else {
            // the level-1 words of the children's other neighbours, only for the
            // branches level 2 re-evaluates (one more round trip; with NB they
            // came with the children's records)
            if constexpr (!NB) {
#pragma unroll
            for (int m = 0; m < D; ++m)
#pragma unroll
                for (int x = 0; x < D; ++x)
#pragma unroll
                    for (int y = 0; y < D; ++y)
                        wg[m][x][y] = (((ch1 >> (1 + m)) & 1u) && A1[m][x] != i && C[m][x][y] != A0[m])
                                          ? w(C[m][x][y], 1) : 0ull;
            }
            const bool c0 = ch1 & 1u;
            const uint32_t vi1 = c0 ? (nv1 & 1u) : bv(wi[1]);
            int64_t acc = 0;
            if (ch1 != 0) {
                int ones = 0;
#pragma unroll
                for (int m = 0; m < D; ++m) ones += (int)(((ch1 >> (1 + m)) & 1u) ? ((nv1 >> (1 + m)) & 1u) : bv(wa[m][1]));
                const uint32_t nb = maj(ones, vi1);
                if (nb != bv(wi[2])) { ch2 |= 1u; acc += nb ? 2 : -2; }
            }
#pragma unroll
            for (int m = 0; m < D; ++m) {
                const bool cm = (ch1 >> (1 + m)) & 1u;
                const uint32_t va1 = cm ? ((nv1 >> (1 + m)) & 1u) : bv(wa[m][1]);
                if (c0 || cm) {
                    int ones = 0;
#pragma unroll
                    for (int x = 0; x < D; ++x) ones += (int)((A1[m][x] == i) ? vi1 : bv(wc[m][x][1]));
                    const uint32_t nb = maj(ones, va1);
                    if (nb != bv(wa[m][2])) { ch2 |= 2u << m; acc += nb ? 2 : -2; }
                }
                if (cm) {
#pragma unroll
                    for (int x = 0; x < D; ++x) {
                        if (A1[m][x] == i) continue;
                        int ones = 0;
#pragma unroll
                        for (int y = 0; y < D; ++y) {
                            uint32_t gv;
                            if constexpr (NB) gv = (wn[m][x] >> (nbs + y)) & 1u;
                            else gv = bv(wg[m][x][y]);
                            ones += (int)((C[m][x][y] == A0[m]) ? va1 : gv);
                        }
                        const uint32_t nb = maj(ones, bv(wc[m][x][1]));
                        if (nb != bv(wc[m][x][2])) { ch2 |= 1u << (1 + D + m * D + x); acc += nb ? 2 : -2; }
                    }
                }
            }
            ds = acc;
            }
        } else if (mine && k == 0) {
            // not a tree: the batched table path, and only as the batch's first proposal
            listpath = true;
            if (simple) ds = lc_delta_mlp<D, true>(adj, NS, colo, bit, T, L, lists, i, cnt, &old_i, A0, A1);
            else ds = lc_delta_mlp<D, false>(adj, NS, colo, bit, T, L, lists, i, cnt, &old_i, A0, A1);
        }
        SA_STAMP(2);
        // the next batch: the rows of its i's neighbours (land during the filter
        // phase and the resolution)
#pragma unroll
        for (int m = 0; m < D; ++m) row(n_A0[m], n_A1[m]);
        // potential writes of every proposal into the replica's filter
        constexpr int NTW = 1 + D + D * D;                  // tree positions: i, the a_m, their children
        if (mine && listpath) {
            fins(i);
#pragma unroll
            for (int lv = 1; lv <= T; ++lv)
                for (int q = 0; q < cnt[lv]; ++q) fins((int32_t)(lists[(L.off[lv] + q) * 64] & 0x7fffffffu));
        } else if (mine && ok) {
            const uint32_t chg = ch1 | ch2;
            int32_t wv[NTW];
            bool wm[NTW];
            wv[0] = i;
            wm[0] = true;
#pragma unroll
            for (int m = 0; m < D; ++m) {
                wv[1 + m] = A0[m];
                wm[1 + m] = (chg >> (1 + m)) & 1u;
#pragma unroll
                for (int x = 0; x < D; ++x) {
                    wv[1 + D + m * D + x] = A1[m][x];
                    wm[1 + D + m * D + x] = (ch2 >> (1 + D + m * D + x)) & 1u;
                }
            }
            fins_n(wv, wm, std::integral_constant<int, NTW>{});
        }
        SA_STAMP(6);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        SA_STAMP(7);
        // does an earlier proposal of the batch write a node this one read?
        // (k > 0 lanes are tree balls: a list-path ball stands only as k = 0)
        bool stands = mine && (ok || listpath);
        if (stands && k > 0) {
            int32_t rv[NTW];
            bool rm[NTW];
            rv[0] = i;
            rm[0] = true;
#pragma unroll
            for (int m = 0; m < D; ++m) {
                rv[1 + m] = A0[m];
                rm[1 + m] = true;
#pragma unroll
                for (int x = 0; x < D; ++x) {
                    rv[1 + D + m * D + x] = A1[m][x];
                    rm[1 + D + m * D + x] = A1[m][x] != i;
                }
            }
            bool hit = fearlier_n(rv, rm, std::integral_constant<int, NTW>{});
            if constexpr (TT == 2) {
                // the grandchildren, read only under the neighbours that changed at level 1
#pragma unroll
                for (int m = 0; m < D; ++m) {
                    if (!((ch1 >> (1 + m)) & 1u)) continue;
                    int32_t gv[D * D];
                    bool gm[D * D];
#pragma unroll
                    for (int x = 0; x < D; ++x)
#pragma unroll
                        for (int y = 0; y < D; ++y) {
                            gv[x * D + y] = C[m][x][y];
                            gm[x * D + y] = A1[m][x] != i && C[m][x][y] != A0[m];
                        }
                    hit |= fearlier_n(gv, gm, std::integral_constant<int, D * D>{});
                }
            }
            stands = !hit;
        }
        SA_STAMP(3);
        // resolution: J0 = first proposal that does not stand
        const int gs = g * K;
        const uint32_t nst = (uint32_t)((__ballot(!stands) >> gs) & GM);
        const int J0 = nst ? __ffs(nst) - 1 : K;
        // schedule and acceptance of proposal k (code/SA_RRG.py:37,74-81)
        double ak = a, bk = b;
        for (int q = 0; q < k; ++q) {
            if (ak < a_cap) ak = par_a * ak;
            if (bk < b_cap) bk = par_b * bk;
        }
        const bool inb = k < J0;
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * ak) * si;
        const double t2 = bk * (double)(-ds);
        const double dE = (t1 + t2) / (double)n;
        const double e = exp(-dE);
        const double prob = (e < 1.0) ? e : 1.0;
        const bool acc = inb && u < prob;
        // the stop: sum_end and t after proposal k
        int64_t pre = acc ? ds : 0;
#pragma unroll
        for (int o = 1; o < K; o <<= 1) {
            const int64_t v = __shfl_up(pre, o, K);
            if (k >= o) pre += v;
        }
        const int64_t sum_after = sum_end + pre;
        const int dn = (t + k + 1 > t_cap) ? 2 : ((sum_after == n) ? 1 : 0);
        const uint32_t dm = (uint32_t)((__ballot(inb && dn != 0) >> gs) & GM);
        const int J = dm ? min(J0, __ffs(dm)) : J0;
        if (k < J) {
            if (e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e)) ++ties;
            if (acc) {
                auto flip = [&](int32_t v, int lv) {
                    atomicXor((unsigned long long*)(cone + (int64_t)v * NS + colo + lv), (unsigned long long)bit);
                };
                flip(i, 0);
                atomicXor((unsigned long long*)(L.s0c + (int64_t)i * W + col), (unsigned long long)bit);
                if (listpath) {
#pragma unroll
                    for (int lv = 1; lv <= T; ++lv)
                        for (int q = 0; q < cnt[lv]; ++q) flip((int32_t)(lists[(L.off[lv] + q) * 64] & 0x7fffffffu), lv);
                    if constexpr (NB) {
                        // a level-1 change of v: its bit in each neighbour's record, at
                        // the slots where that neighbour's row holds v (rows re-read)
                        for (int q = 0; q < cnt[1]; ++q) {
                            const int32_t v = (int32_t)(lists[(L.off[1] + q) * 64] & 0x7fffffffu);
                            int32_t rv[D];
                            row(v, rv);
#pragma unroll
                            for (int e = 0; e < D; ++e) {
                                bool seen = false;               // (a multi-edge: that neighbour once)
#pragma unroll
                                for (int e2 = 0; e2 < e; ++e2) seen |= rv[e2] == rv[e];
                                if (seen) continue;
                                int32_t ru[D];
                                row(rv[e], ru);
                                uint32_t sl = 0;
#pragma unroll
                                for (int y = 0; y < D; ++y) sl |= (ru[y] == v) ? (1u << y) : 0u;
                                nbx(rv[e], sl);
                            }
                        }
                    }
                } else {
                    if (ch1 & 1u) flip(i, 1);
                    if (ch2 & 1u) flip(i, 2);
#pragma unroll
                    for (int m = 0; m < D; ++m) {
                        if ((ch1 >> (1 + m)) & 1u) flip(A0[m], 1);
                        if ((ch2 >> (1 + m)) & 1u) flip(A0[m], 2);
#pragma unroll
                        for (int x = 0; x < D; ++x)
                            if ((ch2 >> (1 + D + m * D + x)) & 1u) flip(A1[m][x], 2);
                    }
                    if constexpr (NB) {
                        // level-1 changes into the neighbours' records: i's (tree: a_m
                        // is slot m of i's row) and the a_m's (i at its slots of a_m's
                        // row; a_m at its slots of each child's row)
                        if (ch1 & 1u) {
#pragma unroll
                            for (int m = 0; m < D; ++m) {
                                uint32_t sl = 0;
#pragma unroll
                                for (int x = 0; x < D; ++x) sl |= (A1[m][x] == i) ? (1u << x) : 0u;
                                nbx(A0[m], sl);
                            }
                        }
                        uint32_t si = 0;
#pragma unroll
                        for (int m = 0; m < D; ++m) si |= ((ch1 >> (1 + m)) & 1u) << m;
                        if (si) nbx(i, si);
#pragma unroll
                        for (int m = 0; m < D; ++m) {
                            if (!((ch1 >> (1 + m)) & 1u)) continue;
#pragma unroll
                            for (int x = 0; x < D; ++x) {
                                if (A1[m][x] == i) continue;
                                uint32_t sl = 0;
#pragma unroll
                                for (int y = 0; y < D; ++y) sl |= (C[m][x][y] == A0[m]) ? (1u << y) : 0u;
                                nbx(A1[m][x], sl);
                            }
                        }
                    }
                }
            }
            if (st.tr_i) st.tr_i[kk * R + r] = i;
            if (st.tr_acc) st.tr_acc[kk * R + r] = acc ? 1 : 0;
            if (st.tr_sum) st.tr_sum[kk * R + r] = sum_after;
            if (st.tr_dE) st.tr_dE[kk * R + r] = dE;
        }
        // the replica's state after the J consumed proposals (lane J-1's)
        if (going) {
            const int src = gs + J - 1;
            sum_end = __shfl(sum_after, src, 64);
            done = __shfl(dn, src, 64);
            for (int q = 0; q < J; ++q) {
                if (a < a_cap) a = par_a * a;
                if (b < b_cap) b = par_b * b;
            }
            t += J;
            pos += J;
            // the prefetched batch is the next one only if all K were consumed
            pf_pos = (J == K) ? pos : -1;
        } else {
            (void)__shfl(sum_after, lane, 64);                // keep the shuffles wave-uniform
            (void)__shfl(dn, lane, 64);
        }
        pf_i = n_i;
        pf_u = n_u;
#pragma unroll
        for (int m = 0; m < D; ++m) {
            pf_A0[m] = n_A0[m];
#pragma unroll
            for (int x = 0; x < D; ++x) pf_A1[m][x] = n_A1[m][x];
        }
        // flips land before the next batch reads; the filter reads end before the next clear
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        SA_STAMP(4);
    }
#ifdef MJX_SA_PROF
    if (threadIdx.x == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&mjx_sa_prof[q], _acc[q]);
#endif
    // steps of this launch after the replica finished
    if (live && (st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE)) {
        for (int64_t q = pos + k; q < nsteps; q += K) {
            if (st.tr_i) st.tr_i[q * R + r] = -1;
            if (st.tr_acc) st.tr_acc[q * R + r] = -1;
            if (st.tr_sum) st.tr_sum[q * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[q * R + r] = 0.0;
        }
    }
#pragma unroll
    for (int o = K / 2; o >= 1; o >>= 1) ties += __shfl_xor(ties, o, K);
    if (live && k == 0) {
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}

static int lc_slots(int d, int T, int* off, bool table = false, int* tab = nullptr, int* ballT = nullptr) {
    int64_t total = 0, ball = 1, shell = 1;
    for (int t = 0; t <= T; ++t) {
        if (t > 0) {
            shell = (t == 1) ? d : shell * (d - 1);
            ball += shell;
        }
        off[t] = (int)total;
        total += ball;
        if (total > (1 << 20)) return -1;
    }
    off[T + 1] = (int)total;
    total += ball;                    // candidates of the last level
    if (table) {
        *tab = (int)total;
        *ballT = (int)ball;
        total += ball * (4 + d) + off[T + 1];   // node, row, candidate, mark, value; change-list entries
        if (total > (1 << 20)) return -1;
    }
    return (int)total;
}

constexpr size_t kLcLdsMax = 150 * 1024;

// waves per word column: fill the CUs with about two waves each (LDS allowing)
static int lc_split(int64_t W, size_t lds) {
    const int64_t per_cu = (lds > 0) ? std::max<int64_t>(1, std::min<int64_t>(2, (int64_t)(160 * 1024) / (int64_t)lds)) : 2;
    const int64_t target = (int64_t)device_cus() * per_cu;
    int s = 1;
    while (s < 64 && W * s * 2 <= target) s *= 2;
    return s;
}

// the batched-load evaluation is instantiated for these degrees
static bool lc_mlp_degree(int d) { return d == 3 || d == 4 || d == 6; }

}  // namespace mjx

using namespace mjx;

static int sa_init_finish(const int32_t* adj, int64_t n, int d, int T, int64_t R, int64_t W, double a0, double b0,
                          uint64_t* s, uint64_t* tmp1, uint64_t* tmp2, const mjx_sa_state& st, void* stream) {
    hipStream_t hs = as_stream(stream);
    MJX_HIP(hipMemsetAsync(st.cnt, 0, (size_t)R * sizeof(unsigned long long), hs), "sa_init memset");
    int rc = st.rep_graph ? mjx_rollout_ell_rp_multi(adj, n, d, R, st.rep_graph, s, tmp1, tmp2, T, st.cnt, stream)
                          : mjx_rollout_ell_rp(adj, n, d, W, s, tmp1, tmp2, T, st.cnt, stream);
    if (rc) return rc;
    k_sa_init_state<<<(unsigned)((R + 255) / 256), 256, 0, hs>>>(n, R, a0, b0, st.cnt, st);
    MJX_LAUNCH_CHECK("k_sa_init_state");
    return MJX_OK;
}

static bool sa_state_complete(const mjx_sa_state& st) {
    return st.mt && st.mt_idx && st.a && st.b && st.t && st.sum_end && st.done && st.prop_i && st.prop_s &&
           st.prop_u && st.cnt;
}

extern "C" int mjx_sa_init_mt(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, const uint32_t* mt_in,
                              const int32_t* idx_in, double a0, double b0, uint64_t* s, uint64_t* tmp1, uint64_t* tmp2,
                              mjx_sa_state* stp, void* stream) {
    if (!stp || n < 2 || R < 1 || d < 1 || p < 0 || c < 0 || p + c < 1 || !adj || !mt_in || !idx_in || !s || !tmp1)
        return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    mjx_sa_state st = *stp;
    if (!sa_state_complete(st)) return MJX_EINVAL;
    const int64_t W = (R + 63) / 64;
    const int T = p + c - 1;
    if (T >= 2 && !tmp2) return MJX_EINVAL;
    // lane per replica: each lane continues its own stream from its own index
    k_sa_init_draw<<<(unsigned)W, 64, 0, as_stream(stream)>>>(n, R, W, nullptr, (u64*)s, st.mt, st.mt_idx, mt_in,
                                                               idx_in);
    MJX_LAUNCH_CHECK("k_sa_init_draw");
    return sa_init_finish(adj, n, d, T, R, W, a0, b0, s, tmp1, tmp2, st, stream);
}

extern "C" int mjx_sa_init(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, const uint32_t* seeds,
                           double a0, double b0, uint64_t* s, uint64_t* tmp1, uint64_t* tmp2, mjx_sa_state* stp,
                           void* stream) {
    if (!stp || n < 2 || R < 1 || d < 1 || p < 0 || c < 0 || p + c < 1 || !adj || !seeds || !s || !tmp1) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    mjx_sa_state st = *stp;
    if (!st.mt || !st.mt_idx || !st.a || !st.b || !st.t || !st.sum_end || !st.done || !st.prop_i || !st.prop_s ||
        !st.prop_u || !st.cnt)
        return MJX_EINVAL;
    const int64_t W = (R + 63) / 64;
    const int T = p + c - 1;
    if (T >= 2 && !tmp2) return MJX_EINVAL;
    hipStream_t hs = as_stream(stream);
    // s0 draws, wave per replica, through node-packed rows in tmp1 (n*W words
    // hold G word columns of 64 rows of ceil(n/64) words each)
    const int64_t nw = (n + 63) / 64;
    int64_t G = (n * W) / (64 * nw);
    if (G > W) G = W;
    if (G < 1) {                                     // tiny n: the lane-per-replica path
        k_sa_init_draw<<<(unsigned)W, 64, 0, hs>>>(n, R, W, seeds, (u64*)s, st.mt, st.mt_idx);
        MJX_LAUNCH_CHECK("k_sa_init_draw");
    } else {
        for (int64_t w0 = 0; w0 < W; w0 += G) {
            const int64_t cols = (W - w0 < G) ? W - w0 : G;
            k_sa_init_np<<<(unsigned)(cols * 64), 64, 0, hs>>>(n, R, w0 * 64, seeds, (u64*)tmp1, st.mt, st.mt_idx);
            MJX_LAUNCH_CHECK("k_sa_init_np");
            const int64_t waves = cols * nw;
            k_np_to_rp<<<(unsigned)((waves + 3) / 4), 256, 0, hs>>>((const u64*)tmp1, n, W, w0, cols, (u64*)s);
            MJX_LAUNCH_CHECK("k_np_to_rp");
        }
    }
    return sa_init_finish(adj, n, d, T, R, W, a0, b0, s, tmp1, tmp2, st, stream);
}

extern "C" int mjx_sa_steps(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, uint64_t* s,
                            uint64_t* tmp1, uint64_t* tmp2, mjx_sa_state* stp, int64_t nsteps, double par_a,
                            double par_b, double a_cap, double b_cap, int64_t t_cap, void* stream) {
    if (!stp || n < 2 || R < 1 || d < 1 || p < 0 || c < 0 || p + c < 1 || !adj || !s || !tmp1 || nsteps < 0)
        return MJX_EINVAL;
    if (stp->philox_key) return MJX_EINVAL;             // draws the MT19937 replay inside the step
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    mjx_sa_state st = *stp;
    const int64_t W = (R + 63) / 64;
    const int T = p + c - 1;
    if (T >= 2 && !tmp2) return MJX_EINVAL;
    hipStream_t hs = as_stream(stream);
    const unsigned gridR = (unsigned)((R + kBlock - 1) / kBlock);
    for (int64_t k = 0; k < nsteps; ++k) {
        k_sa_propose<<<gridR, kBlock, 0, hs>>>(n, R, W, (u64*)s, st, k);
        MJX_LAUNCH_CHECK("k_sa_propose");
        MJX_HIP(hipMemsetAsync(st.cnt, 0, (size_t)R * sizeof(unsigned long long), hs), "sa_steps memset");
        int rc = st.rep_graph ? mjx_rollout_ell_rp_multi(adj, n, d, R, st.rep_graph, s, tmp1, tmp2, T, st.cnt, stream)
                              : mjx_rollout_ell_rp(adj, n, d, W, s, tmp1, tmp2, T, st.cnt, stream);
        if (rc) return rc;
        k_sa_accept<<<gridR, kBlock, 0, hs>>>(n, R, W, (u64*)s, st, k, par_a, par_b, a_cap, b_cap, t_cap);
        MJX_LAUNCH_CHECK("k_sa_accept");
    }
    return MJX_OK;
}


extern "C" int64_t mjx_sa_lightcone_lds(int d, int p, int c) {
    const int T = p + c - 1;
    if (d < 1 || d > LC_MAXD || T < 1 || T > LC_MAXT) return -1;
    int off[LC_MAXT + 2], tab, ball;
    if (lc_mlp_degree(d)) {
        const int s2 = lc_slots(d, T, off, true, &tab, &ball);
        if (s2 > 0 && (size_t)s2 * 64 * 4 <= kLcLdsMax) return (int64_t)s2 * 64 * 4;
    }
    const int slots = lc_slots(d, T, off);
    if (slots < 0) return -1;
    return (int64_t)slots * 64 * 4;
}

extern "C" int mjx_sa_lightcone_prepare(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R,
                                        const int32_t* rep_graph, const uint64_t* s, uint64_t* const* levels,
                                        void* stream) {
    const int T = p + c - 1;
    if (!adj || !s || !levels || n < 2 || R < 1 || d < 1 || T < 1 || T > LC_MAXT) return MJX_EINVAL;
    const int64_t W = (R + 63) / 64;
    const uint64_t* src = s;
    for (int t = 0; t < T; ++t) {
        if (!levels[t]) return MJX_EINVAL;
        int rc = rep_graph ? mjx_rollout_ell_rp_multi(adj, n, d, R, rep_graph, src, levels[t], nullptr, 1, nullptr, stream)
                           : mjx_rollout_ell_rp(adj, n, d, W, src, levels[t], nullptr, 1, nullptr, stream);
        if (rc) return rc;
        src = levels[t];
    }
    return MJX_OK;
}

// Shared body of the two light-cone entry points: L.s / ns / cs / s0c set by
// the caller (separate level arrays or the cone layout).
constexpr int64_t kTapeRamp = 16;      // MT19937 tape chunks: 128, 16x, ..., half the tape
// The proposal-tape side stream of one caller stream: a non-blocking stream
// on the caller stream's device with the five events of the chunk hand-off,
// created on first use and kept (a per-device cache keyed by stream, SURVEY.md
// 8(b)): independent callers on different streams draw their tapes on
// different side streams, never queued behind each other's step events.  `mu`
// serialises two host threads enqueueing on one stream.  A call holds its
// entry by shared_ptr, so the cache may retire an entry only when no call holds
// it and its side stream is idle: past 64 entries (a caller making a fresh
// stream per call must not grow the cache without bound) one such entry goes.
struct TapeSide {
    hipStream_t side = nullptr;
    hipEvent_t ev[5] = {};
    std::mutex mu;
    ~TapeSide() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (side) (void)hipStreamDestroy(side);
    }
};

static std::shared_ptr<TapeSide> tape_side_for(hipStream_t caller) {
    static std::mutex mu;
    // never destroyed: no HIP call from static destructors at process exit
    static auto& per = *new std::map<std::pair<int, hipStream_t>, std::shared_ptr<TapeSide>>();
    hipDevice_t dev = 0;
    if (hipStreamGetDevice(caller, &dev) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(mu);
    const std::pair<int, hipStream_t> key{(int)dev, caller};
    auto hit = per.find(key);
    if (hit != per.end()) return hit->second;
    if (per.size() >= 64) {
        for (auto it = per.begin(); it != per.end(); ++it) {
            if (it->second.use_count() > 1) continue;                  // a call holds it
            if (hipStreamQuery(it->second->side) != hipSuccess) {      // tapes still drawing
                (void)hipGetLastError();
                continue;
            }
            per.erase(it);                                             // (the destructor releases it)
            break;
        }
    }
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    const bool other = cur != (int)dev;
    if (other && hipSetDevice(dev) != hipSuccess) return nullptr;
    auto ts = std::make_shared<TapeSide>();
    bool ok = hipStreamCreateWithFlags(&ts->side, hipStreamNonBlocking) == hipSuccess;
    for (int q = 0; ok && q < 5; ++q)
        ok = hipEventCreateWithFlags(&ts->ev[q], hipEventDisableTiming) == hipSuccess;
    if (!ok) {                                   // nothing half-made is kept (the destructor frees it)
        (void)hipGetLastError();
        ts.reset();
    }
    if (other) (void)hipSetDevice(cur);
    if (ts) per[key] = ts;
    return ts;
}

static int lc_steps(const int32_t* adj, const int32_t* adj_pad, int64_t n, int d, int T, int64_t R, LcLevels L,
                    mjx_sa_state* stp,
                    int64_t nsteps, double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                    void* stream) {
    int slots = -1;
    L.tab = -1;
    L.ball = 0;
    if (lc_mlp_degree(d)) {
        slots = lc_slots(d, T, L.off, true, &L.tab, &L.ball);
        if (slots < 0 || (size_t)slots * 64 * 4 > kLcLdsMax) L.tab = -1;
    }
    if (L.tab < 0) slots = lc_slots(d, T, L.off);
    const size_t lds = (size_t)slots * 64 * 4;
    if (slots < 0 || lds > kLcLdsMax) return MJX_ERANGE;
    for (int t = T + 1; t <= LC_MAXT; ++t) L.s[t] = nullptr;
    if (nsteps == 0) return MJX_OK;
    const int64_t W = (R + 63) / 64;
    hipStream_t hs = as_stream(stream);
    const mjx_sa_state st = *stp;
    const bool tape = st.tape_i && st.tape_u && st.tape_cap > 0;
    if (st.philox_key && !tape) return MJX_EINVAL;       // the Philox stream is drawn into the tape
    const int split = st.opt_split ? st.opt_split : lc_split(W, lds);
    if (split < 1 || split > 64 || (64 % split)) return MJX_EINVAL;
    if (st.opt_spec_k != 0 && st.opt_spec_k != 8 && st.opt_spec_k != 16) return MJX_EINVAL;
    if (st.opt_flags &
        ~(MJX_SA_NO_SPEC | MJX_SA_NO_CONE2 | MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR | MJX_SA_LDS_WAVE))
        return MJX_EINVAL;
    // the one-trip and speculative kernels address a word column's cone slab
    // with 32-bit byte offsets (ConeRd)
    const bool slab32 = L.s0c && n * L.ns * 8 < (int64_t(1) << 31);
    // one launch per tape chunk (the tape kernel fills the chunk's (i, u) first)
    auto launch = [&](auto kern, mjx_sa_state s2, int64_t k) -> int {
        MJX_HIP(set_max_lds(kern, (int)lds), "lightcone lds");
        kern<<<(unsigned)(W * split), 64, lds, hs>>>(adj, d, n, R, W, L, T, s2, k, par_a, par_b, a_cap, b_cap,
                                                     t_cap, s2.tape_i, s2.tape_u, split, st.rep_graph);
        MJX_LAUNCH_CHECK("k_sa_lightcone");
        return MJX_OK;
    };
    // cone layout, p+c-1 = 2, d = 3 with the tape: the one-round-trip kernel
    const bool one_trip = tape && slab32 && adj_pad && T == 2 && d == 3 && L.tab >= 0 &&
                          !(st.opt_flags & MJX_SA_NO_CONE2);
    auto launch_one_trip = [&](mjx_sa_state s2, int64_t k) -> int {
        auto kern = k_sa_cone2<3>;
        MJX_HIP(set_max_lds(kern, (int)lds), "cone2 lds");
        kern<<<(unsigned)(W * split), 64, lds, hs>>>(adj, (const int4*)adj_pad, n, R, W, L, s2, k, par_a, par_b,
                                                     a_cap, b_cap, t_cap, s2.tape_i, s2.tape_u, split, st.rep_graph);
        MJX_LAUNCH_CHECK("k_sa_cone2");
        return MJX_OK;
    };
    // ... and its speculative form: the 8 lanes of a group take 8 proposals of one replica
    // 16-B rows (the record layout reads them from the records)
    const int4* rows4 = (d == 4 || L.lo) ? (const int4*)adj : (const int4*)adj_pad;
    // 8 proposals per batch; 16 when 8 would leave CUs without a wave (few word columns):
    // configs[1] at R = 1024 3.05 -> 1.78 us per step, at R = 4096 16 is slower (3.76 vs 4.10)
    const int spec_k = st.opt_spec_k ? st.opt_spec_k : ((W * 8 < device_cus()) ? 16 : 8);
    const bool spec = tape && slab32 && rows4 && L.tab >= 0 && n < (int64_t(1) << (spec_k == 16 ? 27 : 28)) &&
                      !(st.opt_flags & MJX_SA_NO_SPEC) && ((d == 3 && (T == 1 || T == 2)) || (d == 4 && T == 1));
    const int hoff = slots * 64;
    const size_t lds_spec = lds + SPEC_LDS;
    // d = 3, p+c-1 = 2 records carry their neighbours' level-1 words (nb_byte),
    // kept by the speculative kernel; another kernel's steps leave them stale
    // (stp->rec_nb = 0), and they are rebuilt before the next speculative one
    const bool nbw = L.lo == 2 && d == 3 && T == 2;
    if (nbw && spec && !stp->rec_nb && nsteps > 0) {
        k_rec_nb_fill<<<grid_for(n * W), kBlock, 0, hs>>>((u64*)L.s[0] - L.lo, n, W);
        MJX_LAUNCH_CHECK("k_rec_nb_fill");
        stp->rec_nb = 1;
    }
    if (nbw && !spec && nsteps > 0) stp->rec_nb = 0;
    auto launch_spec = [&](mjx_sa_state s2, int64_t k) -> int {
        auto go = [&](auto kern, int K) {      // K waves per word column (64 / K replicas per wave)
            MJX_HIP(set_max_lds(kern, (int)lds_spec), "spec lds");
            kern<<<(unsigned)(W * K), 64, lds_spec, hs>>>(adj, rows4, n, R, W, L, s2, k, par_a, par_b,
                                                                      a_cap, b_cap, t_cap, s2.tape_i, s2.tape_u,
                                                                      hoff, st.rep_graph);
            MJX_LAUNCH_CHECK("k_sa_spec");
            return MJX_OK;
        };
        if (spec_k == 16) {
            if (d == 4) return go(k_sa_spec<4, 1, 16, false>, 16);
            if (T == 2) return nbw ? go(k_sa_spec<3, 2, 16, true>, 16) : go(k_sa_spec<3, 2, 16, false>, 16);
            return go(k_sa_spec<3, 1, 16, false>, 16);
        }
        if (d == 4) return go(k_sa_spec<4, 1, 8, false>, 8);
        if (T == 2) return nbw ? go(k_sa_spec<3, 2, 8, true>, 8) : go(k_sa_spec<3, 2, 8, false>, 8);
        return go(k_sa_spec<3, 1, 8, false>, 8);
    };
    auto step_chunk = [&](auto kern_tape, mjx_sa_state s2, int64_t k0, int64_t k) -> int {
        if (s2.tr_i) s2.tr_i += k0 * R;     // trace rows of this chunk
        if (s2.tr_acc) s2.tr_acc += k0 * R;
        if (s2.tr_sum) s2.tr_sum += k0 * R;
        if (s2.tr_dE) s2.tr_dE += k0 * R;
        return spec ? launch_spec(s2, k) : one_trip ? launch_one_trip(s2, k) : launch(kern_tape, s2, k);
    };
    auto run = [&](auto kern_plain, auto kern_tape) -> int {
        if (!tape) return launch(kern_plain, st, nsteps);
        const int64_t half = st.tape_cap / 2;
        // (a stream under graph capture keeps the one-stream form: no side stream
        // or per-call events inside a capture)
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        MJX_HIP(hipStreamIsCapturing(hs, &cap), "tape capture status");
        if (st.philox_key || half < 1 || nsteps <= 128 || cap != hipStreamCaptureStatusNone) {
            // one tape at a time on the caller's stream (the Philox tape is a
            // counter function of t: a few microseconds)
            for (int64_t k0 = 0; k0 < nsteps; k0 += st.tape_cap) {
                const int64_t k = (nsteps - k0 < st.tape_cap) ? nsteps - k0 : st.tape_cap;
                if (st.philox_key) {
                    const int64_t blocks = (k * R + 255) / 256;
                    k_sa_tape_philox<<<(unsigned)(blocks < 65536 ? blocks : 65536), 256, 0, hs>>>(
                        n, R, k, st, st.tape_i, st.tape_u);
                    MJX_LAUNCH_CHECK("k_sa_tape_philox");
                } else {
                    k_sa_tape<<<(unsigned)R, 64, 0, hs>>>(n, R, k, st, st.tape_i, st.tape_u);
                    MJX_LAUNCH_CHECK("k_sa_tape");
                }
                const int rc = step_chunk(kern_tape, st, k0, k);
                if (rc) return rc;
            }
            return MJX_OK;
        }
        // MT19937 tapes drawn a chunk ahead on a side stream into the other
        // half of the tape buffer: chunk j+1's draws (one wave per replica, a
        // CU mostly idle under the latency-bound step kernels) overlap chunk
        // j's steps.  Chunk j+1's tape waits for chunk j-1's steps (which read
        // that half); chunk j's steps wait for its tape.  A replica that
        // finishes in chunk j may get chunk j+1 drawn anyway: its stream then
        // stands past its last proposal, as with any tape (mt_state() and
        // checkpoint() refuse a tape).
        const std::shared_ptr<TapeSide> tsd = tape_side_for(hs);
        if (!tsd) {
            set_hip_error(hipErrorInvalidValue, "tape side stream");
            return MJX_EHIP;
        }
        std::lock_guard<std::mutex> tlk(tsd->mu);
        hipStream_t side = tsd->side;
        auto hrc = [](hipError_t e) -> int {
            if (e == hipSuccess) return MJX_OK;
            set_hip_error(e, "tape side stream");
            return MJX_EHIP;
        };
        hipEvent_t* ev = tsd->ev;        // re-recorded every call: a wait binds the latest record
        hipEvent_t* evT = ev;            // chunk's tape drawn (by half)
        hipEvent_t* evS = ev + 2;        // chunk's steps done (by half)
        int rc = MJX_OK;
        // chunk sizes ramp up (128, x16, ..., half) so that only the first,
        // short tape is drawn before any step runs: chunk j+1's tape (16x the
        // rows of chunk j) takes less time than chunk j's steps (a tape row of
        // R = 4096 replicas ~0.1 us, a step ~2.5 us), and a call makes few step
        // launches (each ends on its slowest wave: ~0.1 ms of tail)
        int64_t c0s[2], cks[2];                          // chunk j's first step and size, at j & 1
        int64_t next_k0 = 0, next_c = (half < 128) ? half : 128;
        int64_t nchunks = 0;
        for (int64_t k0 = 0, c = next_c; k0 < nsteps; ++nchunks) {
            k0 += (nsteps - k0 < c) ? nsteps - k0 : c;
            c = (kTapeRamp * c < half) ? kTapeRamp * c : half;
        }
        auto tape_into = [&](int64_t j) -> int {
            c0s[j & 1] = next_k0;
            cks[j & 1] = (nsteps - next_k0 < next_c) ? nsteps - next_k0 : next_c;
            next_k0 += cks[j & 1];
            next_c = (kTapeRamp * next_c < half) ? kTapeRamp * next_c : half;
            int32_t* ti = st.tape_i + (j & 1) * half * R;
            double* tu = st.tape_u + (j & 1) * half * R;
            mjx_sa_state sh = st;
            sh.tape_cap = half;                  // rows per replica in this half
            k_sa_tape<<<(unsigned)R, 64, 0, side>>>(n, R, cks[j & 1], sh, ti, tu);
            MJX_LAUNCH_CHECK("k_sa_tape");
            MJX_HIP(hipEventRecord(evT[j & 1], side), "tape record");
            return MJX_OK;
        };
        do {
            // the side stream starts behind everything already on the caller's
            if ((rc = hrc(hipEventRecord(ev[4], hs))) || (rc = hrc(hipStreamWaitEvent(side, ev[4], 0))))
                break;
            if ((rc = tape_into(0))) break;
            for (int64_t j = 0; j < nchunks && !rc; ++j) {
                if (j + 1 < nchunks) {
                    if (j >= 1 && (rc = hrc(hipStreamWaitEvent(side, evS[(j - 1) & 1], 0)))) break;
                    if ((rc = tape_into(j + 1))) break;
                }
                if ((rc = hrc(hipStreamWaitEvent(hs, evT[j & 1], 0)))) break;
                const int64_t k0 = c0s[j & 1], k = cks[j & 1];
                mjx_sa_state s2 = st;
                s2.tape_i = st.tape_i + (j & 1) * half * R;
                s2.tape_u = st.tape_u + (j & 1) * half * R;
                s2.tape_cap = half;
                if ((rc = step_chunk(kern_tape, s2, k0, k))) break;
                if ((rc = hrc(hipEventRecord(evS[j & 1], hs)))) break;
            }
        } while (false);
        return rc;
    };
    switch (d) {
        case 3: return run(k_sa_lightcone<3, false>, k_sa_lightcone<3, true>);
        case 4: return run(k_sa_lightcone<4, false>, k_sa_lightcone<4, true>);
        case 6: return run(k_sa_lightcone<6, false>, k_sa_lightcone<6, true>);
        default: return run(k_sa_lightcone<0, false>, k_sa_lightcone<0, true>);
    }
}

extern "C" int mjx_sa_lightcone_steps(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, uint64_t* s,
                                      uint64_t* const* levels, mjx_sa_state* stp, int64_t nsteps, double par_a,
                                      double par_b, double a_cap, double b_cap, int64_t t_cap, void* stream) {
    const int T = p + c - 1;
    if (!stp || !adj || !s || !levels || n < 2 || R < 1 || d < 1 || d > LC_MAXD || nsteps < 0) return MJX_EINVAL;
    if (T < 1 || T > LC_MAXT) return MJX_ERANGE;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    LcLevels L;
    L.s[0] = (u64*)s;
    for (int t = 1; t <= T; ++t) {
        if (!levels[t - 1]) return MJX_EINVAL;
        L.s[t] = (u64*)levels[t - 1];
    }
    L.ns = (R + 63) / 64;
    L.cs = 1;
    L.s0c = nullptr;
    L.lo = 0;
    return lc_steps(adj, nullptr, n, d, T, R, L, stp, nsteps, par_a, par_b, a_cap, b_cap, t_cap, stream);
}

// ---------------------------------------------------------------------------
// Cone layout: the T+1 level words of one (node, word column) side by side,
// padded to LV = 2, 4 or 8 words, so the evaluation of a proposal that reads
// several levels of one node fetches one sector instead of one line per level;
// column-major (word column w's n sectors contiguous), so the waves of one
// column, all on one XCD, gather from one n*LV*8-byte slab.
// ---------------------------------------------------------------------------
static int cone_lv(int T) { return (T + 1 <= 2) ? 2 : (T + 1 <= 4) ? 4 : 8; }

extern "C" int mjx_sa_cone_words(int p, int c) {
    const int T = p + c - 1;
    if (T < 1 || T > LC_MAXT) return -1;
    return cone_lv(T);
}

struct ConeSrc {
    const u64* s[LC_MAXT + 1];
};

template <bool PACK>
__global__ void __launch_bounds__(kBlock) k_cone_xfer(int64_t words, int T, int LV, int lo, ConeSrc src, u64* cone,
                                                      int64_t n, int64_t W, const int32_t* __restrict__ adj, int d) {
    for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < words; w += (int64_t)gridDim.x * kBlock) {
        const int64_t v = w / W;
        u64* dst = cone + ((w % W) * n + v) * LV;
        if constexpr (PACK) {
            const bool nbw = lo && d == 3 && T == 2 && LV == 8;      // the record carries neighbour words
            uint32_t nb[7] = {0, 0, 0, 0, 0, 0, 0};
            if (nbw) {
                u64 L[3];
                for (int y = 0; y < 3; ++y) L[y] = src.s[1][(int64_t)adj[v * 3 + y] * W + (w % W)];
                for (int j = 0; j < 7; ++j) nb[j] = nb_pack(L, j);
            }
            if (lo) {                 // record layout: the node's row (int32 x4, zero padded) first
                int32_t r[4] = {0, 0, 0, 0};
                for (int e = 0; e < d; ++e) r[e] = adj[v * d + e];
                if (nbw) r[3] = (int32_t)nb[6];
                *reinterpret_cast<int4*>(dst) = make_int4(r[0], r[1], r[2], r[3]);
            }
            for (int t = 0; t + lo < LV; t += 2) {
                u64 a = (t <= T) ? src.s[t][w] : 0ull;
                u64 b = (t + 1 <= T) ? src.s[t + 1][w] : 0ull;
                if (nbw && t == 2) b = (u64)nb[0] | ((u64)nb[1] << 32);           // words 5, 6, 7
                if (nbw && t == 4) {
                    a = (u64)nb[2] | ((u64)nb[3] << 32);
                    b = (u64)nb[4] | ((u64)nb[5] << 32);
                }
                *reinterpret_cast<ulonglong2*>(dst + lo + t) = make_ulonglong2(a, b);
            }
        } else {
            for (int t = 0; t <= T; ++t) const_cast<u64*>(src.s[t])[w] = dst[lo + t];
        }
    }
}

static int cone_xfer(bool pack, int64_t n, int p, int c, int64_t R, const uint64_t* s, uint64_t* const* levels,
                     uint64_t* cone, void* stream, int LV, int lo = 0, const int32_t* adj = nullptr, int d = 0) {
    const int T = p + c - 1;
    if (!s || !levels || !cone || n < 1 || R < 1) return MJX_EINVAL;
    if (T < 1 || T > LC_MAXT) return MJX_ERANGE;
    ConeSrc src;
    src.s[0] = (const u64*)s;
    for (int t = 1; t <= T; ++t) {
        if (!levels[t - 1]) return MJX_EINVAL;
        src.s[t] = (const u64*)levels[t - 1];
    }
    for (int t = T + 1; t <= LC_MAXT; ++t) src.s[t] = nullptr;
    const int64_t W = (R + 63) / 64, words = n * W;
    const int grid = grid_for(words);
    if (pack)
        k_cone_xfer<true><<<grid, kBlock, 0, as_stream(stream)>>>(words, T, LV, lo, src, (u64*)cone, n, W, adj, d);
    else
        k_cone_xfer<false><<<grid, kBlock, 0, as_stream(stream)>>>(words, T, LV, lo, src, (u64*)cone, n, W, adj, d);
    MJX_LAUNCH_CHECK("k_cone_xfer");
    return MJX_OK;
}

extern "C" int mjx_sa_cone_pack(int64_t n, int p, int c, int64_t R, const uint64_t* s, uint64_t* const* levels,
                                uint64_t* cone, void* stream) {
    if (p + c - 1 < 1 || p + c - 1 > LC_MAXT) return MJX_ERANGE;
    return cone_xfer(true, n, p, c, R, s, levels, cone, stream, cone_lv(p + c - 1));
}

extern "C" int mjx_sa_cone_unpack(int64_t n, int p, int c, int64_t R, const uint64_t* cone, uint64_t* s,
                                  uint64_t* const* levels, void* stream) {
    if (p + c - 1 < 1 || p + c - 1 > LC_MAXT) return MJX_ERANGE;
    return cone_xfer(false, n, p, c, R, s, levels, const_cast<uint64_t*>(cone), stream, cone_lv(p + c - 1));
}

// ---------------------------------------------------------------------------
// Record layout: the cone sector of a (node, word column) preceded by the
// node's adjacency row, one 32- or 64-B record (rows in words 0..1, level t at
// word 2 + t), so the speculative step's row fetches of i, its neighbours and
// their children bring their level words in the same line: one random line per
// ball node instead of two (row + sector).  A graph shared by every replica only
// (a column's replicas share its rows); d <= 4.
// ---------------------------------------------------------------------------
static int rec_lv(int d, int T) {
    if (d < 1 || d > 4 || T < 1 || T > 5) return -1;
    return (2 + T + 1 <= 4) ? 4 : 8;
}

extern "C" int mjx_sa_rec_words(int d, int p, int c) { return rec_lv(d, p + c - 1); }

extern "C" int mjx_sa_state_bytes(void) { return (int)sizeof(mjx_sa_state); }

extern "C" int mjx_sa_rec_pack(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, const uint64_t* s,
                               uint64_t* const* levels, uint64_t* rec, void* stream) {
    const int LV = rec_lv(d, p + c - 1);
    if (!adj) return MJX_EINVAL;
    if (LV < 0) return MJX_ERANGE;
    return cone_xfer(true, n, p, c, R, s, levels, rec, stream, LV, 2, adj, d);
}

extern "C" int mjx_sa_rec_unpack(int64_t n, int d, int p, int c, int64_t R, const uint64_t* rec, uint64_t* s,
                                 uint64_t* const* levels, void* stream) {
    const int LV = rec_lv(d, p + c - 1);
    if (LV < 0) return MJX_ERANGE;
    return cone_xfer(false, n, p, c, R, s, levels, const_cast<uint64_t*>(rec), stream, LV, 2);
}

extern "C" int mjx_sa_cone_steps(const int32_t* adj, const int32_t* adj_pad, int64_t n, int d, int p, int c,
                                 int64_t R, uint64_t* s, uint64_t* cone, mjx_sa_state* stp, int64_t nsteps,
                                 double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                                 void* stream) {
    const int T = p + c - 1;
    if (!stp || !adj || !s || !cone || n < 2 || R < 1 || d < 1 || d > LC_MAXD || nsteps < 0) return MJX_EINVAL;
    if (T < 1 || T > LC_MAXT) return MJX_ERANGE;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    const int LV = cone_lv(T);
    LcLevels L;
    for (int t = 0; t <= T; ++t) L.s[t] = (u64*)cone + t;
    L.ns = LV;
    L.cs = n * LV;
    L.s0c = (u64*)s;
    L.lo = 0;
    return lc_steps(adj, adj_pad, n, d, T, R, L, stp, nsteps, par_a, par_b, a_cap, b_cap, t_cap, stream);
}

extern "C" int mjx_sa_rec_steps(const int32_t* adj, const int32_t* adj_pad, int64_t n, int d, int p, int c,
                                int64_t R, uint64_t* s, uint64_t* rec, mjx_sa_state* stp, int64_t nsteps,
                                double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                                void* stream) {
    const int T = p + c - 1;
    if (!stp || !adj || !s || !rec || n < 2 || R < 1 || d < 1 || nsteps < 0) return MJX_EINVAL;
    if (stp->rep_graph) return MJX_EINVAL;          // rows are per column: one shared graph
    const int LV = rec_lv(d, T);
    if (LV < 0 || n > (int64_t)INT32_MAX) return MJX_ERANGE;
    LcLevels L;
    for (int t = 0; t <= T; ++t) L.s[t] = (u64*)rec + 2 + t;
    L.ns = LV;
    L.cs = n * LV;
    L.s0c = (u64*)s;
    L.lo = 2;
    return lc_steps(adj, adj_pad, n, d, T, R, L, stp, nsteps, par_a, par_b, a_cap, b_cap, t_cap, stream);
}

#ifdef MJX_SA_PROF
extern "C" int mjx_sa_prof_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mjx_sa_prof), 8 * sizeof(unsigned long long)) != hipSuccess) return MJX_EHIP;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mjx_sa_prof), z, sizeof(z)) != hipSuccess) return MJX_EHIP;
    }
    return MJX_OK;
}
#endif
