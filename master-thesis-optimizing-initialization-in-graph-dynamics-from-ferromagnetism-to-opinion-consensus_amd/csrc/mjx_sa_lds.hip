// LDS-resident light-cone SA for the reference's own graph sizes
// (code/SA_RRG.py:44-52: n = 1e4, d = 4; configs[0]).
//
// A workgroup (one wave) owns one replica for a whole launch: its graph's
// adjacency as uint16 rows, the cached rollout levels s_t = onestep^t(s),
// t = 0..T (T = p+c-1), as bit arrays, and its MT19937 state all live in LDS
// (n = 1e4, d = 4, T = 3: 94 KB), so a proposal's light-cone evaluation makes
// LDS round trips only.  The HBM/L2-resident kernels (mjx_sa.hip) pay one
// memory round trip per dependent load -- about 90 us per step at p = 3 --
// which is what makes SA_RRG.py's run to consensus (1e5-1e8+ proposals per
// replica) slow there.
//
// Per step (code/SA_RRG.py:73-85), wave-uniform:
//   * i = randint(0, n), u = rand() from the replica's numpy stream (legacy
//     MT19937: masked rejection over tempered words, 53-bit doubles); the words
//     of one randint are tested 64 at a time with one ballot, the state is
//     twisted in LDS exactly when numpy would twist it, so the stream position
//     after the launch is numpy's (no draw-ahead);
//   * the change sets C_t of the levels (C_0 = {i flipped}): candidates of
//     level t are C_{t-1} and its neighbours, one lane each; a candidate's
//     level-(t-1) inputs are the cached bits XOR the change marks of C_{t-1}
//     (one 8-byte read per node: level word and mark word side by side; a
//     node in C_t holds the complement of its cached value); it joins C_t
//     when the always-stay majority (code/SA_RRG.py:19-20) differs from its
//     cached level-t bit (the mark's atomicOr dedups repeated candidates);
//   * sum(s_end(flipped)) - sum(s_end) = sum over C_T of +-2; delta_H in float64
//     in the reference's operation order (this unit is built with
//     -ffp-contract=off), Metropolis test, schedule, stop tests;
//   * an accepted proposal XORs its change sets into the level bit arrays;
//     every proposal clears the marks it set (from the lists C_t).
// Round 3: the round-2 form kept C_t as an LDS hash of node -> new value,
// probed for every neighbour of every candidate (2-3 dependent LDS reads per
// probe); marks make every value one read: 5.3 -> see DESIGN.md per step at
// SA_RRG.py's p = 3, n = 1e4.
// At the end of the launch the changed level-0 bits go back to the
// replica-packed configuration s (atomicXor of the replica's bit: the other
// 63 replicas of a word are other workgroups) and the MT state, a, b, t,
// sum_end, done back to the state arrays.  Same proposals, accepts and outputs
// as every other SA mode.
#include "mjx_common.h"
#include <type_traits>
#include "mjx_mt.h"
#include <math.h>

#pragma clang fp contract(off)

namespace mjx {
namespace salds {

constexpr int kMaxT = 6;
constexpr size_t kLdsMax = 160 * 1024;

struct Geo {
    int rw;          // uint16 entries per adjacency row (4, 8 or 16)
    int nw;          // uint32 bit words per level (even)
    int lc;          // change-list capacity per level (>= the radius-T ball)
    int lvs;         // uint32 per level word entry: {level, marks} (2) or {level, marks A, marks B, -} (4)
    int off_lev;     // byte offsets into the dynamic LDS
    int off_lev0;
    int off_mt;
    int off_list;
    int off_cnt;
    int bytes;
};

static int64_t ball(int d, int T) {
    int64_t b = 1, shell = 1;
    for (int t = 1; t <= T; ++t) {
        shell = (t == 1) ? d : shell * (d - 1);
        b += shell;
        if (b > (1 << 20)) return b;
    }
    return b;
}

static bool geometry(int64_t n, int d, int T, Geo* g, int planes = 1) {
    if (n < 2 || n > 65535 || d < 1 || d > 16 || T < 1 || T > kMaxT) return false;
    g->lvs = (planes == 1) ? 2 : 4;
    g->rw = (d <= 4) ? 4 : (d <= 8) ? 8 : 16;
    g->nw = (int)(((n + 63) / 64) * 2);
    int64_t lc = ball(d, T);
    if (lc > n) lc = n;
    lc = ((lc + 63) / 64) * 64;
    if (lc > 4096) return false;
    g->lc = (int)lc;
    int64_t off = ((int64_t)n * g->rw * 2 + 15) / 16 * 16;
    g->off_lev = (int)off;   off += (int64_t)(T + 1) * g->nw * 4 * g->lvs;   // {level bits, change bits} per word
    g->off_lev0 = (int)off;  off += (int64_t)g->nw * 4;
    g->off_mt = (int)off;    off += MT_N * 4;
    g->off_list = (int)off;  off += (int64_t)planes * (T + 1) * g->lc * 4;
    g->off_cnt = (int)off;   off += 32 * 4;
    g->bytes = (int)off;
    return (size_t)off <= kLdsMax;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int64_t wave_sum(int64_t x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// lane l's 64-bit value (l wave-uniform): two readlanes, no LDS round trip
__device__ __forceinline__ int64_t rl64(int64_t x, int l) {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)x >> 32), l) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l));
}

// Diagnostic build only (-DMJX_SA_PROF, tools/sa_lds_prof.py): per-phase
// s_memtime cycles of k_sa_lds_fast summed over waves; every stamp drains the
// wave's counters first, so a phase's exposed latency is charged to it.
#ifdef MJX_SA_PROF
__device__ unsigned long long mjx_sa_lds_prof[32];
#define LDS_STAMP(k) do { __builtin_amdgcn_sched_barrier(0); asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); const unsigned long long _c = __builtin_amdgcn_s_memtime(); _acc[k] += _c - _t0; _t0 = _c; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define LDS_STAMP(k) do {} while (0)
#endif

// Level t of the replica is a bit array (bit v = the cached value onestep^t(s)
// of node v) interleaved word by word with a change-bit array: lv[2(t nw + w)]
// = level word w, lv[2(t nw + w) + 1] = change word w.  During a proposal the
// change bits mark C_t, the nodes whose level-t value the flip changes; a
// changed node's new value is the complement of its cached one (that is what
// puts it in C_t), so "level t as the proposal sees it" is level XOR change:
// ONE 8-byte LDS read per node, no hash table.  An accepted proposal XORs the
// marked bits into the levels; every step clears the marks it set (the lists
// hold them).
template <int D>
__global__ void __launch_bounds__(64) k_sa_lds(const int32_t* __restrict__ adj, int dd, int64_t n, int T, int64_t R,
                                               int64_t W, u64* __restrict__ s, mjx_sa_state st, int64_t nsteps,
                                               double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                                               Geo geo) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int d = (D > 0) ? D : dd;
    const int lane = threadIdx.x;
    const int64_t r = blockIdx.x;
    const int64_t col = r >> 6;
    const u64 rbit = 1ull << (r & 63);
    const int nw = geo.nw, rw = geo.rw, lc = geo.lc;
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lv = reinterpret_cast<uint32_t*>(smem + geo.off_lev);       // {level, change} word pairs
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);   // level 0 at launch start
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    uint32_t* lst = reinterpret_cast<uint32_t*>(smem + geo.off_list);     // C_t at lst + t*lc
    int* cnts = reinterpret_cast<int*>(smem + geo.off_cnt);
    const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * d;
    auto lword = [&](int t, int w) -> uint32_t& { return lv[2 * (t * nw + w)]; };
    auto cword = [&](int t, int w) -> uint32_t& { return lv[2 * (t * nw + w) + 1]; };
    // the value of node v at level t as the current proposal sees it
    auto seen = [&](int t, int v) -> uint32_t {
        const uint2 x = *reinterpret_cast<const uint2*>(lv + 2 * (t * nw + (v >> 5)));
        return ((x.x ^ x.y) >> (v & 31)) & 1u;
    };
    // neighbours of v: one 8-byte read for d <= 4
    auto nbrs = [&](int v, int (&o)[D > 0 ? D : 16]) {
        if constexpr (D > 0 && D <= 4) {
            const uint2 x = *reinterpret_cast<const uint2*>(rows + v * 4);
            o[0] = (int)(x.x & 0xffffu);
            if constexpr (D > 1) o[1] = (int)(x.x >> 16);
            if constexpr (D > 2) o[2] = (int)(x.y & 0xffffu);
            if constexpr (D > 3) o[3] = (int)(x.y >> 16);
        } else {
            for (int q = 0; q < d; ++q) o[q] = rows[v * rw + q];
        }
    };

    // ---- launch setup: rows, level 0, MT state; then levels 1..T by sweeps in LDS
    for (int64_t q = lane; q < n * d; q += 64) {
        const int64_t v = q / d;
        rows[v * rw + (q - v * d)] = (uint16_t)g[q];
    }
    for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
        const int64_t v = v0 + lane;
        const bool b = v < n && (s[v * W + col] & rbit);
        const u64 m = __ballot(b);
        if (lane < 2) {
            const uint32_t x = (uint32_t)(m >> (32 * lane));
            lword(0, (int)(v0 >> 5) + lane) = x;
            lev0s[(v0 >> 5) + lane] = x;
        }
    }
    for (int k = lane; k < (T + 1) * nw; k += 64) lv[2 * k + 1] = 0u;
    for (int k = lane; k < MT_N; k += 64) mt[k] = st.mt[r * MT_N + k];
    wave_sync();
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > d) ? 1u : ((2 * ones < d) ? 0u : own);
    };
    for (int t = 1; t <= T; ++t) {
        for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
            const int v = (int)(v0 + lane);
            uint32_t nb = 0;
            if (v < n) {
                int nv[D > 0 ? D : 16];
                nbrs(v, nv);
                int ones = 0;
                for (int q = 0; q < d; ++q) ones += (int)seen(t - 1, nv[q]);
                nb = maj(ones, seen(t - 1, v));
            }
            const u64 m = __ballot(nb != 0);
            if (lane < 2) lword(t, (int)(v0 >> 5) + lane) = (uint32_t)(m >> (32 * lane));
        }
        wave_sync();
    }

    // ---- the steps
    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    int64_t k = 0;
    for (; k < nsteps && done == 0; ++k) {
        // randint(low=0, high=n) (code/SA_RRG.py:73): numpy's masked rejection, 64 words per ballot
        int iv = -1;
        while (iv < 0) {
            if (idx >= MT_N) {
                lds_twist(mt, lane);
                idx = 0;
            }
            const int q = idx + lane;
            uint32_t y = 0;
            bool ok = false;
            if (q < MT_N) {
                y = mt_temper(mt[q]) & mask;
                ok = y <= rng;
            }
            const u64 bal = __ballot(ok);
            if (bal) {
                const int f = __ffsll((unsigned long long)bal) - 1;
                iv = __shfl((int)y, f, 64);
                idx += f + 1;
            } else {
                idx += (MT_N - idx < 64) ? MT_N - idx : 64;
            }
        }
        // rand() (code/SA_RRG.py:76): two consecutive words, one read when no twist falls between
        uint32_t w1, w2;
        if (idx + 1 < MT_N) {
            w1 = mt_temper(mt[idx]);
            w2 = mt_temper(mt[idx + 1]);
            idx += 2;
        } else {
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            w1 = mt_temper(mt[idx++]);
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            w2 = mt_temper(mt[idx++]);
        }
        const double u = mt_double(w1, w2);
        // level 0: C_0 = {i}
        const uint32_t old_i = (lword(0, iv >> 5) >> (iv & 31)) & 1u;
        if (lane == 0) {
            cword(0, iv >> 5) |= 1u << (iv & 31);
            lst[0] = (uint32_t)iv;
            cnts[0] = 1;
        }
        wave_sync();
        int last = 0;                          // deepest level with a change
        for (int l = 1; l <= T; ++l) {
            const uint32_t* prev = lst + (l - 1) * lc;
            uint32_t* cur = lst + l * lc;
            const int np = cnts[l - 1];
            const int m = np * (d + 1);
            int nc = 0;
            for (int base = 0; base < m; base += 64) {
                const int q = base + lane;
                bool add = false;
                int cand = 0;
                if (q < m) {
                    const int slot = q / (d + 1), j = q - slot * (d + 1);
                    const int v = (int)prev[slot];
                    cand = (j == 0) ? v : (int)rows[v * rw + j - 1];
                    int nv[D > 0 ? D : 16];
                    nbrs(cand, nv);
                    int ones = 0;
                    for (int e = 0; e < d; ++e) ones += (int)seen(l - 1, nv[e]);
                    const uint32_t nb = maj(ones, seen(l - 1, cand));
                    const uint32_t bit = 1u << (cand & 31);
                    if (nb != ((lword(l, cand >> 5) >> (cand & 31)) & 1u)) {
                        // first mark of cand at level l (candidates repeat)
                        add = (atomicOr(&cword(l, cand >> 5), bit) & bit) == 0u;
                    }
                }
                const u64 bal = __ballot(add);
                if (add) cur[nc + __popcll(bal & ((1ull << lane) - 1ull))] = (uint32_t)cand;
                nc += __popcll(bal);
            }
            if (lane == 0) cnts[l] = nc;
            wave_sync();
            if (nc == 0) break;
            last = l;
        }
        // sum(s_end(flipped)) - sum(s_end): every node of C_T turned to its complement
        int64_t ds = 0;
        if (last == T) {
            const uint32_t* lt = lst + T * lc;
            for (int q = lane; q < cnts[T]; q += 64) {
                const int v = (int)lt[q];
                ds += ((lword(T, v >> 5) >> (v & 31)) & 1u) ? -2 : 2;
            }
            ds = wave_sum(ds);
        }
        const int64_t sum_new = sum_end + ds;
        // delta_H (code/SA_RRG.py:37), same operation order, no contraction
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * a) * si;
        const double t2 = b * (double)(sum_end - sum_new);
        const double dE = (t1 + t2) / (double)n;
        const double e = exp(-dE);
        const double prob = (e < 1.0) ? e : 1.0;                    // (code/SA_RRG.py:75)
        const bool acc = u < prob;                                  // (code/SA_RRG.py:76)
        if (e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e)) ++ties;
        // accepted (code/SA_RRG.py:77): marked bits into the levels; always: clear the marks
        for (int l = 0; l <= last; ++l) {
            const uint32_t* cl = lst + l * lc;
            for (int q = lane; q < cnts[l]; q += 64) {
                const int v = (int)cl[q];
                const uint32_t bit = 1u << (v & 31);
                if (acc) atomicXor(&lword(l, v >> 5), bit);
                atomicAnd(&cword(l, v >> 5), ~bit);
            }
        }
        if (acc) sum_end = sum_new;
        if (a < a_cap) a = par_a * a;                               // (code/SA_RRG.py:80-81)
        if (b < b_cap) b = par_b * b;
        t += 1;                                                     // (code/SA_RRG.py:82)
        if (t > t_cap) done = 2;                                    // (code/SA_RRG.py:84)
        else if (sum_end == n) done = 1;                            // m(s_endstate(s)) == 1
        if (lane == 0) {
            if (st.tr_i) st.tr_i[k * R + r] = iv;
            if (st.tr_acc) st.tr_acc[k * R + r] = acc ? 1 : 0;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = dE;
        }
        wave_sync();
    }
    // steps of this launch after the replica finished
    if (lane == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    // ---- write back: changed configuration bits, the stream, the replica state
    for (int64_t v0 = 0; v0 < n; v0 += 64) {
        const int v = (int)(v0 + lane);
        if (v < n && (((lword(0, v >> 5) ^ lev0s[v >> 5]) >> (v & 31)) & 1u))
            atomicXor((unsigned long long*)&s[(int64_t)v * W + col], (unsigned long long)rbit);
    }
    for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = mt[q];
    if (lane == 0) {
        st.mt_idx[r] = idx;
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}


// ---------------------------------------------------------------------------
// Latency form for d <= 4 (k_sa_lds_fast<D, T>): the same LDS image and the
// same change sets, but a proposal's step is a chain of few LDS round trips.
// One wave serves one replica, so a step IS its chain of dependent LDS
// accesses (k_sa_lds: ~20 at p = 3 -- list and count reads after every
// level, a mark for C_0, the stream words read per draw).  Here:
//   * proposals are parsed 64 stream words at a time: every lane tempers one
//     word, one ballot marks the randint-acceptable ones, and a scalar scan
//     (first set bit, two readlanes for rand()'s words) cuts the window into
//     up to 21 (i, u) pairs kept one per lane -- ~1/17 of a round trip per
//     proposal; a pair that would cross a twist is drawn serially; the stream
//     index handed back is the end of the last proposal consumed, numpy's;
//   * C_0 = {i} needs no mark: level-0 values are read as cached bit XOR
//     (v == i);
//   * C_t lives in lanes (candidate + a ballot mask): the candidates of level
//     t+1 are gathered from the member lanes by ds_bpermute (no LDS list, no
//     count read), the members' neighbour rows come along (read at level t);
//     marks dedup repeated candidates by the atomicOr's return, as before;
//   * sum(s_end) changes by a wave reduction over the lanes of C_T, and the
//     clears / accepted XORs are issued from the same lanes.
// A level whose candidates exceed one wave (|C_{t-1}| (d+1) > 64) falls back
// to the LDS lists of k_sa_lds for the rest of the step (the lists are written
// on every level for that purpose).  Same draws, accepts and state as k_sa_lds.
template <int D, int T, bool TRACE>
__global__ void __launch_bounds__(64) k_sa_lds_fast(const int32_t* __restrict__ adj, int64_t n, int64_t R,
                                                    int64_t W, u64* __restrict__ s, mjx_sa_state st, int64_t nsteps,
                                                    double par_a, double par_b, double a_cap, double b_cap,
                                                    int64_t t_cap, Geo geo) {
    static_assert(D >= 1 && D <= 4 && T >= 1 && T <= kMaxT, "fast LDS SA: d <= 4");
    constexpr int DP1 = D + 1;
    constexpr int MAXM = 64 / DP1;                 // members of C_{t-1} one wave can expand
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = threadIdx.x;
    const int64_t r = blockIdx.x;
    const int64_t col = r >> 6;
    const u64 rbit = 1ull << (r & 63);
    const int nw = geo.nw, lc = geo.lc;
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lv = reinterpret_cast<uint32_t*>(smem + geo.off_lev);
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    uint32_t* lst = reinterpret_cast<uint32_t*>(smem + geo.off_list);
    const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * D;
    auto lword = [&](int t, int w) -> uint32_t& { return lv[2 * (t * nw + w)]; };
    auto cword = [&](int t, int w) -> uint32_t& { return lv[2 * (t * nw + w) + 1]; };
    auto seen = [&](int t, int v) -> uint32_t {
        const uint2 x = *reinterpret_cast<const uint2*>(lv + 2 * (t * nw + (v >> 5)));
        return ((x.x ^ x.y) >> (v & 31)) & 1u;
    };
    auto nbrs = [&](int v, int (&o)[D]) {
        const uint2 x = *reinterpret_cast<const uint2*>(rows + v * 4);
        o[0] = (int)(x.x & 0xffffu);
        if constexpr (D > 1) o[1] = (int)(x.x >> 16);
        if constexpr (D > 2) o[2] = (int)(x.y & 0xffffu);
        if constexpr (D > 3) o[3] = (int)(x.y >> 16);
    };
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
    };

    // ---- launch setup (as k_sa_lds)
    for (int64_t q = lane; q < n * D; q += 64) {
        const int64_t v = q / D;
        rows[v * 4 + (q - v * D)] = (uint16_t)g[q];
    }
    for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
        const int64_t v = v0 + lane;
        const bool b = v < n && (s[v * W + col] & rbit);
        const u64 m = __ballot(b);
        if (lane < 2) {
            const uint32_t x = (uint32_t)(m >> (32 * lane));
            lword(0, (int)(v0 >> 5) + lane) = x;
            lev0s[(v0 >> 5) + lane] = x;
        }
    }
    for (int k = lane; k < (T + 1) * nw; k += 64) lv[2 * k + 1] = 0u;
    for (int k = lane; k < MT_N; k += 64) mt[k] = st.mt[r * MT_N + k];
    wave_sync();
    for (int t = 1; t <= T; ++t) {
        for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
            const int v = (int)(v0 + lane);
            uint32_t nb = 0;
            if (v < n) {
                int nv[D];
                nbrs(v, nv);
                int ones = 0;
#pragma unroll
                for (int q = 0; q < D; ++q) ones += (int)seen(t - 1, nv[q]);
                nb = maj(ones, seen(t - 1, v));
            }
            const u64 m = __ballot(nb != 0);
            if (lane < 2) lword(t, (int)(v0 >> 5) + lane) = (uint32_t)(m >> (32 * lane));
        }
        wave_sync();
    }

    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    double inv_n = 1.0 / (double)n;                       // screening only (dE itself divides)
    // the float64 schedule lives in VGPRs (its arithmetic is vector anyway):
    // the scalar file is what the step's control flow needs
    asm volatile("" : "+v"(a), "+v"(b), "+v"(par_a), "+v"(par_b), "+v"(a_cap), "+v"(b_cap), "+v"(inv_n));

    // ---- proposal windows: lane j holds proposal j of the current window
    int pb_i = 0, pb_end = 0;
    uint32_t pb_w1 = 0, pb_w2 = 0;
    double pb_u = 0.0;
    int npend = 0, pk = 0;
    auto refill = [&]() {
        npend = 0;
        pk = 0;
        while (npend == 0) {
            if (idx >= MT_N) {
                lds_twist(mt, lane);
                idx = 0;
            }
            const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
            uint32_t tw = 0, y = 0;
            bool ok = false;
            if (lane < lim) {
                tw = mt_temper(mt[idx + lane]);
                y = tw & mask;
                ok = y <= rng;
            }
            const u64 okm = __ballot(ok);
            int pos = 0;
            while (pos < 64) {
                const u64 m = okm >> pos;
                if (!m) break;
                const int f = pos + __ffsll((unsigned long long)m) - 1;
                if (f + 2 >= lim) break;
                const int iv = __builtin_amdgcn_readlane((int)y, f);
                const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)tw, f + 1);
                const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)tw, f + 2);
                if (lane == npend) { pb_i = iv; pb_w1 = w1; pb_w2 = w2; pb_end = idx + f + 3; }
                ++npend;
                pos = f + 3;
            }
            if (npend > 0) { idx += pos; break; }
            if (!okm) { idx += lim; continue; }                  // every word rejected by randint
            const int f = __ffsll((unsigned long long)okm) - 1;
            if (f > 0) { idx += f; continue; }                   // rejected words before the next i
            // i is the window's first word and rand()'s two words cross the end of the
            // state: the serial draw twists between them, as numpy does
            const int iv = __builtin_amdgcn_readlane((int)y, 0);
            idx += 1;
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            const uint32_t w1 = mt_temper(mt[idx]);
            idx += 1;
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            const uint32_t w2 = mt_temper(mt[idx]);
            idx += 1;
            if (lane == 0) { pb_i = iv; pb_w1 = w1; pb_w2 = w2; pb_end = idx; }
            npend = 1;
        }
        pb_u = mt_double(pb_w1, pb_w2);                       // rand() of every proposal at once
    };

    // per level: the candidate a lane holds, its cached bit, whether it is in
    // C_l (fast levels), or the list count (levels taken by the LDS-list path)
    int lc_c[T + 1];
    uint32_t lc_v[T + 1];
    bool lc_in[T + 1];
    int lc_n[T + 1];
    bool lc_fast[T + 1];
    // the next proposal's adjacency rows (static), read during this step
    int ri_n[D], nv_n[D];
    bool pf = false;
    bool drew = false;
    int64_t k = 0;
#ifdef MJX_SA_PROF
    unsigned long long _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _t0 = __builtin_amdgcn_s_memtime();
#endif
    for (; k < nsteps && done == 0; ++k) {
        if (pk == npend) refill();
        drew = true;
        const int iv = __builtin_amdgcn_readlane(pb_i, pk);
        const double u = __builtin_bit_cast(
            double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(uint64_t, pb_u) >> 32), pk) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)__builtin_bit_cast(uint64_t, pb_u), pk));
        ++pk;
        LDS_STAMP(0);
        const uint32_t lw0 = lword(0, iv >> 5);
        const uint32_t old_i = (lw0 >> (iv & 31)) & 1u;
        // ---- level 1: i and its neighbours, values of level 0 with i flipped; a
        // repeated row entry (not in a simple graph) is dropped by lane compares
        int cand, nv[D];
        {
            int ri[D];
            if (pf) {
#pragma unroll
                for (int e = 0; e < D; ++e) { ri[e] = ri_n[e]; nv[e] = nv_n[e]; }
            } else {
                nbrs(iv, ri);
            }
            cand = iv;
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (lane == q + 1) cand = ri[q];
            bool dup = lane > 0 && cand == iv;
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (q + 1 < lane) dup |= ri[q] == cand;
            if (!pf) nbrs(cand, nv);
            // the next proposal's row (its neighbours' rows follow after the levels)
            pf = pk < npend;
            if (pf) nbrs(__builtin_amdgcn_readlane(pb_i, pk), ri_n);
            int ones = 0;
#pragma unroll
            for (int e = 0; e < D; ++e) ones += (int)(((lword(0, nv[e] >> 5) >> (nv[e] & 31)) & 1u) ^ (nv[e] == iv));
            const uint32_t own = ((lword(0, cand >> 5) >> (cand & 31)) & 1u) ^ (cand == iv);
            const uint32_t nb = maj(ones, own);
            const uint32_t cur = (lword(1, cand >> 5) >> (cand & 31)) & 1u;
            const bool chg = lane <= D && !dup && nb != cur;
            const u64 m = __ballot(chg);
            if (chg) {
                atomicOr(&cword(1, cand >> 5), 1u << (cand & 31));
                lst[lc + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)cand;
            }
            lc_c[1] = cand;
            lc_v[1] = cur;
            lc_in[1] = chg;
            lc_n[1] = __popcll(m);
            lc_fast[1] = true;
        }
        int last = lc_n[1] ? 1 : 0;
        LDS_STAMP(1);
        // sum(s_end(flipped)) - sum(s_end): every node of C_T turned to its complement,
        // +2 for a -1 -> +1 change, -2 for +1 -> -1 (counted by ballots)
        int64_t ds = 0;
        if (T == 1 && last == 1) {
            const bool in = lc_in[1];
            ds = 2 * ((int64_t)__popcll(__ballot(in && lc_v[1] == 0u)) - (int64_t)__popcll(__ballot(in && lc_v[1] != 0u)));
        }
        bool fast = true;
#pragma unroll
        for (int l = 2; l <= T; ++l) {
            if (last != l - 1) break;
            wave_sync();                                     // marks of C_{l-1} before they are read
            const u64 pm = __ballot(lc_in[l - 1]);
            const int np = lc_n[l - 1];
            int nc = 0;
            if (fast && np <= MAXM) {
                // candidates: member s = lane / (d+1) of C_{l-1}, j = 0 the member
                // itself, j > 0 its j-th neighbour; member s's lane: every member
                // pushes its lane id to lane (its rank) by ds_permute (others to an
                // unused lane), lane s's entry is pulled by ds_bpermute
                const int sl = lane / DP1, j = lane - sl * DP1;
                const int rank = __popcll(pm & ((1ull << lane) - 1ull));
                const int slot = __builtin_amdgcn_ds_permute((lc_in[l - 1] ? rank : 63) * 4, lane);
                const int src = __builtin_amdgcn_ds_bpermute(sl * 4, slot) & 63;
                const int mc = __shfl(cand, src, 64);
                int pn[D];
#pragma unroll
                for (int e = 0; e < D; ++e) pn[e] = __shfl(nv[e], src, 64);
                const bool act = sl < np;
                int c2 = mc;
#pragma unroll
                for (int e = 0; e < D; ++e)
                    if (j == e + 1) c2 = pn[e];
                if (!act) c2 = iv;
                int nv2[D];
                nbrs(c2, nv2);
                int ones = 0;
#pragma unroll
                for (int e = 0; e < D; ++e) ones += (int)seen(l - 1, nv2[e]);
                const uint32_t nb = maj(ones, seen(l - 1, c2));
                const uint32_t cur = (lword(l, c2 >> 5) >> (c2 & 31)) & 1u;
                const bool chg = act && nb != cur;
                const uint32_t bit = 1u << (c2 & 31);
                bool add = chg;
                if (l == T) {
                    // the last level counts distinct nodes: the first mark wins
                    if (chg) add = (atomicOr(&cword(l, c2 >> 5), bit) & bit) == 0u;
                } else if (chg) {
                    // inner levels keep repeats (marks, clears and the accepted
                    // values are idempotent; the next level's dedup absorbs them)
                    atomicOr(&cword(l, c2 >> 5), bit);
                }
                const u64 m = __ballot(add);
                if (add) lst[l * lc + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)c2;
                nc = __popcll(m);
                cand = c2;
#pragma unroll
                for (int e = 0; e < D; ++e) nv[e] = nv2[e];
                lc_c[l] = c2;
                lc_v[l] = cur;
                lc_in[l] = add;
                lc_fast[l] = true;
                if (l == T)
                    ds = 2 * ((int64_t)__popcll(__ballot(add && cur == 0u)) - (int64_t)__popcll(__ballot(add && cur != 0u)));
            } else {
                // the LDS-list path of k_sa_lds (lists of every level are in lst;
                // this path dedups every level it builds)
                fast = false;
                const uint32_t* prev = lst + (l - 1) * lc;
                uint32_t* curl = lst + l * lc;
                const int m = np * DP1;
                int64_t dsl = 0;
                for (int base = 0; base < m; base += 64) {
                    const int q = base + lane;
                    bool add = false;
                    int cd = 0;
                    uint32_t cur = 0;
                    if (q < m) {
                        const int slot = q / DP1, j = q - slot * DP1;
                        const int v = (int)prev[slot];
                        cd = (j == 0) ? v : (int)rows[v * 4 + j - 1];
                        int nv2[D];
                        nbrs(cd, nv2);
                        int ones = 0;
#pragma unroll
                        for (int e = 0; e < D; ++e) ones += (int)seen(l - 1, nv2[e]);
                        const uint32_t nb = maj(ones, seen(l - 1, cd));
                        const uint32_t bit = 1u << (cd & 31);
                        cur = (lword(l, cd >> 5) >> (cd & 31)) & 1u;
                        if (nb != cur) add = (atomicOr(&cword(l, cd >> 5), bit) & bit) == 0u;
                    }
                    const u64 bal = __ballot(add);
                    if (add) curl[nc + __popcll(bal & ((1ull << lane) - 1ull))] = (uint32_t)cd;
                    nc += __popcll(bal);
                    dsl += 2 * ((int64_t)__popcll(__ballot(add && cur == 0u)) - (int64_t)__popcll(__ballot(add && cur != 0u)));
                }
                if (l == T) ds = dsl;
                lc_fast[l] = false;
                wave_sync();
            }
            lc_n[l] = nc;
            LDS_STAMP(l < 4 ? l : 4);
            if (nc == 0) break;
            last = l;
        }
        if (last != T) ds = 0;
        // the next proposal's neighbour rows
        if (pf) {
            int cn = __builtin_amdgcn_readlane(pb_i, pk);
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (lane == q + 1) cn = ri_n[q];
            nbrs(cn, nv_n);
        }
        const int64_t sum_new = sum_end + ds;
        // delta_H (code/SA_RRG.py:37), same operation order, no contraction
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * a) * si;
        const double t2 = b * (double)(sum_end - sum_new);
        const double num = t1 + t2;
        // u < min(1, exp(-dE)) (code/SA_RRG.py:75-76) decided by an fp32 exp
        // wherever u is farther from it than that exp's error (|x| * 2^-24 from
        // rounding x, a few ulp from the exp itself: 1e-6 (1 + |x|) relative
        // covers both); otherwise, and for the trace, the float64 dE and exp of
        // the reference, unchanged.  Same decision bit for bit.
        const float xf = (float)(-num * inv_n);
        const float ef = __expf(xf);
        const float mg = ef * (1e-6f * (1.0f + fabsf(xf))) + 1e-37f;
        bool acc;
        double dE = 0.0;
        if (fabs(u - (double)ef) > (double)mg) {
            acc = u < (double)ef;
            if (TRACE && st.tr_dE) dE = num / (double)n;
        } else {
            dE = num / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;                // (code/SA_RRG.py:75)
            acc = u < prob;                                         // (code/SA_RRG.py:76)
            if (e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e)) ++ties;
        }
        LDS_STAMP(5);
        // accepted (code/SA_RRG.py:77): every node of C_0..C_last takes its new value
        // (the complement of its cached one: set or clear, idempotent for the repeats
        // of inner fast levels; list levels are duplicate-free and flip); always:
        // clear the marks
        if (acc && lane == 0) atomicXor(&lword(0, iv >> 5), 1u << (iv & 31));
#pragma unroll
        for (int l = 1; l <= T; ++l) {
            if (l > last) break;
            if (lc_fast[l]) {
                if (lc_in[l]) {
                    const int v = lc_c[l];
                    const uint32_t bit = 1u << (v & 31);
                    if (acc) {
                        if (lc_v[l]) atomicAnd(&lword(l, v >> 5), ~bit);
                        else atomicOr(&lword(l, v >> 5), bit);
                    }
                    cword(l, v >> 5) = 0u;            // every mark of the word is this step's
                }
            } else {
                const uint32_t* cl = lst + l * lc;
                for (int q = lane; q < lc_n[l]; q += 64) {
                    const int v = (int)cl[q];
                    const uint32_t bit = 1u << (v & 31);
                    if (acc) atomicXor(&lword(l, v >> 5), bit);
                    cword(l, v >> 5) = 0u;            // every mark of the word is this step's
                }
            }
        }
        if (acc) sum_end = sum_new;
        if (a < a_cap) a = par_a * a;                               // (code/SA_RRG.py:80-81)
        if (b < b_cap) b = par_b * b;
        t += 1;                                                     // (code/SA_RRG.py:82)
        if (t > t_cap) done = 2;                                    // (code/SA_RRG.py:84)
        else if (sum_end == n) done = 1;                            // m(s_endstate(s)) == 1
        if (TRACE && lane == 0) {
            if (st.tr_i) st.tr_i[k * R + r] = iv;
            if (st.tr_acc) st.tr_acc[k * R + r] = acc ? 1 : 0;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = dE;
        }
        wave_sync();
        LDS_STAMP(6);
    }
#ifdef MJX_SA_PROF
    if (lane == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&mjx_sa_lds_prof[q], _acc[q]);
#endif
    // the stream index numpy would hold: the end of the last proposal consumed
    if (drew) idx = __builtin_amdgcn_readlane(pb_end, pk - 1);
    if (TRACE && lane == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    for (int64_t v0 = 0; v0 < n; v0 += 64) {
        const int v = (int)(v0 + lane);
        if (v < n && (((lword(0, v >> 5) ^ lev0s[v >> 5]) >> (v & 31)) & 1u))
            atomicXor((unsigned long long*)&s[(int64_t)v * W + col], (unsigned long long)rbit);
    }
    for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = mt[q];
    if (lane == 0) {
        st.mt_idx[r] = idx;
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}


// ---------------------------------------------------------------------------
// Two proposals per step (k_sa_lds_pair<D, T>, d <= 4): the lane-held step
// of k_sa_lds_fast is ALU-issue bound on its one wave (a few hundred VALU /
// SALU instructions per level, 5-20 lanes busy), so the wave's two halves
// evaluate the next two proposals A = k and B = k+1 of the replica at once,
// both against the current levels, each with its own mark plane (a level
// word entry is {level, marks A, marks B, -}, one 16-B read).  B stands
// unless A is accepted and A may have changed something B read: B's lanes
// read, beside every level-(l-1) value they use, A's level-(l-1) marks, and a
// node B reads at level l-1 or whose cached level-l value B reads (one of
// B's candidates) can change under A only if it or one of its neighbours is
// in A's C_{l-1} -- exactly the nodes B reads; level 0 (no marks) by
// comparing with i_A.  The acceptance of each is its own (dE depends on the
// step's schedule value and its own ds only), so both are decided at once;
// A's consequences (stop, t cap) are resolved first, then B is taken or
// drawn again next step.  Proposal windows carry a leftover proposal into
// the next window when no twist can fall between them.  A half whose C_{l-1}
// exceeds 32 / (d+1) members takes its LDS lists for the rest of the step
// (3 % of the steps at p = 3; two candidate slots per lane instead measured
// slower).  Same draws, accepts and state as k_sa_lds.
template <int D, int T, bool TRACE>
__global__ void __launch_bounds__(64) k_sa_lds_pair(const int32_t* __restrict__ adj, int64_t n, int64_t R,
                                                    int64_t W, u64* __restrict__ s, mjx_sa_state st, int64_t nsteps,
                                                    double par_a, double par_b, double a_cap, double b_cap,
                                                    int64_t t_cap, Geo geo) {
    static_assert(D >= 1 && D <= 4 && T >= 1 && T <= kMaxT, "paired LDS SA: d <= 4");
    constexpr int DP1 = D + 1;
    constexpr int MAXM = 32 / DP1;                 // members of C_{t-1} one half-wave can expand
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = threadIdx.x;
    const int h = lane >> 5, hl = lane & 31;
    const u64 hmask = h ? 0xffffffff00000000ull : 0x00000000ffffffffull;
    const u64 ltmask = (1ull << lane) - 1ull;
    const int64_t r = blockIdx.x;
    const int64_t col = r >> 6;
    const u64 rbit = 1ull << (r & 63);
    const int nw = geo.nw, lc = geo.lc;
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lv = reinterpret_cast<uint32_t*>(smem + geo.off_lev);       // {level, marks A, marks B, -}
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    uint32_t* lsth = reinterpret_cast<uint32_t*>(smem + geo.off_list) + h * (T + 1) * lc;   // this half's lists
    const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * D;
    auto lword = [&](int t, int w) -> uint32_t& { return lv[4 * (t * nw + w)]; };
    auto mword = [&](int t, int w, int pl) -> uint32_t& { return lv[4 * (t * nw + w) + 1 + pl]; };
    // node v at level t as this half's proposal sees it, and A's mark on it
    auto look = [&](int t, int v, uint32_t& val, uint32_t& amark) {
        const uint4 x = *reinterpret_cast<const uint4*>(lv + 4 * (t * nw + (v >> 5)));
        const int sh = v & 31;
        val = ((x.x ^ (h ? x.z : x.y)) >> sh) & 1u;
        amark = (x.y >> sh) & 1u;
    };
    auto nbrs = [&](int v, int (&o)[D]) {
        const uint2 x = *reinterpret_cast<const uint2*>(rows + v * 4);
        o[0] = (int)(x.x & 0xffffu);
        if constexpr (D > 1) o[1] = (int)(x.x >> 16);
        if constexpr (D > 2) o[2] = (int)(x.y & 0xffffu);
        if constexpr (D > 3) o[3] = (int)(x.y >> 16);
    };
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
    };
    auto half_count = [&](bool x) -> int { return __popcll(__ballot(x) & hmask); };

    // ---- launch setup
    for (int64_t q = lane; q < n * D; q += 64) {
        const int64_t v = q / D;
        rows[v * 4 + (q - v * D)] = (uint16_t)g[q];
    }
    for (int k = lane; k < (T + 1) * nw * 4; k += 64) lv[k] = 0u;
    wave_sync();
    for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
        const int64_t v = v0 + lane;
        const bool b = v < n && (s[v * W + col] & rbit);
        const u64 m = __ballot(b);
        if (lane < 2) {
            const uint32_t x = (uint32_t)(m >> (32 * lane));
            lword(0, (int)(v0 >> 5) + lane) = x;
            lev0s[(v0 >> 5) + lane] = x;
        }
    }
    for (int k = lane; k < MT_N; k += 64) mt[k] = st.mt[r * MT_N + k];
    wave_sync();
    for (int t = 1; t <= T; ++t) {
        for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
            const int v = (int)(v0 + lane);
            uint32_t nb = 0;
            if (v < n) {
                int nv[D];
                nbrs(v, nv);
                int ones = 0;
#pragma unroll
                for (int q = 0; q < D; ++q) ones += (int)((lword(t - 1, nv[q] >> 5) >> (nv[q] & 31)) & 1u);
                nb = maj(ones, (lword(t - 1, v >> 5) >> (v & 31)) & 1u);
            }
            const u64 m = __ballot(nb != 0);
            if (lane < 2) lword(t, (int)(v0 >> 5) + lane) = (uint32_t)(m >> (32 * lane));
        }
        wave_sync();
    }

    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    // the pointers the write-back needs are parked in LDS for the steps: kept in
    // scalar registers across the loop they spilled into VGPR lanes (restored by
    // readlanes every step)
    u64* park = reinterpret_cast<u64*>(smem + geo.off_cnt);
    if (lane == 0) {
        park[0] = (u64)s;
        park[1] = (u64)st.mt;
        park[2] = (u64)st.mt_idx;
        park[3] = (u64)st.a;
        park[4] = (u64)st.b;
        park[5] = (u64)st.t;
        park[6] = (u64)st.sum_end;
        park[7] = (u64)st.done;
        park[8] = (u64)st.tr_tie;
        park[9] = (u64)W;
    }
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    double inv_n = 1.0 / (double)n;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(par_a), "+v"(par_b), "+v"(a_cap), "+v"(b_cap), "+v"(inv_n));

    // ---- proposal windows: lane j holds proposal j
    int pb_i = 0, pb_end = 0;
    uint32_t pb_w1 = 0, pb_w2 = 0;
    double pb_u = 0.0;
    int npend = 0, pk = 0;
    // append the proposals of stream windows at lanes npend..; with `one`, at
    // most one window and no twist (a carried proposal's stream must not be
    // twisted away under it)
    auto parse = [&](bool one) {
        for (;;) {
            if (idx >= MT_N) {
                if (one) break;
                lds_twist(mt, lane);
                idx = 0;
            }
            const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
            uint32_t tw = 0, y = 0;
            bool ok = false;
            if (lane < lim) {
                tw = mt_temper(mt[idx + lane]);
                y = tw & mask;
                ok = y <= rng;
            }
            const u64 okm = __ballot(ok);
            int pos = 0, got = 0;
            while (pos < 64 && npend < 64) {
                const u64 m = okm >> pos;
                if (!m) break;
                const int f = pos + __ffsll((unsigned long long)m) - 1;
                if (f + 2 >= lim) break;
                const int iv = __builtin_amdgcn_readlane((int)y, f);
                const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)tw, f + 1);
                const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)tw, f + 2);
                if (lane == npend) { pb_i = iv; pb_w1 = w1; pb_w2 = w2; pb_end = idx + f + 3; }
                ++npend;
                ++got;
                pos = f + 3;
            }
            if (got > 0) { idx += pos; break; }
            if (one) break;
            if (!okm) { idx += lim; continue; }
            const int f = __ffsll((unsigned long long)okm) - 1;
            if (f > 0) { idx += f; continue; }
            const int iv = __builtin_amdgcn_readlane((int)y, 0);
            idx += 1;
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            const uint32_t w1 = mt_temper(mt[idx]);
            idx += 1;
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            const uint32_t w2 = mt_temper(mt[idx]);
            idx += 1;
            if (lane == npend) { pb_i = iv; pb_w1 = w1; pb_w2 = w2; pb_end = idx; }
            ++npend;
            break;
        }
        pb_u = mt_double(pb_w1, pb_w2);
    };
    auto rl_double = [&](double x, int l) -> double {
        const uint64_t bits = __builtin_bit_cast(uint64_t, x);
        return __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(bits >> 32), l) << 32) |
                                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, l));
    };

    int lc_c[T + 1];
    uint32_t lc_v[T + 1];
    bool lc_in[T + 1];
    int lc_n[T + 1];
    bool lc_fast[T + 1];
    bool drew = false;
    int64_t k = 0;
#ifdef MJX_SA_PROF
    unsigned long long _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _t0 = __builtin_amdgcn_s_memtime();
#endif
    while (k < nsteps && done == 0) {
        const int avail = npend - pk;
        if (avail == 1 && idx + 64 <= MT_N) {
            // carry the leftover proposal to lane 0, append one window
            const int ci = __builtin_amdgcn_readlane(pb_i, pk), ce = __builtin_amdgcn_readlane(pb_end, pk);
            const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)pb_w1, pk);
            const uint32_t c2 = (uint32_t)__builtin_amdgcn_readlane((int)pb_w2, pk);
            if (lane == 0) { pb_i = ci; pb_end = ce; pb_w1 = c1; pb_w2 = c2; }
            npend = 1;
            pk = 0;
            parse(true);
        } else if (avail == 0) {
            npend = 0;
            pk = 0;
            parse(false);
            if (npend == 1 && idx + 64 <= MT_N) parse(true);
        }
        drew = true;
        const bool both = npend - pk >= 2 && k + 1 < nsteps;
        const int iA = __builtin_amdgcn_readlane(pb_i, pk);
        const int iB = both ? __builtin_amdgcn_readlane(pb_i, pk + 1) : iA;
        const double uA = rl_double(pb_u, pk);
        const double uB = both ? rl_double(pb_u, pk + 1) : uA;
        const int iv = h ? iB : iA;
        const double u = h ? uB : uA;
        const bool act = h == 0 || both;
        LDS_STAMP(0);
        const uint32_t old_i = (lword(0, iv >> 5) >> (iv & 31)) & 1u;
        bool conf = false;
        // ---- level 1 (per half): i and its neighbours, level 0 with i flipped
        int cand, nv[D];
        int last;
        {
            int ri[D];
            nbrs(iv, ri);
            cand = iv;
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (hl == q + 1) cand = ri[q];
            bool dup = hl > 0 && cand == iv;
#pragma unroll
            for (int q = 0; q < D; ++q)
                if (q + 1 < hl) dup |= ri[q] == cand;
            nbrs(cand, nv);
            const bool live = act && hl <= D && !dup;
            int ones = 0;
            bool hitA = cand == iA;
#pragma unroll
            for (int e = 0; e < D; ++e) {
                ones += (int)(((lword(0, nv[e] >> 5) >> (nv[e] & 31)) & 1u) ^ (nv[e] == iv));
                hitA |= nv[e] == iA;
            }
            if (h == 1 && live && hitA) conf = true;
            const uint32_t own = ((lword(0, cand >> 5) >> (cand & 31)) & 1u) ^ (cand == iv);
            const uint32_t nb = maj(ones, own);
            const uint32_t cur = (lword(1, cand >> 5) >> (cand & 31)) & 1u;
            const bool chg = live && nb != cur;
            const u64 m = __ballot(chg);
            if (chg) {
                atomicOr(&mword(1, cand >> 5, h), 1u << (cand & 31));
                lsth[lc + __popcll(m & hmask & ltmask)] = (uint32_t)cand;
            }
            lc_c[1] = cand;
            lc_v[1] = cur;
            lc_in[1] = chg;
            lc_fast[1] = true;
            lc_n[1] = __popcll(m & hmask);
            last = lc_n[1] ? 1 : 0;
        }
        LDS_STAMP(1);
        int64_t ds = 0;
        if (T == 1 && last == 1) {
            const bool in = lc_in[1];
            ds = 2 * ((int64_t)half_count(in && lc_v[1] == 0u) - (int64_t)half_count(in && lc_v[1] != 0u));
        }
#pragma unroll
        for (int l = 2; l <= T; ++l) {
            lc_in[l] = false;
            lc_fast[l] = true;
            lc_n[l] = 0;
            const bool go = last == l - 1;
            if (!__any(go)) break;
            wave_sync();                                     // marks of C_{l-1} before they are read
            const u64 pm = __ballot(lc_in[l - 1]) & hmask;
            const int np = lc_n[l - 1];
            int nc = 0;
            if (go && np <= MAXM && lc_fast[l - 1]) {
                // candidates: member s = hl / (d+1) of this half's C_{l-1}, j = 0 the
                // member itself, j > 0 its j-th neighbour; member s's lane: every member
                // pushes its lane id to lane 32h + rank by ds_permute (the others to
                // the half's unused lane 32h + 31), lane 32h + s's entry is pulled
                const int sl = hl / DP1, j = hl - sl * DP1;
                const int rank = __popcll(pm & ltmask);
                const int slot = __builtin_amdgcn_ds_permute((h * 32 + (lc_in[l - 1] ? rank : 31)) * 4, lane);
                const int src = __builtin_amdgcn_ds_bpermute((h * 32 + sl) * 4, slot) & 63;
                const int mc = __shfl(cand, src, 64);
                int pn[D];
#pragma unroll
                for (int e = 0; e < D; ++e) pn[e] = __shfl(nv[e], src, 64);
                const bool act2 = sl < np;
                int c2 = mc;
#pragma unroll
                for (int e = 0; e < D; ++e)
                    if (j == e + 1) c2 = pn[e];
                if (!act2) c2 = iv;
                int nv2[D];
                nbrs(c2, nv2);
                int ones = 0;
                uint32_t am = 0, val;
#pragma unroll
                for (int e = 0; e < D; ++e) {
                    uint32_t mk;
                    look(l - 1, nv2[e], val, mk);
                    ones += (int)val;
                    am |= mk;
                }
                uint32_t own, mk;
                look(l - 1, c2, own, mk);
                am |= mk;
                if (h == 1 && act2 && am) conf = true;
                const uint32_t nb = maj(ones, own);
                const uint32_t cur = (lword(l, c2 >> 5) >> (c2 & 31)) & 1u;
                const bool chg = act2 && nb != cur;
                const uint32_t bit = 1u << (c2 & 31);
                bool add = chg;
                if (l == T) {
                    if (chg) add = (atomicOr(&mword(l, c2 >> 5, h), bit) & bit) == 0u;
                } else if (chg) {
                    atomicOr(&mword(l, c2 >> 5, h), bit);
                }
                const u64 m = __ballot(add);
                if (add) lsth[l * lc + __popcll(m & hmask & ltmask)] = (uint32_t)c2;
                nc = __popcll(m & hmask);
                cand = c2;
#pragma unroll
                for (int e = 0; e < D; ++e) nv[e] = nv2[e];
                lc_c[l] = c2;
                lc_v[l] = cur;
                lc_in[l] = add;
                if (l == T) ds = 2 * ((int64_t)__popcll(__ballot(add && cur == 0u) & hmask) -
                                      (int64_t)__popcll(__ballot(add && cur != 0u) & hmask));
            } else if (go) {
                // this half's LDS-list path (its lists hold every level; deduped here)
                const uint32_t* prev = lsth + (l - 1) * lc;
                uint32_t* curl = lsth + l * lc;
                const int m = np * DP1;
                int64_t dsl = 0;
                for (int base = 0; base < m; base += 32) {
                    const int q = base + hl;
                    bool add = false;
                    int cd = 0;
                    uint32_t cur = 0;
                    if (q < m) {
                        const int slot = q / DP1, j = q - slot * DP1;
                        const int v = (int)prev[slot];
                        cd = (j == 0) ? v : (int)rows[v * 4 + j - 1];
                        int nv2[D];
                        nbrs(cd, nv2);
                        int ones = 0;
                        uint32_t am = 0, val, mk;
#pragma unroll
                        for (int e = 0; e < D; ++e) {
                            look(l - 1, nv2[e], val, mk);
                            ones += (int)val;
                            am |= mk;
                        }
                        uint32_t own;
                        look(l - 1, cd, own, mk);
                        am |= mk;
                        if (h == 1 && am) conf = true;
                        const uint32_t nb = maj(ones, own);
                        const uint32_t bit = 1u << (cd & 31);
                        cur = (lword(l, cd >> 5) >> (cd & 31)) & 1u;
                        if (nb != cur) add = (atomicOr(&mword(l, cd >> 5, h), bit) & bit) == 0u;
                    }
                    const u64 bal = __ballot(add) & hmask;
                    if (add) curl[nc + __popcll(bal & ltmask)] = (uint32_t)cd;
                    nc += __popcll(bal);
                    dsl += 2 * ((int64_t)__popcll(__ballot(add && cur == 0u) & hmask) -
                                (int64_t)__popcll(__ballot(add && cur != 0u) & hmask));
                }
                if (l == T) ds = dsl;
                lc_fast[l] = false;
            }
            wave_sync();
            if (go) {
                lc_n[l] = nc;
                if (nc > 0) last = l;
            }
            LDS_STAMP(l < 4 ? l : 4);
        }
        if (last != T) ds = 0;
        // ---- delta_H and the Metropolis test of each half's proposal (code/SA_RRG.py:37,74-76)
        const double aA = a, bA = b;
        const double aB = (a < a_cap) ? par_a * a : a;               // the schedule after step A (:80-81)
        const double bB = (b < b_cap) ? par_b * b : b;
        const double ah = h ? aB : aA, bh = h ? bB : bA;
        const double anx = (ah < a_cap) ? par_a * ah : ah;          // the schedule after this half's step
        const double bnx = (bh < b_cap) ? par_b * bh : bh;
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * ah) * si;
        const double t2 = bh * (double)(-ds);
        const double num = t1 + t2;
        const float xf = (float)(-num * inv_n);
        const float ef = __expf(xf);
        const float mg = ef * (1e-6f * (1.0f + fabsf(xf))) + 1e-37f;
        bool acc, tie = false;
        double dE = 0.0;
        if (fabs(u - (double)ef) > (double)mg) {
            acc = u < (double)ef;
            if (TRACE && st.tr_dE) dE = num / (double)n;
        } else {
            dE = num / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;
            acc = u < prob;
            tie = e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e);
        }
        LDS_STAMP(5);
        // ---- resolve: A first; B stands unless A is accepted and touched B's reads
        const bool accA = __builtin_amdgcn_readlane((int)acc, 0) != 0;
        const bool accB = __builtin_amdgcn_readlane((int)acc, 32) != 0;
        const int64_t dsA = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)ds >> 32), 0) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ds, 0));
        const int64_t dsB = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)ds >> 32), 32) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ds, 32));
        const bool confB = (__ballot(conf) & 0xffffffff00000000ull) != 0ull;
        const int64_t sumA = accA ? sum_end + dsA : sum_end;
        const int64_t tA = t + 1;
        const int doneA = (tA > t_cap) ? 2 : ((sumA == n) ? 1 : 0);             // (:84), m(s_endstate) == 1
        const bool takeB = both && doneA == 0 && !(accA && confB);
#ifdef MJX_SA_PROF
        _acc[7] += (both ? 1000 : 0) + (takeB ? 1000000 : 0);   // pairs tried (x1e3), B taken (x1e6)
#endif
        ties += (__builtin_amdgcn_readlane((int)tie, 0) ? 1 : 0) + ((takeB && __builtin_amdgcn_readlane((int)tie, 32)) ? 1 : 0);
        const bool mine = h ? (takeB && accB) : accA;
        if (lane == 0 && accA) atomicXor(&lword(0, iA >> 5), 1u << (iA & 31));
        if (lane == 32 && takeB && accB) atomicXor(&lword(0, iB >> 5), 1u << (iB & 31));
#pragma unroll
        for (int l = 1; l <= T; ++l) {
            if (l <= last) {
                if (lc_fast[l]) {
                    if (lc_in[l]) {
                        const int v = lc_c[l];
                        const uint32_t bit = 1u << (v & 31);
                        if (mine) {
                            if (lc_v[l]) atomicAnd(&lword(l, v >> 5), ~bit);
                            else atomicOr(&lword(l, v >> 5), bit);
                        }
                        mword(l, v >> 5, h) = 0u;         // every mark of the word is this step's
                    }
                } else {
                    const uint32_t* cl = lsth + l * lc;
                    for (int q = hl; q < lc_n[l]; q += 32) {
                        const int v = (int)cl[q];
                        const uint32_t bit = 1u << (v & 31);
                        if (mine) atomicXor(&lword(l, v >> 5), bit);
                        mword(l, v >> 5, h) = 0u;         // every mark of the word is this step's
                    }
                }
            }
        }
        // step A (code/SA_RRG.py:77-84)
        sum_end = sumA;
        a = aB;
        b = bB;
        t = tA;
        done = doneA;
        if (TRACE && lane == 0) {
            if (st.tr_i) st.tr_i[k * R + r] = iA;
            if (st.tr_acc) st.tr_acc[k * R + r] = accA ? 1 : 0;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = dE;
        }
        ++k;
        ++pk;
        if (takeB) {
            if (accB) sum_end += dsB;
            a = __shfl(anx, 32, 64);
            b = __shfl(bnx, 32, 64);
            t += 1;
            if (t > t_cap) done = 2;
            else if (sum_end == n) done = 1;
            if (TRACE && lane == 32) {
                if (st.tr_i) st.tr_i[k * R + r] = iB;
                if (st.tr_acc) st.tr_acc[k * R + r] = accB ? 1 : 0;
                if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
                if (st.tr_dE) st.tr_dE[k * R + r] = dE;
            }
            ++k;
            ++pk;
        }
        wave_sync();
        LDS_STAMP(6);
    }
#ifdef MJX_SA_PROF
    if (lane == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&mjx_sa_lds_prof[q], _acc[q]);
#endif
    if (drew) idx = __builtin_amdgcn_readlane(pb_end, pk - 1);
    if (TRACE && lane == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    wave_sync();
    u64* const ps = (u64*)park[0];
    const int64_t Wp = (int64_t)park[9];
    const int64_t rr = blockIdx.x;
    for (int64_t v0 = 0; v0 < n; v0 += 64) {
        const int v = (int)(v0 + lane);
        if (v < n && (((lword(0, v >> 5) ^ lev0s[v >> 5]) >> (v & 31)) & 1u))
            atomicXor((unsigned long long*)&ps[(int64_t)v * Wp + (rr >> 6)], 1ull << (rr & 63));
    }
    uint32_t* const pmt = (uint32_t*)park[1];
    for (int q = lane; q < MT_N; q += 64) pmt[rr * MT_N + q] = mt[q];
    if (lane == 0) {
        ((int32_t*)park[2])[rr] = idx;
        ((double*)park[3])[rr] = a;
        ((double*)park[4])[rr] = b;
        ((int64_t*)park[5])[rr] = t;
        ((int64_t*)park[6])[rr] = sum_end;
        ((int32_t*)park[7])[rr] = done;
        int32_t* const tie = (int32_t*)park[8];
        if (tie) tie[rr] += ties;
    }
}


// ---------------------------------------------------------------------------
// p + c - 1 = 1 (configs[0], SA_RRG.py with p = c = 1): NQ proposals per step
// (k_sa_lds_multi<D, NQ>, NQ groups of 64/NQ >= d+1 lanes).  At one level the
// light cone of proposal q is i_q and its neighbours (C_1 needs no marks:
// those candidates are distinct) and what it reads is level 0 on the radius-2
// ball and the cached level 1 of the radius-1 ball; an earlier proposal j
// changes level 0 at i_j and level 1 only inside N[i_j], so q's evaluation
// stands after an accepted j unless i_j is one of the nodes q's lanes read at
// level 0 (a candidate or a neighbour of one) -- which also covers q's reads
// of level 1 (a candidate in N[i_j] has i_j among its neighbours).  The taken
// proposals are a prefix: the first one that conflicts with an accepted
// earlier one, or follows a stop, and all after it are drawn again next step.
template <int D, int NQ, bool TRACE>
__global__ void __launch_bounds__(64) k_sa_lds_multi(const int32_t* __restrict__ adj, int64_t n, int64_t R,
                                                     int64_t W, u64* __restrict__ s, mjx_sa_state st, int64_t nsteps,
                                                     double par_a, double par_b, double a_cap, double b_cap,
                                                     int64_t t_cap, Geo geo) {
    static_assert(D >= 1 && D <= 4 && NQ >= 2 && 64 / NQ >= D + 1, "multi-proposal LDS SA: d <= 4, T = 1");
    constexpr int G = 64 / NQ;
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = threadIdx.x;
    const int gq = lane / G, gl = lane % G;
    const int64_t r = blockIdx.x;
    const int nw = geo.nw;
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lv = reinterpret_cast<uint32_t*>(smem + geo.off_lev);       // {level, marks} (marks unused)
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * D;
    auto lword = [&](int t, int w) -> uint32_t& { return lv[2 * (t * nw + w)]; };
    auto bit_of = [&](int t, int v) -> uint32_t { return (lword(t, v >> 5) >> (v & 31)) & 1u; };
    auto nbrs = [&](int v, int (&o)[D]) {
        const uint2 x = *reinterpret_cast<const uint2*>(rows + v * 4);
        o[0] = (int)(x.x & 0xffffu);
        if constexpr (D > 1) o[1] = (int)(x.x >> 16);
        if constexpr (D > 2) o[2] = (int)(x.y & 0xffffu);
        if constexpr (D > 3) o[3] = (int)(x.y >> 16);
    };
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
    };

    // ---- launch setup (level 0 from s, level 1 by one sweep in LDS)
    {
        const int64_t col = r >> 6;
        const u64 rbit = 1ull << (r & 63);
        for (int64_t q = lane; q < n * D; q += 64) {
            const int64_t v = q / D;
            rows[v * 4 + (q - v * D)] = (uint16_t)g[q];
        }
        for (int k = lane; k < 2 * nw * 2; k += 64) lv[k] = 0u;
        wave_sync();
        for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
            const int64_t v = v0 + lane;
            const bool b = v < n && (s[v * W + col] & rbit);
            const u64 m = __ballot(b);
            if (lane < 2) {
                const uint32_t x = (uint32_t)(m >> (32 * lane));
                lword(0, (int)(v0 >> 5) + lane) = x;
                lev0s[(v0 >> 5) + lane] = x;
            }
        }
        for (int k = lane; k < MT_N; k += 64) mt[k] = st.mt[r * MT_N + k];
        wave_sync();
        for (int64_t v0 = 0; v0 < (int64_t)nw * 32; v0 += 64) {
            const int v = (int)(v0 + lane);
            uint32_t nb = 0;
            if (v < n) {
                int nv[D];
                nbrs(v, nv);
                int ones = 0;
#pragma unroll
                for (int q = 0; q < D; ++q) ones += (int)bit_of(0, nv[q]);
                nb = maj(ones, bit_of(0, v));
            }
            const u64 m = __ballot(nb != 0);
            if (lane < 2) lword(1, (int)(v0 >> 5) + lane) = (uint32_t)(m >> (32 * lane));
        }
        wave_sync();
    }

    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    u64* park = reinterpret_cast<u64*>(smem + geo.off_cnt);     // write-back pointers, off the scalar file
    if (lane == 0) {
        park[0] = (u64)s;
        park[1] = (u64)st.mt;
        park[2] = (u64)st.mt_idx;
        park[3] = (u64)st.a;
        park[4] = (u64)st.b;
        park[5] = (u64)st.t;
        park[6] = (u64)st.sum_end;
        park[7] = (u64)st.done;
        park[8] = (u64)st.tr_tie;
        park[9] = (u64)W;
    }
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    double inv_n = 1.0 / (double)n;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(par_a), "+v"(par_b), "+v"(a_cap), "+v"(b_cap), "+v"(inv_n));

    int pb_i = 0, pb_end = 0;
    uint32_t pb_w1 = 0, pb_w2 = 0;
    double pb_u = 0.0;
    int npend = 0, pk = 0;
    auto parse = [&](bool one) {
        for (;;) {
            if (idx >= MT_N) {
                if (one) break;
                lds_twist(mt, lane);
                idx = 0;
            }
            const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
            uint32_t tw = 0, y = 0;
            bool ok = false;
            if (lane < lim) {
                tw = mt_temper(mt[idx + lane]);
                y = tw & mask;
                ok = y <= rng;
            }
            const u64 okm = __ballot(ok);
            int pos = 0, got = 0;
            while (pos < 64 && npend < 64) {
                const u64 m = okm >> pos;
                if (!m) break;
                const int f = pos + __ffsll((unsigned long long)m) - 1;
                if (f + 2 >= lim) break;
                const int iv = __builtin_amdgcn_readlane((int)y, f);
                const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)tw, f + 1);
                const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)tw, f + 2);
                if (lane == npend) { pb_i = iv; pb_w1 = w1; pb_w2 = w2; pb_end = idx + f + 3; }
                ++npend;
                ++got;
                pos = f + 3;
            }
            if (got > 0) { idx += pos; break; }
            if (one) break;
            if (!okm) { idx += lim; continue; }
            const int f = __ffsll((unsigned long long)okm) - 1;
            if (f > 0) { idx += f; continue; }
            const int iv = __builtin_amdgcn_readlane((int)y, 0);
            idx += 1;
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            const uint32_t w1 = mt_temper(mt[idx]);
            idx += 1;
            if (idx >= MT_N) { lds_twist(mt, lane); idx = 0; }
            const uint32_t w2 = mt_temper(mt[idx]);
            idx += 1;
            if (lane == npend) { pb_i = iv; pb_w1 = w1; pb_w2 = w2; pb_end = idx; }
            ++npend;
            break;
        }
        pb_u = mt_double(pb_w1, pb_w2);
    };

    bool drew = false;
    int64_t k = 0;
#ifdef MJX_SA_PROF
    unsigned long long _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _t0 = __builtin_amdgcn_s_memtime();
#endif
    while (k < nsteps && done == 0) {
        int avail = npend - pk;
        if (avail < NQ && idx + 64 <= MT_N) {
            // carry the unconsumed proposals to lanes 0.. and append one window
            const int src = (lane + pk < 64) ? lane + pk : 63;
            pb_i = __shfl(pb_i, src, 64);
            pb_end = __shfl(pb_end, src, 64);
            pb_w1 = (uint32_t)__shfl((int)pb_w1, src, 64);
            pb_w2 = (uint32_t)__shfl((int)pb_w2, src, 64);
            npend = avail;
            pk = 0;
            parse(true);
            if (npend == 0) parse(false);
        } else if (avail == 0) {
            npend = 0;
            pk = 0;
            parse(false);
        }
        drew = true;
        LDS_STAMP(0);
        avail = npend - pk;
        int nq = avail < NQ ? avail : NQ;
        if ((int64_t)nq > nsteps - k) nq = (int)(nsteps - k);
        // group gq's proposal
        const bool act = gq < nq;
        const int mine = __shfl(pb_i, pk + (act ? gq : 0), 64);
        const uint64_t ub = __builtin_bit_cast(uint64_t, pb_u);
        const uint32_t ulo = (uint32_t)__shfl((int)(uint32_t)ub, pk + (act ? gq : 0), 64);
        const uint32_t uhi = (uint32_t)__shfl((int)(uint32_t)(ub >> 32), pk + (act ? gq : 0), 64);
        const double u = __builtin_bit_cast(double, ((uint64_t)uhi << 32) | ulo);
        const int iv = mine;
        const uint32_t old_i = bit_of(0, iv);
        // level 1: i and its neighbours, level 0 with i flipped
        int ri[D];
        nbrs(iv, ri);
        int cand = iv;
#pragma unroll
        for (int q = 0; q < D; ++q)
            if (gl == q + 1) cand = ri[q];
        bool dup = gl > 0 && cand == iv;
#pragma unroll
        for (int q = 0; q < D; ++q)
            if (q + 1 < gl) dup |= ri[q] == cand;
        int nv[D];
        nbrs(cand, nv);
        const bool live = act && gl <= D && !dup;
        int ones = 0;
#pragma unroll
        for (int e = 0; e < D; ++e) ones += (int)(bit_of(0, nv[e]) ^ (nv[e] == iv));
        const uint32_t own = bit_of(0, cand) ^ (cand == iv);
        const uint32_t nb = maj(ones, own);
        const uint32_t cur = bit_of(1, cand);
        const bool chg = live && nb != cur;
        // conflicts with the earlier proposals of the step: bit j of cf = i_j read here
        uint32_t cf = 0;
#pragma unroll
        for (int j = 0; j < NQ - 1; ++j) {
            const int ij = __shfl(pb_i, pk + j, 64);
            bool hit = cand == ij;
#pragma unroll
            for (int e = 0; e < D; ++e) hit |= nv[e] == ij;
            if (live && j < gq && hit) cf |= 1u << j;
        }
        // per group: sum(s_end) change, conflicts (uniform masks, sliced per group below)
        const u64 up = __ballot(chg && cur == 0u), dn = __ballot(chg && cur != 0u);
        u64 cfm[NQ - 1];
#pragma unroll
        for (int j = 0; j < NQ - 1; ++j) cfm[j] = __ballot((cf >> j) & 1u);
        LDS_STAMP(1);
        const u64 gm = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (gq * G);
        const int64_t ds = 2 * ((int64_t)__popcll(up & gm) - (int64_t)__popcll(dn & gm));
        // schedule value of step k + gq (code/SA_RRG.py:80-81), delta_H and the Metropolis test
        double ag = a, bg = b;
        for (int q = 0; q < gq; ++q) {
            if (ag < a_cap) ag = par_a * ag;
            if (bg < b_cap) bg = par_b * bg;
        }
        const double an = (ag < a_cap) ? par_a * ag : ag;           // the schedule after this step
        const double bn = (bg < b_cap) ? par_b * bg : bg;
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * ag) * si;
        const double t2 = bg * (double)(-ds);
        const double num = t1 + t2;
        const float xf = (float)(-num * inv_n);
        const float ef = __expf(xf);
        const float mg = ef * (1e-6f * (1.0f + fabsf(xf))) + 1e-37f;
        bool acc, tie = false;
        double dE = 0.0;
        if (fabs(u - (double)ef) > (double)mg) {
            acc = u < (double)ef;
            if (TRACE && st.tr_dE) dE = num / (double)n;
        } else {
            dE = num / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;
            acc = u < prob;
            tie = e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e);
        }
        const u64 accm = __ballot(acc && gl == 0), tiem = __ballot(tie && gl == 0);
        LDS_STAMP(5);
        // ---- resolve in proposal order: the taken proposals are a prefix, ended by
        // the first proposal that read an accepted earlier one's i (one ballot) or
        // by a stop; the walk over the prefix is integer work only
        constexpr u64 GM = (G == 64) ? ~0ull : ((1ull << G) - 1ull);
        uint32_t accg = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) accg |= (uint32_t)((accm >> (q * G)) & 1ull) << q;
        const u64 clm = __ballot(live && (cf & accg) != 0u);
        int qstop = nq;
        if (clm) {
            const int qc = (__ffsll((unsigned long long)clm) - 1) / G;
            if (qc < qstop) qstop = qc;
        }
        int taken = 0;
        for (int q = 0; q < qstop; ++q) {
            const bool aq = (accg >> q) & 1u;
            if (aq) sum_end += 2 * ((int64_t)__popcll((up >> (q * G)) & GM) - (int64_t)__popcll((dn >> (q * G)) & GM));
            if ((tiem >> (q * G)) & 1ull) ++ties;
            t += 1;                                                 // (code/SA_RRG.py:77,82)
            ++taken;
            if (TRACE && lane == q * G) {
                if (st.tr_i) st.tr_i[(k + q) * R + r] = iv;
                if (st.tr_acc) st.tr_acc[(k + q) * R + r] = aq ? 1 : 0;
                if (st.tr_sum) st.tr_sum[(k + q) * R + r] = sum_end;
                if (st.tr_dE) st.tr_dE[(k + q) * R + r] = dE;
            }
            if (t > t_cap) { done = 2; break; }                     // (:84)
            if (sum_end == n) { done = 1; break; }                  // m(s_endstate(s)) == 1
        }
        const uint32_t acc_taken = accg & ((1u << taken) - 1u);
        a = __shfl(an, (taken - 1) * G, 64);                        // (:80-81) after the taken steps
        b = __shfl(bn, (taken - 1) * G, 64);
        // ---- the accepted proposals among the taken ones: level 1 on their C_1, level 0 at i
        if (gq < taken && ((acc_taken >> gq) & 1u)) {
            if (chg) {
                const uint32_t bit = 1u << (cand & 31);
                if (cur) atomicAnd(&lword(1, cand >> 5), ~bit);
                else atomicOr(&lword(1, cand >> 5), bit);
            }
            if (gl == 0) atomicXor(&lword(0, iv >> 5), 1u << (iv & 31));
        }
        k += taken;
        pk += taken;
        wave_sync();
        LDS_STAMP(6);
#ifdef MJX_SA_PROF
        _acc[7] += 1000 * (unsigned long long)taken;
#endif
    }
#ifdef MJX_SA_PROF
    if (lane == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&mjx_sa_lds_prof[q], _acc[q]);
#endif
    if (drew) idx = __builtin_amdgcn_readlane(pb_end, pk - 1);
    if (TRACE && lane == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    wave_sync();
    u64* const ps = (u64*)park[0];
    const int64_t Wp = (int64_t)park[9];
    const int64_t rr = blockIdx.x;
    for (int64_t v0 = 0; v0 < n; v0 += 64) {
        const int v = (int)(v0 + lane);
        if (v < n && (((lword(0, v >> 5) ^ lev0s[v >> 5]) >> (v & 31)) & 1u))
            atomicXor((unsigned long long*)&ps[(int64_t)v * Wp + (rr >> 6)], 1ull << (rr & 63));
    }
    uint32_t* const pmt = (uint32_t*)park[1];
    for (int q = lane; q < MT_N; q += 64) pmt[rr * MT_N + q] = mt[q];
    if (lane == 0) {
        ((int32_t*)park[2])[rr] = idx;
        ((double*)park[3])[rr] = a;
        ((double*)park[4])[rr] = b;
        ((int64_t*)park[5])[rr] = t;
        ((int64_t*)park[6])[rr] = sum_end;
        ((int32_t*)park[7])[rr] = done;
        int32_t* const tie = (int32_t*)park[8];
        if (tie) tie[rr] += ties;
    }
}

// ---------------------------------------------------------------------------
// The whole CU for one replica (k_sa_lds_wg<D, T, NW>, d <= 4, 1 < T <= 4).
// The one-wave kernels above leave 3 of a CU's 4 SIMDs idle: a replica's step
// is a chain of dependent LDS round trips on one wave.  Here NW waves share the
// replica's LDS image; NW-1 of them evaluate as many consecutive proposals k,
// k+1, ... at once, each against the levels as they stand at the start of the round,
// wave q exactly as k_sa_lds_fast evaluates one proposal.  The change marks
// are one BYTE per (level, node): bit q = proposal q's C_t, so "level t as
// proposal q sees it" is the level bit XOR mark bit q, and the bits below q in
// the same byte say which EARLIER proposals changed that value.  A proposal q
// stands unless an earlier proposal j of the round is taken and accepted and
// changed something q read -- a node q reads at level l-1, or whose cached
// level-l value it reads, changes under j only if it or a neighbour is in j's
// C_{l-1}, i.e. only if q read j's mark at level l-1 (k_sa_lds_pair's rule;
// level 0 by comparing with i_j).  Acceptance needs no order (delta_H of step
// k+q depends on the schedule after q steps, computed by q multiplications as
// the reference does, and on q's own sum change), so every wave decides its
// own; the taken proposals are the prefix before the first conflict with a
// taken accepted one, or up to the first stop (consensus, t cap).  Taken
// accepted change sets are disjoint (a shared node would be a conflict), so
// they are applied concurrently.  Workgroup barriers: one after the proposals
// are published, one after every proposal's marks (the conflict checks read
// them), one before the resolution.  The last wave parses the numpy stream's
// windows (as k_sa_lds_multi) into an LDS ring of proposals while the others
// evaluate, off the round's critical path.  Same draws, accepts and state as
// k_sa_lds.
struct GeoW {
    int nw;        // uint32 bit words per level (even)
    int lc;        // change-list capacity per level
    int off_lev;   // nw level-0 words
    int off_mk;    // T * nw * 32 marks (levels 1..T): a byte each, 16 bits above 8 waves;
                   // the top bit holds the level's value
    int off_lev0;  // nw words: level 0 at launch start
    int off_mt;
    int off_list;  // (NW - 1) * T * lc list words (one set per evaluating wave, levels 1..T)
    int off_q;     // proposal queue: i[64], end[64], u[64]
    int off_res;   // per proposal: conflict word, packed word, schedule a, b after its step; control words
    int bytes;
};

static bool geometry_wg(int64_t n, int d, int T, int NW, GeoW* g) {
    if (n < 2 || n > 65535 || d < 1 || d > 4 || T < 1 || T > kMaxT || NW < 2 || NW > 16) return false;
    const int mkb = NW > 8 ? 2 : 1;                 // bytes per mark
    g->nw = (int)(((n + 63) / 64) * 2);
    int64_t lc = ball(d, T);
    if (lc > n) lc = n;
    lc = ((lc + 63) / 64) * 64;
    if (lc > 4096) return false;
    g->lc = (int)lc;
    int64_t off = ((int64_t)n * 4 * 2 + 15) / 16 * 16;
    g->off_lev = (int)off;   off += (int64_t)g->nw * 4;
    g->off_mk = (int)off;    off += (int64_t)T * g->nw * 32 * mkb;
    g->off_lev0 = (int)off;  off += (int64_t)g->nw * 4;
    g->off_mt = (int)off;    off += MT_N * 4;
    g->off_list = (int)off;  off += (int64_t)(NW - 1) * T * g->lc * 4;
    off = (off + 15) / 16 * 16;
    g->off_q = (int)off;     off += 64 * 4 + 64 * 4 + 64 * 8;
    g->off_res = (int)off;   off += (int64_t)NW * (4 + 4 + 8 + 8) + 4 * 4;
    g->bytes = (int)off;
    return (size_t)off <= kLdsMax;
}

// waves of the whole-CU kernel: 16 where its LDS fits (d = 4, T = 3: n <= ~1e4,
// SA_RRG.py's own size), else 8; kernel option split = 4 or 8 forces that many
static int wg_waves(int64_t n, int d, int T, int split) {
    if (split == 4 || split == 8) return split;
    GeoW g;
    return geometry_wg(n, d, T, 16, &g) ? 16 : 8;
}

template <int D, int T, int NW, bool TRACE>
__global__ void __launch_bounds__(64 * NW) k_sa_lds_wg(const int32_t* __restrict__ adj, int64_t n, int64_t R,
                                                      int64_t W, u64* __restrict__ s, mjx_sa_state st, int64_t nsteps,
                                                      double par_a, double par_b, double a_cap, double b_cap,
                                                      int64_t t_cap, GeoW geo) {
    static_assert(D >= 1 && D <= 4 && T >= 2 && T <= 4 && NW >= 2 && NW <= 16, "whole-CU LDS SA: d <= 4, 2 <= T <= 4");
    // a mark per (level >= 1, node): bit q = proposal q of the round; bytes up to
    // 8 waves, 16-bit words for 16 (n = 1e4, T = 3 then fits in 159 KB)
    using MK = typename std::conditional<(NW > 8), uint16_t, uint8_t>::type;
    constexpr int MKB = 8 * (int)sizeof(MK);       // bits per mark
    constexpr int MPW = 4 / (int)sizeof(MK);       // marks per 32-bit word
    constexpr int DP1 = D + 1;
    constexpr int MAXM = 64 / DP1;                 // members of C_{t-1} one wave can expand
    constexpr int NT = 64 * NW;
    constexpr int NE = NW - 1;                     // waves evaluating proposals; wave NE parses
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wave's proposal slot in a round
    const int lane = tid & 63;
    const u64 ltmask = (1ull << lane) - 1ull;
    const int64_t r = blockIdx.x;
    const int nw = geo.nw, lc = geo.lc;
    const int mkl = nw * 32;                       // mark bytes per level
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lev = reinterpret_cast<uint32_t*>(smem + geo.off_lev);
    MK* mk = reinterpret_cast<MK*>(smem + geo.off_mk);
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    // this wave's lists of levels 1..T (level l at (l-1)*lc)
    uint32_t* lst = reinterpret_cast<uint32_t*>(smem + geo.off_list) + w * T * lc - lc;
    int* q_i = reinterpret_cast<int*>(smem + geo.off_q);
    int* q_end = q_i + 64;
    double* q_u = reinterpret_cast<double*>(q_end + 64);
    uint32_t* res_cf = reinterpret_cast<uint32_t*>(smem + geo.off_res);   // per proposal: conflict bits
    uint32_t* res = res_cf + NW;                                           // packed result per proposal
    double* res_a = reinterpret_cast<double*>(res + NW);
    double* res_b = res_a + NW;
    int* ctl = reinterpret_cast<int*>(res_b + NW);
    constexpr int LVB = MKB - 1;                   // the level value's bit in a mark (above NE proposals)
    static_assert(NE <= LVB, "a mark holds NE proposal bits and the level bit");
    const uint32_t obit = 1u << w;                 // this proposal's mark bit
    const int l1 = (lane >= 1 && lane <= D) ? lane - 1 : 0;      // (clamped row entry)
    const uint32_t early = obit - 1u;              // the earlier proposals' mark bits

    auto bit_of = [&](int v) -> uint32_t { return (lev[v >> 5] >> (v & 31)) & 1u; };     // level 0
    auto lvl = [&](int t, int v) -> uint32_t { return ((uint32_t)mk[(t - 1) * mkl + v] >> LVB) & 1u; };   // t >= 1
    // node v at level t >= 1 as this proposal sees it (one read: the level bit
    // and the marks); earlier proposals' marks into cfm
    auto look = [&](int t, int v, uint32_t& cfm) -> uint32_t {
        const uint32_t mb = mk[(t - 1) * mkl + v];
        cfm |= mb & early;
        return ((mb >> LVB) ^ (mb >> w)) & 1u;
    };
    auto mark_word = [&](int t, int v) -> uint32_t* {
        return reinterpret_cast<uint32_t*>(mk + (t - 1) * mkl + (v & ~(MPW - 1)));
    };
    auto mark_bit = [&](int v) -> uint32_t { return obit << (MKB * (v & (MPW - 1))); };
    auto nbrs = [&](int v, int (&o)[D]) {
        const uint2 x = *reinterpret_cast<const uint2*>(rows + v * 4);
        o[0] = (int)(x.x & 0xffffu);
        if constexpr (D > 1) o[1] = (int)(x.x >> 16);
        if constexpr (D > 2) o[2] = (int)(x.y & 0xffffu);
        if constexpr (D > 3) o[3] = (int)(x.y >> 16);
    };
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
    };

    // ---- launch setup: rows, level 0, marks cleared, MT state; levels 1..T by sweeps in LDS
    {
        const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * D;
        for (int64_t q = tid; q < n * D; q += NT) {
            const int64_t v = q / D;
            rows[v * 4 + (q - v * D)] = (uint16_t)g[q];
        }
        for (int q = tid; q < nw; q += NT) lev[q] = 0u;
        for (int q = tid; q < T * nw * 8 * (int)sizeof(MK); q += NT) reinterpret_cast<uint32_t*>(mk)[q] = 0u;
        for (int q = tid; q < MT_N; q += NT) mt[q] = st.mt[r * MT_N + q];
        const int64_t col = r >> 6;
        const u64 rbit = 1ull << (r & 63);
        __syncthreads();
        for (int64_t v0 = (int64_t)w * 64; v0 < (int64_t)nw * 32; v0 += NT) {
            const int64_t v = v0 + lane;
            const bool b = v < n && (s[v * W + col] & rbit);
            const u64 m = __ballot(b);
            if (lane < 2) {
                const uint32_t x = (uint32_t)(m >> (32 * lane));
                lev[(v0 >> 5) + lane] = x;
                lev0s[(v0 >> 5) + lane] = x;
            }
        }
        __syncthreads();
        for (int t = 1; t <= T; ++t) {
            for (int v = tid; v < n; v += NT) {
                int nv[D];
                nbrs(v, nv);
                int ones = 0;
#pragma unroll
                for (int q = 0; q < D; ++q) ones += (int)(t == 1 ? bit_of(nv[q]) : lvl(t - 1, nv[q]));
                const uint32_t nb = maj(ones, t == 1 ? bit_of(v) : lvl(t - 1, v));
                mk[(t - 1) * mkl + v] = (MK)(nb << LVB);
            }
            __syncthreads();
        }
    }

    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    double inv_n = 1.0 / (double)n;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(par_a), "+v"(par_b), "+v"(a_cap), "+v"(b_cap), "+v"(inv_n));

    // ---- the proposal ring (wave P = NE parses, the NE others evaluate): slot
    // q & 63 holds proposal q of the launch (i, u, end: the MT index after its
    // draws, bit 10 its state generation's parity).  npend proposals parsed, pk
    // taken (running counts, every wave tracks pk); the parse wave appends while
    // the round evaluates, into slots the round does not read, and keeps slot
    // pk-1 (the last taken proposal's end) for the launch's MT position.  A twist
    // under unconsumed proposals first saves the old state to st.mt: the launch
    // ends on either generation (the buffer the last taken proposal drew from).
    uint32_t npend = 0, pk = 0;
    int gen = 0;
    const int idx0 = idx;
    auto twist = [&]() {
        for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = mt[q];
        lds_twist(mt, lane);
        idx = 0;
        gen ^= 1;
    };
    // A twist is refused while the last taken proposal (slot pk-1, kept for the
    // launch's end) still draws from the previous generation: st.mt holds one
    // old generation only, so the end's generation is never more than one
    // behind and bit 10's parity names it.  (With nothing pending -- 624 words
    // parsed without one acceptable proposal, never in practice -- the twist
    // goes ahead rather than stall.)
    auto twist_ok = [&]() -> bool {
        const int lg = (pk > 0u) ? ((q_end[(pk - 1u) & 63u] >> 10) & 1) : 0;
        return lg == gen || npend == pk;
    };
    // one window of up to 64 words at idx: at most `room` proposals appended;
    // false when a refused twist leaves it for after the round
    auto parse_window = [&](uint32_t room) -> bool {
        if (idx >= MT_N) {
            if (!twist_ok()) return false;
            twist();
        }
        const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
        uint32_t tw = 0, y = 0;
        bool ok = false;
        if (lane < lim) {
            tw = mt_temper(mt[idx + lane]);
            y = tw & mask;
            ok = y <= rng;
        }
        const u64 okm = __ballot(ok);
        // the proposal starts (each: the first acceptable word at or after the
        // previous end, then rand()'s two words) whose words fit the window, at
        // most `room` of them
        u64 stm = mt_window_starts(ok) & ((lim >= 2) ? ((1ull << (lim - 2)) - 1ull) : 0ull);
        while ((uint32_t)__popcll(stm) > room) stm &= ~(1ull << (63 - __clzll(stm)));
        const uint32_t got = (uint32_t)__popcll(stm);
        const int pos = got ? 66 - __clzll(stm) : 0;          // after the last start's two words
        if (got > 0) {
            const uint32_t x1 = mt_next_lane(tw);
            const uint32_t x2 = mt_next_lane(x1);
            if ((stm >> lane) & 1ull) {
                const int q = (int)((npend + (uint32_t)__popcll(stm & ltmask)) & 63u);
                q_i[q] = (int)y;
                q_u[q] = mt_double(x1, x2);
                q_end[q] = (idx + lane + 3) | (gen << 10);
            }
            npend += got;
            idx += pos;
            return true;
        }
        if (room == 0) return true;
        if (!okm) { idx += lim; return true; }
        const int f = __ffsll((unsigned long long)okm) - 1;
        if (f > 0) { idx += f; return true; }
        if (idx + 2 >= MT_N && !twist_ok()) return false;
        // i is the window's first word and rand()'s two words cross the end of
        // the state: the serial draw twists between them, as numpy does
        const int iv = __builtin_amdgcn_readlane((int)y, 0);
        idx += 1;
        if (idx >= MT_N) twist();
        const uint32_t w1 = mt_temper(mt[idx]);
        idx += 1;
        if (idx >= MT_N) twist();
        const uint32_t w2 = mt_temper(mt[idx]);
        idx += 1;
        if (lane == 0) {
            const int q = (int)(npend & 63u);
            q_i[q] = iv;
            q_u[q] = mt_double(w1, w2);
            q_end[q] = idx | (gen << 10);
        }
        npend += 1;
        return true;
    };
    auto room = [&]() -> uint32_t { return 63u - (npend - pk); };     // slot pk-1 kept

    int lc_c[T + 1];
    uint32_t lc_v[T + 1];
    bool lc_in[T + 1];
    int lc_n[T + 1];
    bool lc_fast[T + 1];
    int64_t k = 0;
#ifdef MJX_SA_PROF
    // (32-bit sums: a launch's rounds fit; slot 8 this wave's levels + test, 9 the
    // parse wave's parsing, 10 the barrier-1 wait; per-wave sums of slot 8 at 16 + w)
    unsigned int _acc[11] = {};
    unsigned long long _t0 = __builtin_amdgcn_s_memtime();
#endif
    while (k < nsteps && done == 0) {
        if (w == NE) {
            // a full round's proposals before it starts (the ring is normally
            // that far ahead: this parses only at launch start or after a dry spell)
            // (a refused twist ends the loop: the round runs on what is pending)
            while (npend - pk < (uint32_t)NE)
                if (!parse_window(room())) break;
            if (lane == 0) ctl[0] = (int)npend;
        }
        __syncthreads();                                   // the round's proposals are published
        LDS_STAMP(0);
        const uint32_t npd = (uint32_t)__builtin_amdgcn_readfirstlane(ctl[0]);
        int nq = (int)(npd - pk);
        if (nq > NE) nq = NE;
        if ((int64_t)nq > nsteps - k) nq = (int)(nsteps - k);
        const bool act = w < nq;
        int iv = 0;
        uint32_t old_i = 0, cf = 0;                        // cf bit j: read something proposal j changed
        uint32_t cf0 = 0;                                  // (level 0, wave-uniform)
        int riq[D];                                        // i's neighbours
        int last = 0;
        int64_t ds = 0;
        // the nodes this wave read at each level l >= 2 (a candidate and its
        // neighbours per lane): checked against the earlier proposals' marks of
        // level l-1 once every wave is through its levels (no barrier per level)
        int rd_c[T + 1], rd_n[T + 1][D];
        bool rd_on[T + 1];
        bool rd_all = false;                               // a list level: conflicts with every earlier one
#pragma unroll
        for (int l = 0; l <= T; ++l) {
            rd_on[l] = false;
            lc_fast[l] = true;
            lc_in[l] = false;
            lc_n[l] = 0;
        }
        bool acc = false, tie = false;
        double dE = 0.0, anx = a, bnx = b;
        if (w < NE) {
        // the round's proposals' i, lane j = proposal j (one read; readlanes below)
        const int ipv = q_i[(pk + (uint32_t)(lane < NE ? lane : 0)) & 63u];
        const double u = q_u[(pk + (uint32_t)(act ? w : 0)) & 63u];
        iv = __builtin_amdgcn_readlane(ipv, act ? w : 0);
        int rj[D];                                         // lane j: proposal j's neighbours
        nbrs(ipv, rj);
        old_i = bit_of(iv);
        int cand, nv[D];
        // ---- level 1: i and its neighbours, level 0 with i flipped
        {
            int ri[D];
            nbrs(iv, ri);
            // lane l in 1..D: i's l-th neighbour, by its own read (no per-lane selects)
            const int c1 = (int)rows[iv * 4 + l1];
            cand = (lane >= 1 && lane <= D) ? c1 : iv;
            // a repeat of i or of an earlier lane's neighbour (multi-edges) is not live
            int first = D;
#pragma unroll
            for (int q = D - 1; q >= 0; --q)
                if (ri[q] == cand) first = q;
            const bool dup = lane > 0 && (cand == iv || first + 1 < lane);
            nbrs(cand, nv);
            const bool live = act && lane <= D && !dup;
            int ones = 0;
#pragma unroll
            for (int e = 0; e < D; ++e) ones += (int)(bit_of(nv[e]) ^ (nv[e] == iv));
#pragma unroll
            for (int q = 0; q < D; ++q) riq[q] = ri[q];
            const uint32_t own = bit_of(cand) ^ (cand == iv);
            const uint32_t nb = maj(ones, own);
            const uint32_t cur = lvl(1, cand);
            const bool chg = live && nb != cur;
            const u64 m = __ballot(chg);
            if (chg) {
                atomicOr(mark_word(1, cand), mark_bit(cand));
                lst[lc + __popcll(m & ltmask)] = (uint32_t)cand;
            }
            lc_c[1] = cand;
            lc_v[1] = cur;
            lc_in[1] = chg;
            lc_fast[1] = true;
            lc_n[1] = __popcll(m);
            last = lc_n[1] ? 1 : 0;
        }
        LDS_STAMP(1);
#pragma unroll
        for (int l = 2; l <= T; ++l) {
            rd_c[l] = 0;
#pragma unroll
            for (int e = 0; e < D; ++e) rd_n[l][e] = 0;
            if (last != l - 1) {                           // (wave-uniform)
                LDS_STAMP(l < 4 ? l : 3);
                continue;
            }
            wave_sync();                                   // this wave's marks of C_{l-1}
            const int np = lc_n[l - 1];
            int nc = 0;
            if (np <= MAXM && lc_fast[l - 1]) {
                // candidates: member sl = lane / (d+1) of C_{l-1} (this wave's list
                // of level l-1, in lane-rank order), j = 0 the member itself, j > 0
                // its j-th neighbour: two LDS reads, no cross-lane moves
                const int sl = lane / DP1, j = lane - sl * DP1;
                const bool act2 = sl < np;
                const int mc = act2 ? (int)lst[(l - 1) * lc + sl] : iv;
                int c2 = (act2 && j > 0) ? (int)rows[mc * 4 + (j > 0 ? j - 1 : 0)] : mc;
                int nv2[D];
                nbrs(c2, nv2);
                int ones = 0;
                uint32_t cfm = 0;                          // (the other waves' marks may still be coming)
#pragma unroll
                for (int e = 0; e < D; ++e) ones += (int)look(l - 1, nv2[e], cfm);
                const uint32_t own = look(l - 1, c2, cfm);
                rd_on[l] = act2;
                rd_c[l] = c2;
#pragma unroll
                for (int e = 0; e < D; ++e) rd_n[l][e] = nv2[e];
                const uint32_t nb = maj(ones, own);
                const uint32_t cur = lvl(l, c2);
                const bool chg = act2 && nb != cur;
                const uint32_t mb = mark_bit(c2);
                bool add = chg;
                if (l == T) {
                    // the last level counts distinct nodes: the first mark wins
                    if (chg) add = (atomicOr(mark_word(l, c2), mb) & mb) == 0u;
                } else if (chg) {
                    // inner levels keep repeats (marks, clears and the accepted values
                    // are idempotent; the next level's dedup absorbs them)
                    atomicOr(mark_word(l, c2), mb);
                }
                const u64 m = __ballot(add);
                if (add) lst[l * lc + __popcll(m & ltmask)] = (uint32_t)c2;
                nc = __popcll(m);
                cand = c2;
#pragma unroll
                for (int e = 0; e < D; ++e) nv[e] = nv2[e];
                lc_c[l] = c2;
                lc_v[l] = cur;
                lc_in[l] = add;
                if (l == T) ds = 2 * ((int64_t)__popcll(__ballot(add && cur == 0u)) - (int64_t)__popcll(__ballot(add && cur != 0u)));
            } else {
                // this wave's LDS-list path (its lists hold every level; deduped here);
                // its reads are not kept: the proposal stands only as the round's first
                // taken one or after rejected ones (conflict with every earlier one)
                rd_all = true;
                const uint32_t* prev = lst + (l - 1) * lc;
                uint32_t* curl = lst + l * lc;
                const int m = np * DP1;
                int64_t dsl = 0;
                for (int base = 0; base < m; base += 64) {
                    const int q = base + lane;
                    bool add = false;
                    int cd = 0;
                    uint32_t cur = 0;
                    if (q < m) {
                        const int slot = q / DP1, jj = q - slot * DP1;
                        const int v = (int)prev[slot];
                        cd = (jj == 0) ? v : (int)rows[v * 4 + jj - 1];
                        int nv2[D];
                        nbrs(cd, nv2);
                        int ones = 0;
                        uint32_t cfm = 0;
#pragma unroll
                        for (int e = 0; e < D; ++e) ones += (int)look(l - 1, nv2[e], cfm);
                        const uint32_t own = look(l - 1, cd, cfm);
                        const uint32_t nb = maj(ones, own);
                        const uint32_t mb = mark_bit(cd);
                        cur = lvl(l, cd);
                        if (nb != cur) add = (atomicOr(mark_word(l, cd), mb) & mb) == 0u;
                    }
                    const u64 bal = __ballot(add);
                    if (add) curl[nc + __popcll(bal & ltmask)] = (uint32_t)cd;
                    nc += __popcll(bal);
                    dsl += 2 * ((int64_t)__popcll(__ballot(add && cur == 0u)) - (int64_t)__popcll(__ballot(add && cur != 0u)));
                }
                if (l == T) ds = dsl;
                lc_fast[l] = false;
            }
            lc_n[l] = nc;
            if (nc > 0) last = l;
            LDS_STAMP(l < 4 ? l : 3);
        }
        if (last != T) ds = 0;
        // ---- delta_H and the Metropolis test of this wave's proposal, step k + w
        // (code/SA_RRG.py:37,74-76); the schedule after w steps (:80-81)
        double ah = a, bh = b;
        if (!(ah >= a_cap && bh >= b_cap)) {                         // both capped after ~1.2e4 steps
            for (int q = 0; q < w; ++q) {
                if (ah < a_cap) ah = par_a * ah;
                if (bh < b_cap) bh = par_b * bh;
            }
        }
        anx = (ah < a_cap) ? par_a * ah : ah;                       // the schedule after this step
        bnx = (bh < b_cap) ? par_b * bh : bh;
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * ah) * si;
        const double t2 = bh * (double)(-ds);
        const double num = t1 + t2;
        // u < min(1, exp(-dE)) by an fp32 exp where u is farther from it than that
        // exp's error, else by the reference's float64 dE and exp (as k_sa_lds_fast)
        const float xf = (float)(-num * inv_n);
        const float ef = __expf(xf);
        const float mg = ef * (1e-6f * (1.0f + fabsf(xf))) + 1e-37f;
        if (fabs(u - (double)ef) > (double)mg) {
            acc = u < (double)ef;
            if (TRACE && st.tr_dE) dE = num / (double)n;
        } else {
            dE = num / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;
            acc = u < prob;
            tie = e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e);
        }
        // level-0 conflicts: the level-0 values read here are those of the ball of
        // radius 2 around i, and i_j is in it iff the closed neighbourhoods of i
        // and i_j meet (lane j compares the two, off the level chain)
        if (act) {
            bool meet = ipv == iv;
#pragma unroll
            for (int e = 0; e < D; ++e) meet |= (rj[e] == iv) | (ipv == riq[e]);
#pragma unroll
            for (int e = 0; e < D; ++e)
#pragma unroll
                for (int f = 0; f < D; ++f) meet |= rj[e] == riq[f];
            cf0 = (uint32_t)__ballot(meet) & early;
        }
        LDS_STAMP(4);
#ifdef MJX_SA_PROF
        _acc[8] = _acc[1] + _acc[2] + _acc[3] + _acc[4];
#endif
        } else {
            // the parse wave: windows into the ring's free slots while the round evaluates
            for (int it = 0; it < 2 && room() >= 8u; ++it)
                if (!parse_window(room())) break;
            LDS_STAMP(9);
        }
        __syncthreads();                                   // every proposal's marks of every level
        LDS_STAMP(10);
        // what this proposal read at level l-1 that an earlier one changed
#pragma unroll
        for (int l = 2; l <= T; ++l) {
            if (rd_on[l]) {
                uint32_t mb = mk[(l - 2) * mkl + rd_c[l]];
#pragma unroll
                for (int e = 0; e < D; ++e) mb |= mk[(l - 2) * mkl + rd_n[l][e]];
                cf |= mb & early;
            }
        }
        if (rd_all) cf |= early;
        // the lanes' conflicts OR-ed: DPP row prefixes, the four row ends
        cf |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cf, 0x111, 0xf, 0xf, false);   // row_shr:1
        cf |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cf, 0x112, 0xf, 0xf, false);   // row_shr:2
        cf |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cf, 0x114, 0xf, 0xf, false);   // row_shr:4
        cf |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cf, 0x118, 0xf, 0xf, false);   // row_shr:8
        const uint32_t cfw = cf0 | (uint32_t)__builtin_amdgcn_readlane((int)cf, 15) |
                             (uint32_t)__builtin_amdgcn_readlane((int)cf, 31) |
                             (uint32_t)__builtin_amdgcn_readlane((int)cf, 47) |
                             (uint32_t)__builtin_amdgcn_readlane((int)cf, 63);
        if (lane == 0 && w < NE) {
            res_cf[w] = cfw;
            res[w] = (acc ? 1u : 0u) | (tie ? 2u : 0u) | ((uint32_t)(ds & 0xffff) << 16);
            res_a[w] = anx;
            res_b[w] = bnx;
        }
        __syncthreads();                                   // every proposal's result
        LDS_STAMP(5);
        // ---- resolve in proposal order (every wave alike): the taken proposals are
        // the prefix before the first that read an accepted earlier one's change, or
        // up to a stop
        // lane-parallel over the NW proposals: lane q holds proposal q's result
        const bool lq = lane < nq;
        const uint32_t pq = lq ? res[lane] : 0u;
        const uint32_t pcf = lq ? res_cf[lane] : 0u;
        const bool aq = pq & 1u;
        const uint32_t accm = (uint32_t)__ballot(lq && aq);
        const u64 clm = __ballot(lq && (pcf & accm) != 0u);             // read an accepted earlier one's change
        int qstop = nq;
        if (clm) {
            const int qc = __ffsll((unsigned long long)clm) - 1;
            if (qc < qstop) qstop = qc;
        }
        // sum(s_end) after each proposal: prefix over the accepted ones (NW lanes)
        // (DPP row shifts: lanes 0..15 are one row and hold every proposal)
        int pre = (lq && aq) ? (int)(int16_t)(pq >> 16) : 0;
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x111, 0xf, 0xf, false);     // row_shr:1
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x112, 0xf, 0xf, false);     // row_shr:2
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x114, 0xf, 0xf, false);     // row_shr:4
        if constexpr (NE > 8) pre += __builtin_amdgcn_update_dpp(0, pre, 0x118, 0xf, 0xf, false);   // row_shr:8
        const int64_t sum_after = sum_end + (int64_t)pre;
        const int dnq = (t + lane + 1 > t_cap) ? 2 : ((sum_after == n) ? 1 : 0);
        const u64 stq = __ballot(lane < qstop && dnq != 0);            // (code/SA_RRG.py:84), m == 1
        int taken = qstop;
        if (stq) {
            const int qs = __ffsll((unsigned long long)stq) - 1;
            if (qs + 1 < taken) taken = qs + 1;
        }
        ties += __popcll(__ballot(lane < taken && ((pq >> 1) & 1u)));
        if constexpr (TRACE) {
            const int64_t my_sum = rl64(sum_after, w);              // sum(s_end) after this wave's step
            if (w < taken && lane == 0) {
                const int64_t kk = k + w;
                if (st.tr_i) st.tr_i[kk * R + r] = iv;
                if (st.tr_acc) st.tr_acc[kk * R + r] = ((accm >> w) & 1u) ? 1 : 0;
                if (st.tr_sum) st.tr_sum[kk * R + r] = my_sum;
                if (st.tr_dE) st.tr_dE[kk * R + r] = dE;
            }
        }
        sum_end = rl64(sum_after, taken - 1);
        done = __builtin_amdgcn_readlane(dnq, taken - 1);
        t += taken;                                                 // (code/SA_RRG.py:77,82)
        a = res_a[taken - 1];                                       // (:80-81) after the taken steps
        b = res_b[taken - 1];
        // ---- the taken accepted proposals' changes (the level bit of the mark set,
        // its proposal bits cleared: the other proposals that marked the node clear
        // only their own bits, atomically); every proposal clears its marks
        const bool mine = w < taken && ((accm >> w) & 1u);
        if (mine && lane == 0) atomicXor(&lev[iv >> 5], 1u << (iv & 31));
#pragma unroll
        for (int l = 1; l <= T; ++l) {
            if (l <= last) {
                if (lc_fast[l]) {
                    if (lc_in[l]) {
                        const int v = lc_c[l];
                        if (mine) mk[(l - 1) * mkl + v] = (MK)((lc_v[l] ^ 1u) << LVB);   // (repeats store alike)
                        else atomicAnd(mark_word(l, v), ~mark_bit(v));
                    }
                } else {
                    const uint32_t* cl = lst + l * lc;
                    for (int q = lane; q < lc_n[l]; q += 64) {
                        const int v = (int)cl[q];      // (distinct: the list path dedups every level)
                        if (mine) atomicXor(mark_word(l, v), mark_bit(v) | ((1u << LVB) << (MKB * (v & (MPW - 1)))));
                        else atomicAnd(mark_word(l, v), ~mark_bit(v));
                    }
                }
            }
        }
        k += taken;
        pk += (uint32_t)taken;
        LDS_STAMP(6);
#ifdef MJX_SA_PROF
        _acc[7] += 1;                                      // rounds (every wave counts)
#endif
    }
#ifdef MJX_SA_PROF
    if (lane == 0) {
        for (int q = 0; q < 11; ++q) atomicAdd(&mjx_sa_lds_prof[q], (unsigned long long)_acc[q]);
        atomicAdd(&mjx_sa_lds_prof[16 + w], (unsigned long long)_acc[8]);
    }
#endif
    if (TRACE && tid == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    __syncthreads();
    {
        const int64_t col = r >> 6;
        for (int64_t v = tid; v < n; v += NT) {
            if (((lev[v >> 5] ^ lev0s[v >> 5]) >> (v & 31)) & 1u)
                atomicXor((unsigned long long*)&s[v * W + col], 1ull << (r & 63));
        }
    }
    if (w == NE) {
        // the launch's MT position: after the last taken proposal's draws, in the
        // generation it drew from (st.mt holds the old one when the ring ran past a twist)
        const int e = (pk > 0) ? q_end[(pk - 1u) & 63u] : idx0;
        if (((e >> 10) & 1) == gen)
            for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = mt[q];
        if (lane == 0) st.mt_idx[r] = e & 1023;
    }
    if (tid == 0) {
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}

// ---------------------------------------------------------------------------
// The whole CU, level-synchronous (k_sa_lds_cu<D, T>, round 6; kernel option
// lds_cu).  k_sa_lds_wg gives each of its 15 proposals a wave and walks that
// wave through levels 1..T, so every level costs 15 waves' instruction
// streams for a handful of live lanes each (at SA_RRG.py's p = 3: ~5 of 64 at
// level 1) -- the round was VALU-issue bound at four waves a SIMD.  Here the
// round's proposals are evaluated together, one level at a time: the
// (proposal, candidate) items of a level are packed densely over the CU's
// lanes (level 1: proposal q's i_q and its d neighbours; level l: every member
// of C_{l-1} of every proposal and its d neighbours), so a level costs as many
// waves as it has items / 64.  Members go to one CU-wide list per level (node,
// proposal, cached value), appended with one LDS atomic per wave; a barrier
// separates the levels, so a level-l item reads the complete level-(l-1)
// marks and its conflict word (what it read that an earlier proposal changed)
// is final when it is read -- no second pass after the levels.  The marks, the
// change rule, the taken prefix and the accept test are k_sa_lds_wg's; the
// level-0 conflicts (closed neighbourhoods of i_q and i_j meet) are items of
// the level-1 pass, one per pair j < q.  Wave 15 parses the stream into the
// ring exactly as k_sa_lds_wg's parse wave.  Same draws, accepts and state.
struct GeoC {
    int nw;         // uint32 bit words per level
    int cap[4];     // list capacity of levels 1..T (index l)
    int off_lev;
    int off_mk;     // T * nw * 32 16-bit marks (bit q = proposal q, bit 15 = the level value)
    int off_lev0;
    int off_mt;
    int off_list;   // levels 1..T, cap[l] uint32 each: node | q << 16 | cached value << 20
    int off_q;      // ring: i[64], end[64], u[64]
    int off_qc;     // ring, per proposal and candidate j = 0..d: node | dup << 16 | (its neighbours == i) << 17 | (== i) << 21
    int off_qr;     // ring, per proposal and candidate: its row (uint2)
    int off_gln;    // levels 1..T-1: each list entry's row (uint2)
    int off_res;    // per proposal: -2 a s_i, b, u, a and b after; ds, cf and list lengths by parity
    int bytes;
};

// waves of k_sa_lds_cu: 8 (a cheaper barrier, the items fit), 16 with split = 16
static int cu_waves(int split) { return split == 16 ? 16 : 8; }

static bool geometry_cu(int64_t n, int d, int T, GeoC* g);

// k_sa_lds_cu is the LDS kernel at d = 3, 4, p+c-1 = 2, 3 where it fits: by
// default (no kernel options), or asked for (MJX_SA_LDS_CU, split 8 or 16);
// split = 4 / 8 / 16 alone keep k_sa_lds_wg with that many waves
static bool use_cu(int64_t n, int d, int T, uint32_t flags, int split, GeoC* g) {
    if (!(d == 3 || d == 4) || !(T == 2 || T == 3) || !geometry_cu(n, d, T, g)) return false;
    if (flags & MJX_SA_LDS_CU) return true;
    return split == 0 && !(flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR | MJX_SA_LDS_WAVE));
}

static bool geometry_cu(int64_t n, int d, int T, GeoC* g) {
    if (n < 2 || n > 65535 || d < 3 || d > 4 || T < 2 || T > 3) return false;
    g->nw = (int)(((n + 63) / 64) * 2);
    // level 1: 15 proposals x (d + 1); inner levels keep repeats: (d + 1) x the
    // level before; the last level is distinct per proposal: 15 x the ball
    g->cap[0] = 0;
    g->cap[1] = 15 * (d + 1);
    g->cap[2] = (T == 2) ? (int)std::min<int64_t>((int64_t)(d + 1) * g->cap[1], 15 * ball(d, 2))
                         : (d + 1) * g->cap[1];
    g->cap[3] = (T == 3) ? (int)std::min<int64_t>((int64_t)(d + 1) * g->cap[2], 15 * ball(d, 3)) : 0;
    int64_t off = ((int64_t)n * 4 * 2 + 15) / 16 * 16;
    g->off_lev = (int)off;   off += (int64_t)g->nw * 4;
    g->off_mk = (int)off;    off += (int64_t)T * g->nw * 32 * 2;
    g->off_lev0 = (int)off;  off += (int64_t)g->nw * 4;
    g->off_mt = (int)off;    off += MT_N * 4;
    g->off_list = (int)off;  off += (int64_t)(g->cap[1] + g->cap[2] + g->cap[3]) * 4;
    off = (off + 15) / 16 * 16;
    g->off_q = (int)off;     off += 64 * 4 + 64 * 4 + 64 * 8;
    g->off_qc = (int)off;    off += 64 * 5 * 4;
    g->off_qr = (int)off;    off += 64 * 5 * 8;
    g->off_gln = (int)off;   off += (int64_t)(g->cap[1] + (T == 3 ? g->cap[2] : 0)) * 8;
    g->off_res = (int)off;   off += 5 * 16 * 8 + 2 * 2 * 16 * 4 + 2 * 4 * 4 + 4 * 4;
    g->bytes = (int)off;
    return (size_t)off <= kLdsMax;
}

template <int D, int T, int NW, bool TRACE>
__global__ void __launch_bounds__(64 * NW) k_sa_lds_cu(const int32_t* __restrict__ adj, int64_t n, int64_t R,
                                                   int64_t W, u64* __restrict__ s, mjx_sa_state st, int64_t nsteps,
                                                   double par_a, double par_b, double a_cap, double b_cap,
                                                   int64_t t_cap, GeoC geo) {
    static_assert((D == 3 || D == 4) && (T == 2 || T == 3), "level-synchronous LDS SA: d = 3, 4; p+c-1 = 2, 3");
    using MK = uint16_t;
    static_assert(NW == 8 || NW == 16, "8 or 16 waves");
    // NQ proposals a round; waves 0..NI-1 take items, wave TW also the test
    // set-up, wave PW parses the stream
    constexpr int NQ = 15, NI = NW - 1, TW = NW - 2, PW = NW - 1, NT = 64 * NW, LVB = 15, DP1 = D + 1;
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const u64 ltmask = (1ull << lane) - 1ull;
    const int64_t r = blockIdx.x;
    const int nw = geo.nw;
    const int mkl = nw * 32;
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lev = reinterpret_cast<uint32_t*>(smem + geo.off_lev);
    MK* mk = reinterpret_cast<MK*>(smem + geo.off_mk);
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    uint32_t* gl[T + 1];                               // the CU-wide change lists of levels 1..T
    gl[0] = nullptr;
    gl[1] = reinterpret_cast<uint32_t*>(smem + geo.off_list);
#pragma unroll
    for (int l = 2; l <= T; ++l) gl[l] = gl[l - 1] + geo.cap[l - 1];
    int* q_i = reinterpret_cast<int*>(smem + geo.off_q);
    int* q_end = q_i + 64;
    double* q_u = reinterpret_cast<double*>(q_end + 64);
    uint32_t* q_cn = reinterpret_cast<uint32_t*>(smem + geo.off_qc);
    uint2* q_cr = reinterpret_cast<uint2*>(smem + geo.off_qr);
    uint2* gln[T + 1];                                 // the rows of the list entries of levels 1..T-1
    gln[0] = nullptr;
    gln[1] = reinterpret_cast<uint2*>(smem + geo.off_gln);
    gln[2] = (T == 3) ? gln[1] + geo.cap[1] : nullptr;
    gln[T] = nullptr;
    // per proposal, by the test wave at round start: -2 a_q s_i, b_q, u, the
    // schedule after the step
    double* pre_t1 = reinterpret_cast<double*>(smem + geo.off_res);
    double* pre_bh = pre_t1 + 16;
    double* pre_u = pre_bh + 16;
    double* pre_anx = pre_u + 16;
    double* pre_bnx = pre_anx + 16;
    int* dsv = reinterpret_cast<int*>(pre_bnx + 16);                        // [2][16] sum(s_end) change by parity
    uint32_t* cfv = reinterpret_cast<uint32_t*>(dsv + 32);                  // [2][16] conflict bits, being ORed
    uint32_t* cnt = cfv + 32;                                               // [2][4] list lengths by round parity
    int* ctl = reinterpret_cast<int*>(cnt + 8);

    auto bit_of = [&](int v) -> uint32_t { return (lev[v >> 5] >> (v & 31)) & 1u; };
    auto lvl = [&](int t, int v) -> uint32_t { return ((uint32_t)mk[(t - 1) * mkl + v] >> LVB) & 1u; };
    auto mark_word = [&](int t, int v) -> uint32_t* { return reinterpret_cast<uint32_t*>(mk + (t - 1) * mkl + (v & ~1)); };
    auto row = [&](int v) -> uint2 { return *reinterpret_cast<const uint2*>(rows + v * 4); };
    auto unpack = [&](uint2 x, int (&o)[D]) {
        o[0] = (int)(x.x & 0xffffu);
        o[1] = (int)(x.x >> 16);
        o[2] = (int)(x.y & 0xffffu);
        if constexpr (D > 3) o[3] = (int)(x.y >> 16);
    };
    auto nbrs = [&](int v, int (&o)[D]) { unpack(row(v), o); };
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
    };
    // the wave's items appended to a list (with their rows below the last
    // level): one LDS atomic per wave
    auto append = [&](uint32_t* list, uint2* lrow, uint32_t* counter, bool add, uint32_t entry, uint2 erow) {
        const u64 m = __ballot(add);
        if (!m) return;
        uint32_t base = 0;
        if (lane == (int)(__ffsll((unsigned long long)m) - 1)) base = atomicAdd(counter, (uint32_t)__popcll(m));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, __ffsll((unsigned long long)m) - 1);
        if (add) {
            const uint32_t at = base + (uint32_t)__popcll(m & ltmask);
            list[at] = entry;
            if (lrow) lrow[at] = erow;
        }
    };
    // a ring entry's static neighbourhood, by the parse wave when it is parsed:
    // candidate j = 0..d of level 1 (i, then its neighbours), its row, whether
    // it repeats an earlier candidate, which of its neighbours are i
    auto prep = [&](int slot, int iv) {
        const uint2 xi = row(iv);
        int ri[D];
        unpack(xi, ri);
#pragma unroll
        for (int j = 0; j <= D; ++j) {
            const int cand = (j == 0) ? iv : ri[j > 0 ? j - 1 : 0];
            int first = D;
#pragma unroll
            for (int e = D - 1; e >= 0; --e)
                if (ri[e] == cand) first = e;
            const bool dup = j > 0 && (cand == iv || first + 1 < j);
            const uint2 xc = (j == 0) ? xi : row(cand);
            int nv[D];
            unpack(xc, nv);
            uint32_t eqm = 0;
#pragma unroll
            for (int e = 0; e < D; ++e) eqm |= (nv[e] == iv ? 1u : 0u) << e;
            q_cn[slot * DP1 + j] = (uint32_t)cand | (dup ? 1u << 16 : 0u) | (eqm << 17) | ((cand == iv) ? 1u << 21 : 0u);
            q_cr[slot * DP1 + j] = xc;
        }
    };

    // ---- launch setup (k_sa_lds_wg's): rows, level 0, marks cleared, MT state; levels 1..T
    {
        const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * D;
        for (int64_t q = tid; q < n * D; q += NT) {
            const int64_t v = q / D;
            rows[v * 4 + (q - v * D)] = (uint16_t)g[q];
        }
        for (int q = tid; q < nw; q += NT) lev[q] = 0u;
        for (int q = tid; q < T * nw * 16; q += NT) reinterpret_cast<uint32_t*>(mk)[q] = 0u;
        for (int q = tid; q < MT_N; q += NT) mt[q] = st.mt[r * MT_N + q];
        if (tid < 32) {
            dsv[tid] = 0;
            cfv[tid] = 0u;
        }
        if (tid < 8) cnt[tid] = 0u;
        const int64_t col = r >> 6;
        const u64 rbit = 1ull << (r & 63);
        __syncthreads();
        for (int64_t v0 = (int64_t)w * 64; v0 < (int64_t)nw * 32; v0 += NT) {
            const int64_t v = v0 + lane;
            const bool b = v < n && (s[v * W + col] & rbit);
            const u64 m = __ballot(b);
            if (lane < 2) {
                const uint32_t x = (uint32_t)(m >> (32 * lane));
                lev[(v0 >> 5) + lane] = x;
                lev0s[(v0 >> 5) + lane] = x;
            }
        }
        __syncthreads();
        for (int t = 1; t <= T; ++t) {
            for (int v = tid; v < n; v += NT) {
                int nv[D];
                nbrs(v, nv);
                int ones = 0;
#pragma unroll
                for (int q = 0; q < D; ++q) ones += (int)(t == 1 ? bit_of(nv[q]) : lvl(t - 1, nv[q]));
                const uint32_t nb = maj(ones, t == 1 ? bit_of(v) : lvl(t - 1, v));
                mk[(t - 1) * mkl + v] = (MK)(nb << LVB);
            }
            __syncthreads();
        }
    }

    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    double inv_n = 1.0 / (double)n;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(par_a), "+v"(par_b), "+v"(a_cap), "+v"(b_cap), "+v"(inv_n));

    // ---- the proposal ring, parsed by wave PW (k_sa_lds_wg's, and each entry's prep)
    uint32_t npend = 0, pk = 0;
    int gen = 0;
    const int idx0 = idx;
    auto twist = [&]() {
        for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = mt[q];
        lds_twist(mt, lane);
        idx = 0;
        gen ^= 1;
    };
    auto twist_ok = [&]() -> bool {
        const int lg = (pk > 0u) ? ((q_end[(pk - 1u) & 63u] >> 10) & 1) : 0;
        return lg == gen || npend == pk;
    };
    auto parse_window = [&](uint32_t room) -> bool {
        if (idx >= MT_N) {
            if (!twist_ok()) return false;
            twist();
        }
        const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
        uint32_t tw = 0, y = 0;
        bool ok = false;
        if (lane < lim) {
            tw = mt_temper(mt[idx + lane]);
            y = tw & mask;
            ok = y <= rng;
        }
        const u64 okm = __ballot(ok);
        u64 stm = mt_window_starts(ok) & ((lim >= 2) ? ((1ull << (lim - 2)) - 1ull) : 0ull);
        while ((uint32_t)__popcll(stm) > room) stm &= ~(1ull << (63 - __clzll(stm)));
        const uint32_t got = (uint32_t)__popcll(stm);
        const int pos = got ? 66 - __clzll(stm) : 0;
        if (got > 0) {
            const uint32_t x1 = mt_next_lane(tw);
            const uint32_t x2 = mt_next_lane(x1);
            if ((stm >> lane) & 1ull) {
                const int q = (int)((npend + (uint32_t)__popcll(stm & ltmask)) & 63u);
                q_i[q] = (int)y;
                q_u[q] = mt_double(x1, x2);
                q_end[q] = (idx + lane + 3) | (gen << 10);
                prep(q, (int)y);
            }
            npend += got;
            idx += pos;
            return true;
        }
        if (room == 0) return true;
        if (!okm) { idx += lim; return true; }
        const int f = __ffsll((unsigned long long)okm) - 1;
        if (f > 0) { idx += f; return true; }
        if (idx + 2 >= MT_N && !twist_ok()) return false;
        const int iv = __builtin_amdgcn_readlane((int)y, 0);
        idx += 1;
        if (idx >= MT_N) twist();
        const uint32_t w1 = mt_temper(mt[idx]);
        idx += 1;
        if (idx >= MT_N) twist();
        const uint32_t w2 = mt_temper(mt[idx]);
        idx += 1;
        if (lane == 0) {
            const int q = (int)(npend & 63u);
            q_i[q] = iv;
            q_u[q] = mt_double(w1, w2);
            q_end[q] = idx | (gen << 10);
            prep(q, iv);
        }
        npend += 1;
        return true;
    };
    auto room = [&]() -> uint32_t { return 63u - (npend - pk); };

    int64_t k = 0;
    int par = 0;                                       // round parity: the list-length set in use
#ifdef MJX_SA_PROF
    // (slots: 0 publish barrier, 1 level work, 2 level barriers, 3 accept test,
    // 5 resolve + apply; 6 rounds; 7 taken; 8..10 |C_1..3|; wave 0's own at 16 + slot)
    unsigned int _acc[16] = {};
    unsigned long long _t0 = __builtin_amdgcn_s_memtime();
#endif
    while (k < nsteps && done == 0) {
        if (w == PW) {
            while (npend - pk < (uint32_t)NQ)
                if (!parse_window(room())) break;
            if (lane == 0) ctl[0] = (int)npend;
        }
        __syncthreads();                                   // the round's proposals are published
        LDS_STAMP(0);
        const uint32_t npd = (uint32_t)__builtin_amdgcn_readfirstlane(ctl[0]);
        int nq = (int)(npd - pk);
        if (nq > NQ) nq = NQ;
        if ((int64_t)nq > nsteps - k) nq = (int)(nsteps - k);
        uint32_t* cn = cnt + 4 * par;                      // this round's list lengths (zeroed)
        int* dsp = dsv + 16 * par;                         // this round's accumulators (zeroed)
        uint32_t* cfp = cfv + 16 * par;
        // ---- level 1 (items q*(d+1) + j), and the level-0 conflicts (items: pairs j < q)
        if (w < NI) {
            if (w == TW) {
                // each proposal's schedule, -2 a s_i and u (code/SA_RRG.py:74-76,80-81)
                // for the accept test after the levels; the other parity's
                // accumulators and list lengths cleared for the next round
                const bool lq = lane < nq;
                const int q = lq ? lane : 0;
                const int iv = q_i[(pk + (uint32_t)q) & 63u];
                const double u = q_u[(pk + (uint32_t)q) & 63u];
                const uint32_t old_i = bit_of(iv);
                double ah = a, bh = b;
                if (!(ah >= a_cap && bh >= b_cap)) {
                    for (int qq = 0; qq < NQ; ++qq) {
                        if (qq < q) {
                            if (ah < a_cap) ah = par_a * ah;
                            if (bh < b_cap) bh = par_b * bh;
                        }
                    }
                }
                const double si = old_i ? 1.0 : -1.0;
                if (lq) {
                    pre_t1[q] = (-2.0 * ah) * si;
                    pre_bh[q] = bh;
                    pre_u[q] = u;
                    pre_anx[q] = (ah < a_cap) ? par_a * ah : ah;
                    pre_bnx[q] = (bh < b_cap) ? par_b * bh : bh;
                }
                if (lane < 16) {
                    dsv[16 * (par ^ 1) + lane] = 0;
                    cfv[16 * (par ^ 1) + lane] = 0u;
                }
                if (lane < 4) cnt[4 * (par ^ 1) + lane] = 0u;
            }
            const int n1 = nq * DP1, np = nq * (nq - 1) / 2;
            for (int base = 64 * w; base < n1 + np; base += 64 * NI) {
                const int it = base + lane;
                bool add = false;
                uint32_t entry = 0;
                uint2 xc = make_uint2(0u, 0u);
                if (it < n1) {
                    const int q = it / DP1, j = it - q * DP1;
                    const int slot = (int)((pk + (uint32_t)q) & 63u);
                    const uint32_t ce = q_cn[slot * DP1 + j];
                    xc = q_cr[slot * DP1 + j];
                    const int cand = (int)(ce & 0xffffu);
                    int nv[D];
                    unpack(xc, nv);
                    int ones = 0;
#pragma unroll
                    for (int e = 0; e < D; ++e) ones += (int)(bit_of(nv[e]) ^ ((ce >> (17 + e)) & 1u));
                    const uint32_t own = bit_of(cand) ^ ((ce >> 21) & 1u);
                    const uint32_t nb = maj(ones, own);
                    const uint32_t cur = lvl(1, cand);
                    add = !((ce >> 16) & 1u) && nb != cur;
                    if (add) atomicOr(mark_word(1, cand), (1u << q) << (16 * (cand & 1)));
                    entry = (uint32_t)cand | ((uint32_t)q << 16) | (cur << 20);
                } else if (it < n1 + np) {
                    // pair (q, j < q): the closed neighbourhoods of i_q and i_j meet
                    const int k2 = it - n1;
                    int q = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)k2)) * 0.5f);
                    if (q * (q - 1) / 2 > k2) --q;
                    if ((q + 1) * q / 2 <= k2) ++q;
                    const int j = k2 - q * (q - 1) / 2;
                    const int sq = (int)((pk + (uint32_t)q) & 63u), sj = (int)((pk + (uint32_t)j) & 63u);
                    const int iq = (int)(q_cn[sq * DP1] & 0xffffu), ij = (int)(q_cn[sj * DP1] & 0xffffu);
                    int rq[D], rj[D];
                    unpack(q_cr[sq * DP1], rq);
                    unpack(q_cr[sj * DP1], rj);
                    bool meet = iq == ij;
#pragma unroll
                    for (int e = 0; e < D; ++e) meet |= (rj[e] == iq) | (ij == rq[e]);
#pragma unroll
                    for (int e = 0; e < D; ++e)
#pragma unroll
                        for (int f = 0; f < D; ++f) meet |= rj[e] == rq[f];
                    if (meet) atomicOr(&cfp[q], 1u << j);
                }
                append(gl[1], gln[1], &cn[1], add, entry, xc);
            }
        } else if (room() >= 8u) {
            parse_window(room());                          // one window a level: its prep outlasts a level's items
        }
        LDS_STAMP(1);
        __syncthreads();                                   // level-1 marks and C_1 lists complete
        LDS_STAMP(2);
        // the test wave's values, read while the levels run
        const int ql = (lane < nq) ? lane : 0;
        const double bh = pre_bh[ql];
        const double t1 = pre_t1[ql];
        const double u = pre_u[ql];
        const double anx = pre_anx[ql], bnx = pre_bnx[ql];
        // ---- levels 2..T: every member of C_{l-1} of every proposal and its d neighbours
#pragma unroll
        for (int l = 2; l <= T; ++l) {
            if (w < NI) {
                const int nm = (int)cn[l - 1];
                for (int base = 64 * w; base < nm * DP1; base += 64 * NI) {
                    const int it = base + lane;
                    bool add = false;
                    uint32_t entry = 0;
                    uint2 xc = make_uint2(0u, 0u);
                    if (it < nm * DP1) {
                        const int mi = it / DP1, j = it - mi * DP1;
                        const uint32_t me = gl[l - 1][mi];
                        const uint2 xm = gln[l - 1][mi];
                        const int mc = (int)(me & 0xffffu), q = (int)((me >> 16) & 15u);
                        int nm2[D];
                        unpack(xm, nm2);
                        const int c2 = (j == 0) ? mc : nm2[j > 0 ? j - 1 : 0];
                        const uint32_t early = (1u << q) - 1u;
                        xc = row(c2);
                        int nv2[D];
                        unpack(xc, nv2);
                        int ones = 0;
                        uint32_t cfm = 0;
                        // node v at level l-1 as proposal q sees it; the earlier proposals' marks into cfm
                        auto look = [&](int v) -> uint32_t {
                            const uint32_t mb = mk[(l - 2) * mkl + v];
                            cfm |= mb & early;
                            return ((mb >> LVB) ^ (mb >> q)) & 1u;
                        };
#pragma unroll
                        for (int e = 0; e < D; ++e) ones += (int)look(nv2[e]);
                        const uint32_t own = look(c2);
                        if (cfm) atomicOr(&cfp[q], cfm);
                        const uint32_t nb = maj(ones, own);
                        const uint32_t cur = lvl(l, c2);
                        const bool chg = nb != cur;
                        const uint32_t mb = (1u << q) << (16 * (c2 & 1));
                        add = chg;
                        if (l == T) {
                            // the last level counts distinct nodes: the first mark wins
                            if (chg) add = (atomicOr(mark_word(l, c2), mb) & mb) == 0u;
                            if (add) atomicAdd(&dsp[q], cur == 0u ? 2 : -2);
                        } else if (chg) {
                            atomicOr(mark_word(l, c2), mb);
                        }
                        entry = (uint32_t)c2 | ((uint32_t)q << 16) | (cur << 20);
                    }
                    append(gl[l], gln[l], &cn[l], add, entry, xc);
                }
            } else if (w == PW && room() >= 8u) {
                parse_window(room());
            }
            LDS_STAMP(1);
            __syncthreads();                               // level-l marks, C_l lists, conflict bits complete
            LDS_STAMP(2);
        }
        // the lists' first entries this wave applies below, read ahead of the test
        const int c1 = (int)cn[1];
        const int c2 = c1 + (int)cn[2];
        const int c3 = c2 + (T == 3 ? (int)cn[3] : 0);
        auto list_at = [&](int it, int& l) -> uint32_t {
            l = (it < c1) ? 1 : ((it < c2) ? 2 : 3);
            return gl[l][it - ((l == 1) ? 0 : ((l == 2) ? c1 : c2))];
        };
        int l0 = 1;
        const int it0 = 64 * w + lane;
        const uint32_t e0 = (w < PW && it0 < c3) ? list_at(it0, l0) : 0u;
        // ---- delta_H and the Metropolis test of each proposal, lane q of every wave
        // (code/SA_RRG.py:37,74-76): the same arithmetic in every wave, so no
        // barrier hands the results over
        const bool lq = lane < nq;
        const int64_t ds = (int64_t)dsp[ql];
        const uint32_t pcf = lq ? cfp[ql] : 0u;
        const double t2 = bh * (double)(-ds);
        const double num = t1 + t2;
        bool acc;
        bool tie = false;
        double dE = 0.0;
        {
            const float xf = (float)(-num * inv_n);
            const float ef = __expf(xf);
            const float mg = ef * (1e-6f * (1.0f + fabsf(xf))) + 1e-37f;
            if (fabs(u - (double)ef) > (double)mg) {
                acc = u < (double)ef;
                if (TRACE && st.tr_dE) dE = num / (double)n;
            } else {
                dE = num / (double)n;
                const double e = exp(-dE);
                const double prob = (e < 1.0) ? e : 1.0;
                acc = u < prob;
                tie = e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e);
            }
        }
        LDS_STAMP(3);
        // ---- resolve in proposal order (every wave alike, k_sa_lds_wg's rule)
        const bool aq = lq && acc;
        const uint32_t accm = (uint32_t)__ballot(aq);
        const u64 clm = __ballot(lq && (pcf & accm) != 0u);
        int qstop = nq;
        if (clm) {
            const int qc = __ffsll((unsigned long long)clm) - 1;
            if (qc < qstop) qstop = qc;
        }
        int pre = aq ? (int)ds : 0;
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x111, 0xf, 0xf, false);     // row_shr:1
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x112, 0xf, 0xf, false);     // row_shr:2
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x114, 0xf, 0xf, false);     // row_shr:4
        pre += __builtin_amdgcn_update_dpp(0, pre, 0x118, 0xf, 0xf, false);     // row_shr:8
        const int64_t sum_after = sum_end + (int64_t)pre;
        const int dnq = (t + lane + 1 > t_cap) ? 2 : ((sum_after == n) ? 1 : 0);
        const u64 stq = __ballot(lane < qstop && dnq != 0);            // (code/SA_RRG.py:84), m == 1
        int taken = qstop;
        if (stq) {
            const int qs = __ffsll((unsigned long long)stq) - 1;
            if (qs + 1 < taken) taken = qs + 1;
        }
        ties += __popcll(__ballot(lane < taken && tie));
        if constexpr (TRACE) {
            if (w == 0 && lane < taken) {
                const int64_t kk = k + lane;
                const int iv = q_i[(pk + (uint32_t)lane) & 63u];
                if (st.tr_i) st.tr_i[kk * R + r] = iv;
                if (st.tr_acc) st.tr_acc[kk * R + r] = acc ? 1 : 0;
                if (st.tr_sum) st.tr_sum[kk * R + r] = sum_after;
                if (st.tr_dE) st.tr_dE[kk * R + r] = dE;
            }
        }
        sum_end = rl64(sum_after, taken - 1);
        done = __builtin_amdgcn_readlane(dnq, taken - 1);
        t += taken;                                                 // (code/SA_RRG.py:77,82)
        a = __longlong_as_double(rl64(__double_as_longlong(anx), taken - 1));   // (:80-81) after the taken steps
        b = __longlong_as_double(rl64(__double_as_longlong(bnx), taken - 1));
        // ---- the taken accepted proposals' changes (the level bit of the mark set,
        // its proposal bits cleared); every other proposal clears its own bits
        if (w == 0 && lane < taken && aq) {
            const int iv = q_i[(pk + (uint32_t)lane) & 63u];
            atomicXor(&lev[iv >> 5], 1u << (iv & 31));
        }
        if (w < PW) {
            auto apply = [&](uint32_t e, int l) {
                const int v = (int)(e & 0xffffu), q = (int)((e >> 16) & 15u);
                const uint32_t cur = (e >> 20) & 1u;
                const bool mine = q < taken && ((accm >> q) & 1u);
                if (mine) mk[(l - 1) * mkl + v] = (MK)((cur ^ 1u) << LVB);    // (repeats store alike)
                else atomicAnd(mark_word(l, v), ~((1u << q) << (16 * (v & 1))));
            };
            if (it0 < c3) apply(e0, l0);
            for (int it = it0 + 64 * PW; it < c3; it += 64 * PW) {
                int l;
                const uint32_t e = list_at(it, l);
                apply(e, l);
            }
        }
        LDS_STAMP(5);
#ifdef MJX_SA_PROF
        _acc[6] += 1;
        _acc[7] += (unsigned int)taken;
        _acc[8] += cn[1];
        _acc[9] += cn[2];
        _acc[10] += (T == 3) ? cn[3] : 0u;
#endif
        k += taken;
        pk += (uint32_t)taken;
        par ^= 1;
    }
#ifdef MJX_SA_PROF
    if (lane == 0 && w < PW)
        for (int q = 0; q < 11; ++q) atomicAdd(&mjx_sa_lds_prof[q + (w == 0 ? 16 : 0)], (unsigned long long)_acc[q]);   // (16.. wave 0)
    if (lane == 0 && w == PW) {                    // the parse wave's phases at 11..15
        atomicAdd(&mjx_sa_lds_prof[11], (unsigned long long)_acc[0]);
        atomicAdd(&mjx_sa_lds_prof[12], (unsigned long long)_acc[1]);
        atomicAdd(&mjx_sa_lds_prof[13], (unsigned long long)_acc[2]);
        atomicAdd(&mjx_sa_lds_prof[14], (unsigned long long)_acc[3]);
        atomicAdd(&mjx_sa_lds_prof[15], (unsigned long long)_acc[5]);
    }
#endif
    if (TRACE && tid == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    __syncthreads();
    {
        const int64_t col = r >> 6;
        for (int64_t v = tid; v < n; v += NT) {
            if (((lev[v >> 5] ^ lev0s[v >> 5]) >> (v & 31)) & 1u)
                atomicXor((unsigned long long*)&s[v * W + col], 1ull << (r & 63));
        }
    }
    if (w == PW) {
        const int e = (pk > 0) ? q_end[(pk - 1u) & 63u] : idx0;
        if (((e >> 10) & 1) == gen)
            for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = mt[q];
        if (lane == 0) st.mt_idx[r] = e & 1023;
    }
    if (tid == 0) {
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}

// ---------------------------------------------------------------------------
// The whole CU at p + c - 1 = 1 (k_sa_lds_wg1<D, NW, NQ>, configs[0]'s
// SA_RRG.py p = c = 1): NW waves of NQ lane groups, k_sa_lds_multi's step in
// every wave, K = NW * NQ consecutive proposals per round.  Proposal q's
// evaluation stands after an accepted earlier j unless i_j is one of the nodes
// q's lanes read at level 0 (k_sa_lds_multi's rule); across waves that test is
// a TAG word per node: bit j of tag[v] = (i_j == v), set by each proposal with
// one LDS atomic before the round's reads, so a lane ORs the tags of the nodes
// it reads.  The resolution is lane-parallel: proposal q's packed result sits
// in lane q, one ballot finds the first proposal that read an accepted
// earlier one's i, a prefix sum the first stop.  Rounds: proposals published,
// tags set, level 1 evaluated and results written, each behind a workgroup
// barrier.  A wave of its own (wave NW) parses the numpy stream into a ring of
// proposals indexed by their absolute number while the others evaluate (32
// proposals a round: the parse in wave 0 was 60 % of a round); it may run past
// an MT twist with proposals of the old state unconsumed, keeping that state,
// so the stream handed back is numpy's at the end of the last proposal taken.
struct GeoW1 {
    int nw;
    int off_lev;    // 2 * nw level words (levels 0 and 1)
    int off_lev0;
    int off_tag;    // nw * 32 tag words
    int off_mt;
    int off_mtb;    // the MT state before the parser's latest twist
    int off_q;      // ring: i[128], u[128], end[128]
    int off_res;    // per proposal: packed word, a, b after its step, dE
    int bytes;
};

static bool geometry_wg1(int64_t n, int d, int K, GeoW1* g) {
    if (n < 2 || n > 65535 || d < 1 || d > 4 || K < 2 || K > 32) return false;
    g->nw = (int)(((n + 63) / 64) * 2);
    int64_t off = ((int64_t)n * 4 * 2 + 15) / 16 * 16;
    g->off_lev = (int)off;   off += (int64_t)2 * g->nw * 4;
    g->off_lev0 = (int)off;  off += (int64_t)g->nw * 4;
    g->off_tag = (int)off;   off += (int64_t)g->nw * 32 * 4;
    g->off_mt = (int)off;    off += MT_N * 4;
    g->off_mtb = (int)off;   off += MT_N * 4;
    off = (off + 15) / 16 * 16;
    g->off_q = (int)off;     off += 128 * 4 + 128 * 8 + 128 * 4;
    g->off_res = (int)off;   off += 64 * 4 + 64 * 8 * 3 + 4 * 4;
    g->bytes = (int)off;
    return (size_t)off <= kLdsMax;
}

template <int D, int NW, int NQ, bool TRACE>
__global__ void __launch_bounds__(64 * (NW + 1)) k_sa_lds_wg1(const int32_t* __restrict__ adj, int64_t n, int64_t R,
                                                       int64_t W, u64* __restrict__ s, mjx_sa_state st,
                                                       int64_t nsteps, double par_a, double par_b, double a_cap,
                                                       double b_cap, int64_t t_cap, GeoW1 geo) {
    constexpr int G = 64 / NQ;                     // lanes per proposal
    constexpr int K = NW * NQ;                     // proposals per round
    static_assert(D >= 1 && D <= 4 && G >= D + 1 && K <= 32 && NW >= 2, "whole-CU LDS SA at T = 1");
    constexpr int NT = 64 * (NW + 1);
    constexpr int QN = 128;                        // ring slots
    constexpr int RCAP = QN - 1;                   // ring entries ahead of the consumer
    extern __shared__ __align__(16) unsigned char smem[];
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool parser = w == NW;                   // wave NW parses the stream
    const int lane = tid & 63;
    const u64 ltmask = (1ull << lane) - 1ull;
    const int gq = lane / G, gl = lane % G;
    const int qi = parser ? 31 : w * NQ + gq;      // this lane group's proposal in the round
    const int64_t r = blockIdx.x;
    const int nw = geo.nw;
    uint16_t* rows = reinterpret_cast<uint16_t*>(smem);
    uint32_t* lev = reinterpret_cast<uint32_t*>(smem + geo.off_lev);
    uint32_t* lev0s = reinterpret_cast<uint32_t*>(smem + geo.off_lev0);
    uint32_t* tag = reinterpret_cast<uint32_t*>(smem + geo.off_tag);
    uint32_t* mt = reinterpret_cast<uint32_t*>(smem + geo.off_mt);
    uint32_t* mtb = reinterpret_cast<uint32_t*>(smem + geo.off_mtb);
    int* q_i = reinterpret_cast<int*>(smem + geo.off_q);
    double* q_u = reinterpret_cast<double*>(q_i + QN);
    int* q_end = reinterpret_cast<int*>(q_u + QN);
    uint32_t* res = reinterpret_cast<uint32_t*>(smem + geo.off_res);
    double* res_a = reinterpret_cast<double*>(res + 64);
    double* res_b = res_a + 64;
    double* res_e = res_b + 64;
    int* ctl = reinterpret_cast<int*>(res_e + 64);
    auto bit_of = [&](int t, int v) -> uint32_t { return (lev[t * nw + (v >> 5)] >> (v & 31)) & 1u; };
    auto nbrs = [&](int v, int (&o)[D]) {
        const uint2 x = *reinterpret_cast<const uint2*>(rows + v * 4);
        o[0] = (int)(x.x & 0xffffu);
        if constexpr (D > 1) o[1] = (int)(x.x >> 16);
        if constexpr (D > 2) o[2] = (int)(x.y & 0xffffu);
        if constexpr (D > 3) o[3] = (int)(x.y >> 16);
    };
    auto maj = [&](int ones, uint32_t own) -> uint32_t {       // always-stay majority (code/SA_RRG.py:19-20)
        return (2 * ones > D) ? 1u : ((2 * ones < D) ? 0u : own);
    };

    // ---- launch setup: rows, level 0, tags cleared, MT state; level 1 by one sweep
    {
        const int32_t* g = adj + (st.rep_graph ? (int64_t)st.rep_graph[r] : 0) * n * D;
        for (int64_t q = tid; q < n * D; q += NT) {
            const int64_t v = q / D;
            rows[v * 4 + (q - v * D)] = (uint16_t)g[q];
        }
        for (int q = tid; q < 2 * nw; q += NT) lev[q] = 0u;
        for (int q = tid; q < nw * 32; q += NT) tag[q] = 0u;
        for (int q = tid; q < MT_N; q += NT) mt[q] = st.mt[r * MT_N + q];
        for (int q = tid; q < QN; q += NT) q_i[q] = 0;
        const int64_t col = r >> 6;
        const u64 rbit = 1ull << (r & 63);
        __syncthreads();
        for (int64_t v0 = (int64_t)w * 64; v0 < (int64_t)nw * 32; v0 += NT) {
            const int64_t v = v0 + lane;
            const bool b = v < n && (s[v * W + col] & rbit);
            const u64 m = __ballot(b);
            if (lane < 2) {
                const uint32_t x = (uint32_t)(m >> (32 * lane));
                lev[(v0 >> 5) + lane] = x;
                lev0s[(v0 >> 5) + lane] = x;
            }
        }
        __syncthreads();
        for (int64_t v0 = (int64_t)w * 64; v0 < (int64_t)nw * 32; v0 += NT) {
            const int v = (int)(v0 + lane);
            uint32_t nb = 0;
            if (v < n) {
                int nv[D];
                nbrs(v, nv);
                int ones = 0;
#pragma unroll
                for (int q = 0; q < D; ++q) ones += (int)bit_of(0, nv[q]);
                nb = maj(ones, bit_of(0, v));
            }
            const u64 m = __ballot(nb != 0);
            if (lane < 2) lev[nw + (int)(v0 >> 5) + lane] = (uint32_t)(m >> (32 * lane));
        }
        __syncthreads();
    }

    double a = st.a[r], b = st.b[r];
    int64_t t = st.t[r], sum_end = st.sum_end[r];
    int done = st.done[r];
    int idx = st.mt_idx[r];
    int ties = 0;
    const uint32_t rng = (uint32_t)(n - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    double inv_n = 1.0 / (double)n;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(par_a), "+v"(par_b), "+v"(a_cap), "+v"(b_cap), "+v"(inv_n));

    int64_t k = 0;                                 // proposals taken in this launch (absolute ring index)
    // ---- the parser wave: randint(0, n) + rand() pairs (code/SA_RRG.py:73,76) into
    // the ring, one 64-word window per call (as k_sa_lds_wg's wave 0 parses them)
    const int idx0 = idx;
    int64_t produced = 0;                          // proposals in the ring (absolute count)
    int64_t bak_at = -1;                           // proposals >= bak_at end after the latest twist
    auto twist = [&]() {
        for (int q = lane; q < MT_N; q += 64) mtb[q] = mt[q];   // the state of the proposals before it
        bak_at = produced;
        wave_sync();
        lds_twist(mt, lane);
        idx = 0;
    };
    // a second twist while proposals drawn before the first are still to be taken
    // would lose their state: the parser then waits for the consumer (a state
    // yields ~170 proposals, the ring holds 127; the last clause keeps the ring
    // from ever running dry)
    auto can_twist = [&]() -> bool { return bak_at < 0 || k > bak_at || produced == k; };
    // up to `windows` windows while fewer than `want` proposals are ready
    auto refill = [&](int windows, int want) {
        for (int wd = 0; wd < windows; ++wd) {
            const int room = (int)(k + RCAP - produced);
            if (room <= 0 || produced - k >= want) return;
            if (idx >= MT_N) {
                if (!can_twist()) return;
                twist();
            }
            const int lim = (MT_N - idx < 64) ? MT_N - idx : 64;
            uint32_t tw = 0, y = 0;
            bool ok = false;
            if (lane < lim) {
                tw = mt_temper(mt[idx + lane]);
                y = tw & mask;
                ok = y <= rng;
            }
            const u64 okm = __ballot(ok);
            // the proposal starts whose words fit the window, at most `room`
            u64 stm = mt_window_starts(ok) & ((lim >= 2) ? ((1ull << (lim - 2)) - 1ull) : 0ull);
            while (__popcll(stm) > room) stm &= ~(1ull << (63 - __clzll(stm)));
            const int got = __popcll(stm);
            const int pos = got ? 66 - __clzll(stm) : 0;      // after the last start's two words
            const uint32_t x1 = mt_next_lane(tw);
            const uint32_t x2 = mt_next_lane(x1);
            if (got > 0) {
                if ((stm >> lane) & 1ull) {
                    const int e = (int)((produced + __popcll(stm & ltmask)) & (QN - 1));
                    q_i[e] = (int)y;
                    q_u[e] = mt_double(x1, x2);
                    q_end[e] = idx + lane + 3;
                }
                produced += got;
                idx += pos;
                continue;
            }
            if (!okm) { idx += lim; continue; }
            const int f = __ffsll((unsigned long long)okm) - 1;
            if (f > 0) { idx += f; continue; }
            // i is the window's first word and rand()'s two words cross the end of
            // the state: the serial draw twists between them, as numpy does
            if (!can_twist()) return;
            const int iv = __builtin_amdgcn_readlane((int)y, 0);
            idx += 1;
            if (idx >= MT_N) twist();
            const uint32_t w1 = mt_temper(mt[idx]);
            idx += 1;
            if (idx >= MT_N) twist();
            const uint32_t w2 = mt_temper(mt[idx]);
            idx += 1;
            if (lane == 0) {
                const int e = (int)(produced & (QN - 1));
                q_i[e] = iv;
                q_u[e] = mt_double(w1, w2);
                q_end[e] = idx;
            }
            produced += 1;
        }
    };

#ifdef MJX_SA_PROF
    unsigned long long _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _t0 = __builtin_amdgcn_s_memtime();
#endif
    while (k < nsteps && done == 0) {
        if (parser) {
            refill(4, K);                                  // the round's proposals, if the ring fell short
            if (lane == 0) ctl[0] = (int)(produced - k);   // proposals ready for this round
        }
        __syncthreads();                                   // the round's proposals are published
        LDS_STAMP(0);
        const int nready = __builtin_amdgcn_readfirstlane(ctl[0]);   // (rewritten before the next publish)
        int nq = nready;
        if (nq > K) nq = K;
        if ((int64_t)nq > nsteps - k) nq = (int)(nsteps - k);
        const bool act = !parser && qi < nq;
        const int iv = act ? q_i[(k + qi) & (QN - 1)] : 0;
        const double u = act ? q_u[(k + qi) & (QN - 1)] : 0.0;
        if (act && gl == 0) atomicOr(&tag[iv], 1u << qi);
        LDS_STAMP(3);
        __syncthreads();                                   // every proposal's tag
        LDS_STAMP(1);
        int cand = iv;
        uint32_t cur = 0;
        bool chg = false;
        if (parser) {
            refill(2, RCAP);                               // the next rounds', while the proposal waves evaluate
        } else {
        const uint32_t old_i = bit_of(0, iv);
        // level 1: i and its neighbours, level 0 with i flipped
        int ri[D];
        nbrs(iv, ri);
#pragma unroll
        for (int q = 0; q < D; ++q)
            if (gl == q + 1) cand = ri[q];
        bool dup = gl > 0 && cand == iv;
#pragma unroll
        for (int q = 0; q < D; ++q)
            if (q + 1 < gl) dup |= ri[q] == cand;
        int nv[D];
        nbrs(cand, nv);
        const bool live = act && gl <= D && !dup;
        int ones = 0;
        uint32_t tg = tag[cand];
#pragma unroll
        for (int e = 0; e < D; ++e) {
            ones += (int)(bit_of(0, nv[e]) ^ (nv[e] == iv));
            tg |= tag[nv[e]];
        }
        const uint32_t own = bit_of(0, cand) ^ (cand == iv);
        const uint32_t nb = maj(ones, own);
        cur = bit_of(1, cand);
        chg = live && nb != cur;
        const uint32_t cf = live ? (tg & ((1u << qi) - 1u)) : 0u;  // earlier proposals whose i this lane read
        // per group: sum(s_end) change and conflicts
        const u64 up = __ballot(chg && cur == 0u), dn = __ballot(chg && cur != 0u);
        const u64 gm = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (gq * G);
        const int64_t ds = 2 * ((int64_t)__popcll(up & gm) - (int64_t)__popcll(dn & gm));
        uint32_t cfg = cf;                                 // OR over the group's lanes
#pragma unroll
        for (int o = 1; o < G; o <<= 1) cfg |= (uint32_t)__shfl_xor((int)cfg, o, G);
        // schedule of step k + qi (code/SA_RRG.py:80-81): qi multiplications until
        // both reach their caps (~1.2e4 steps into a run), then constant
        double ag = a, bg = b;
        if (!(ag >= a_cap && bg >= b_cap)) {
            for (int q = 0; q < qi; ++q) {
                if (ag < a_cap) ag = par_a * ag;
                if (bg < b_cap) bg = par_b * bg;
            }
        }
        const double an = (ag < a_cap) ? par_a * ag : ag;
        const double bn = (bg < b_cap) ? par_b * bg : bg;
        const double si = old_i ? 1.0 : -1.0;
        const double t1 = (-2.0 * ag) * si;
        const double t2 = bg * (double)(-ds);
        const double num = t1 + t2;
        const float xf = (float)(-num * inv_n);
        const float ef = __expf(xf);
        const float mg = ef * (1e-6f * (1.0f + fabsf(xf))) + 1e-37f;
        bool acc, tie = false;
        double dE = 0.0;
        if (fabs(u - (double)ef) > (double)mg) {
            acc = u < (double)ef;
            if (TRACE && st.tr_dE) dE = num / (double)n;
        } else {
            dE = num / (double)n;
            const double e = exp(-dE);
            const double prob = (e < 1.0) ? e : 1.0;
            acc = u < prob;
            tie = e < 1.0 && fabs(u - e) <= 4.0 * (nextafter(e, 2.0) - e);
        }
        if (gl == 0 && !parser) {
            // proposal qi: the earlier proposals it read (bits < qi), accept and tie
            // flags, sum(s_end) change, the schedule after its step, delta_H
            res[qi] = cfg;
            res[32 + qi] = (acc ? 1u : 0u) | (tie ? 2u : 0u);
            res_a[qi] = an;
            res_b[qi] = bn;
            res_e[qi] = (double)ds;
            if (TRACE) res_e[32 + qi] = dE;
        }
        }
        LDS_STAMP(4);
        __syncthreads();                                   // every proposal's result
        LDS_STAMP(5);
        // ---- resolve (every wave alike, lane-parallel over the K proposals): lane q
        // holds proposal q
        const bool lq = lane < nq;
        const uint32_t cfq = lq ? res[lane] : 0u;
        const uint32_t fl = lq ? res[32 + lane] : 0u;
        const bool accq = fl & 1u;
        const u64 accm = __ballot(accq);
        const u64 clm = __ballot(lq && (cfq & (uint32_t)accm) != 0u);   // read an accepted earlier one's i
        int qstop = nq;
        if (clm) {
            const int qc = __ffsll((unsigned long long)clm) - 1;
            if (qc < qstop) qstop = qc;
        }
        // sum(s_end) after each proposal (prefix over the accepted ones), and stops
        int64_t pre = (lq && accq) ? (int64_t)res_e[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t v = __shfl_up(pre, o, 64);
            if (lane >= o) pre += v;
        }
        const int64_t sum_after = sum_end + pre;
        const int dn_q = (t + lane + 1 > t_cap) ? 2 : ((sum_after == n) ? 1 : 0);
        const u64 stm = __ballot(lane < qstop && dn_q != 0);
        int taken = qstop;
        if (stm) {
            const int qs = __ffsll((unsigned long long)stm) - 1;
            if (qs + 1 < taken) taken = qs + 1;
        }
        const u64 tk = (taken >= 64) ? ~0ull : ((1ull << taken) - 1ull);
        ties += __popcll(__ballot((fl & 2u) != 0u) & tk);
        if (TRACE && w == 0 && lane < taken) {
            const int64_t kk = k + lane;
            if (st.tr_i) st.tr_i[kk * R + r] = q_i[(k + lane) & (QN - 1)];
            if (st.tr_acc) st.tr_acc[kk * R + r] = accq ? 1 : 0;
            if (st.tr_sum) st.tr_sum[kk * R + r] = sum_after;
            if (st.tr_dE) st.tr_dE[kk * R + r] = res_e[32 + lane];
        }
        {
            const int src = taken > 0 ? taken - 1 : 0;
            const int64_t sum_n = __shfl(sum_after, src, 64);
            const int done_n = __shfl(dn_q, src, 64);
            if (taken > 0) {                               // (a round without proposals: none)
                sum_end = sum_n;
                done = done_n;
                t += taken;
                a = res_a[taken - 1];
                b = res_b[taken - 1];
            }
        }
        // ---- the taken accepted proposals: level 1 on their C_1, level 0 at i;
        // every proposal clears its tag
        const bool mine = !parser && qi < taken && ((accm >> qi) & 1ull);
        if (mine) {
            if (chg) {
                const uint32_t bt = 1u << (cand & 31);
                if (cur) atomicAnd(&lev[nw + (cand >> 5)], ~bt);
                else atomicOr(&lev[nw + (cand >> 5)], bt);
            }
            if (gl == 0) atomicXor(&lev[iv >> 5], 1u << (iv & 31));
        }
        if (act && gl == 0) tag[iv] = 0u;
        k += taken;
        LDS_STAMP(6);
#ifdef MJX_SA_PROF
        _acc[7] += 1;                                      // rounds (every wave counts)
#endif
    }
#ifdef MJX_SA_PROF
    if (lane == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&mjx_sa_lds_prof[q], _acc[q]);
#endif

    if (TRACE && tid == 0) {
        for (; k < nsteps; ++k) {
            if (st.tr_i) st.tr_i[k * R + r] = -1;
            if (st.tr_acc) st.tr_acc[k * R + r] = -1;
            if (st.tr_sum) st.tr_sum[k * R + r] = sum_end;
            if (st.tr_dE) st.tr_dE[k * R + r] = 0.0;
        }
    }
    __syncthreads();
    {
        const int64_t col = r >> 6;
        for (int64_t v = tid; v < n; v += NT) {
            if (((lev[v >> 5] ^ lev0s[v >> 5]) >> (v & 31)) & 1u)
                atomicXor((unsigned long long*)&s[v * W + col], 1ull << (r & 63));
        }
    }
    if (parser) {
        // the stream numpy holds after the last proposal taken (before the first:
        // the launch's position), in the state it was drawn from
        const int64_t L = k - 1;
        const int end = (L < 0) ? idx0 : q_end[L & (QN - 1)];
        const bool useb = bak_at >= 0 && L < bak_at;
        for (int q = lane; q < MT_N; q += 64) st.mt[r * MT_N + q] = useb ? mtb[q] : mt[q];
        if (lane == 0) st.mt_idx[r] = end;
    }
    if (tid == 0) {
        st.a[r] = a;
        st.b[r] = b;
        st.t[r] = t;
        st.sum_end[r] = sum_end;
        st.done[r] = done;
        if (st.tr_tie) st.tr_tie[r] += ties;
    }
}

}  // namespace salds
}  // namespace mjx

using namespace mjx;

#ifdef MJX_SA_PROF
extern "C" int mjx_sa_lds_prof_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(salds::mjx_sa_lds_prof), 32 * sizeof(unsigned long long)) != hipSuccess)
        return MJX_EHIP;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(salds::mjx_sa_lds_prof), z, sizeof(z)) != hipSuccess) return MJX_EHIP;
    }
    return MJX_OK;
}
#endif

extern "C" int64_t mjx_sa_lds_bytes(int64_t n, int d, int p, int c) {
    salds::Geo g;
    if (p < 0 || c < 0 || !salds::geometry(n, d, p + c - 1, &g)) return -1;
    return g.bytes;
}

// The LDS bytes and threads per workgroup of the kernel mjx_sa_lds_steps runs
// for (n, d, p, c) and the kernel options (opt_flags, opt_split): the same
// selection as mjx_sa_lds_steps below.
extern "C" int64_t mjx_sa_lds_plan(int64_t n, int d, int p, int c, uint32_t flags, int split, int* threads) {
    if (p < 0 || c < 0) return -1;
    const int T = p + c - 1;
    salds::Geo g;
    if (!salds::geometry(n, d, T, &g)) return -1;
    int th = 64;
    int64_t bytes = g.bytes;
    const bool small_d = d == 3 || d == 4;
    salds::GeoW gw;
    salds::Geo g2;
    const int nwv = salds::wg_waves(n, d, T, split);
    salds::GeoW1 gw1;
    salds::GeoC gc;
    if (salds::use_cu(n, d, T, flags, split, &gc)) {
        th = 64 * salds::cu_waves(split);           // k_sa_lds_cu: item waves + the parser
        bytes = gc.bytes;
    } else if (!(flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR | MJX_SA_LDS_WAVE)) && small_d && T == 1 &&
        salds::geometry_wg1(n, d, 32, &gw1)) {
        th = 320;                                   // k_sa_lds_wg1: 4 waves x 8 proposals + the parser
        bytes = gw1.bytes;
    } else if (!(flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR)) && small_d && T == 1) {
        // k_sa_lds_multi: the one-plane geometry
    } else if (!(flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_WAVE)) && small_d && T >= 2 && T <= 4 &&
               salds::geometry_wg(n, d, T, nwv, &gw)) {
        th = 64 * nwv;
        bytes = gw.bytes;
    } else if (!(flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE)) && small_d && T <= 4 &&
               salds::geometry(n, d, T, &g2, 2)) {
        bytes = g2.bytes;
    }
    if (threads) *threads = th;
    return bytes;
}

extern "C" int mjx_sa_lds_steps(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, uint64_t* s,
                                mjx_sa_state* stp, int64_t nsteps, double par_a, double par_b, double a_cap,
                                double b_cap, int64_t t_cap, void* stream) {
    if (!stp || !adj || !s || R < 1 || nsteps < 0 || p < 0 || c < 0) return MJX_EINVAL;
    if (stp->philox_key) return MJX_EINVAL;             // the LDS kernels replay MT19937 inside the step
    const int T = p + c - 1;
    salds::Geo g;
    if (!salds::geometry(n, d, T, &g)) return MJX_ERANGE;
    const mjx_sa_state st = *stp;
    if (!st.mt || !st.mt_idx || !st.a || !st.b || !st.t || !st.sum_end || !st.done) return MJX_EINVAL;
    if (st.opt_flags & ~(MJX_SA_NO_SPEC | MJX_SA_NO_CONE2 | MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR |
                         MJX_SA_LDS_WAVE | MJX_SA_LDS_CU))
        return MJX_EINVAL;
    if (nsteps == 0) return MJX_OK;
    if (R > INT32_MAX) return MJX_ERANGE;
    const int64_t W = (R + 63) / 64;
    hipStream_t hs = as_stream(stream);
    salds::GeoC gc;
    if (salds::use_cu(n, d, T, st.opt_flags, st.opt_split, &gc)) {
        const bool trc = st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE;
        const int nwc = salds::cu_waves(st.opt_split);
        auto goc = [&](auto kern) -> int {
            MJX_HIP(set_max_lds(kern, gc.bytes), "sa_lds lds");
            kern<<<(unsigned)R, 64 * nwc, (size_t)gc.bytes, hs>>>(adj, n, R, W, (u64*)s, st, nsteps, par_a, par_b,
                                                                  a_cap, b_cap, t_cap, gc);   // item waves + the parser
            MJX_LAUNCH_CHECK("k_sa_lds_cu");
            return MJX_OK;
        };
#define MJX_LDS_CU(DD, NN)                                                                                          \
        if (T == 2) return trc ? goc(salds::k_sa_lds_cu<DD, 2, NN, true>) : goc(salds::k_sa_lds_cu<DD, 2, NN, false>); \
        return trc ? goc(salds::k_sa_lds_cu<DD, 3, NN, true>) : goc(salds::k_sa_lds_cu<DD, 3, NN, false>);
        if (nwc == 16) {
            if (d == 3) { MJX_LDS_CU(3, 16) }
            MJX_LDS_CU(4, 16)
        }
        if (d == 3) { MJX_LDS_CU(3, 8) }
        MJX_LDS_CU(4, 8)
#undef MJX_LDS_CU
    }
    auto go = [&](auto kern) -> int {
        MJX_HIP(set_max_lds(kern, g.bytes), "sa_lds lds");
        kern<<<(unsigned)R, 64, (size_t)g.bytes, hs>>>(adj, d, n, T, R, W, (u64*)s, st, nsteps, par_a, par_b, a_cap,
                                                       b_cap, t_cap, g);
        MJX_LAUNCH_CHECK("k_sa_lds");
        return MJX_OK;
    };
    salds::GeoW1 gw1;
    if (!(st.opt_flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR | MJX_SA_LDS_WAVE)) &&
        (d == 3 || d == 4) && T == 1 && salds::geometry_wg1(n, d, 32, &gw1)) {
        const bool trw = st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE;
        auto gow1 = [&](auto kern) -> int {
            MJX_HIP(set_max_lds(kern, gw1.bytes), "sa_lds lds");
            kern<<<(unsigned)R, 320, (size_t)gw1.bytes, hs>>>(adj, n, R, W, (u64*)s, st, nsteps, par_a, par_b, a_cap,
                                                              b_cap, t_cap, gw1);          // 4 waves + the parser
            MJX_LAUNCH_CHECK("k_sa_lds_wg1");
            return MJX_OK;
        };
        if (d == 3) return trw ? gow1(salds::k_sa_lds_wg1<3, 4, 8, true>) : gow1(salds::k_sa_lds_wg1<3, 4, 8, false>);
        return trw ? gow1(salds::k_sa_lds_wg1<4, 4, 8, true>) : gow1(salds::k_sa_lds_wg1<4, 4, 8, false>);
    }
    if (!(st.opt_flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_PAIR)) && (d == 3 || d == 4) && T == 1) {
        const bool trm = st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE;
        auto gom = [&](auto kern) -> int {
            MJX_HIP(set_max_lds(kern, g.bytes), "sa_lds lds");
            kern<<<(unsigned)R, 64, (size_t)g.bytes, hs>>>(adj, n, R, W, (u64*)s, st, nsteps, par_a, par_b, a_cap,
                                                           b_cap, t_cap, g);
            MJX_LAUNCH_CHECK("k_sa_lds_multi");
            return MJX_OK;
        };
        if (d == 3) return trm ? gom(salds::k_sa_lds_multi<3, 8, true>) : gom(salds::k_sa_lds_multi<3, 8, false>);
        return trm ? gom(salds::k_sa_lds_multi<4, 8, true>) : gom(salds::k_sa_lds_multi<4, 8, false>);
    }
    salds::GeoW gw;
    const int nwv = salds::wg_waves(n, d, T, st.opt_split);
    if (!(st.opt_flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE | MJX_SA_LDS_WAVE)) && (d == 3 || d == 4) && T >= 2 &&
        T <= 4 && salds::geometry_wg(n, d, T, nwv, &gw)) {
        const bool trw = st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE;
        auto gow = [&](auto kern) -> int {
            MJX_HIP(set_max_lds(kern, gw.bytes), "sa_lds lds");
            kern<<<(unsigned)R, 64 * nwv, (size_t)gw.bytes, hs>>>(adj, n, R, W, (u64*)s, st, nsteps, par_a, par_b,
                                                                 a_cap, b_cap, t_cap, gw);
            MJX_LAUNCH_CHECK("k_sa_lds_wg");
            return MJX_OK;
        };
#define MJX_LDS_WG3(DD, TT)                                                                                       \
        if (nwv == 4) return trw ? gow(salds::k_sa_lds_wg<DD, TT, 4, true>) : gow(salds::k_sa_lds_wg<DD, TT, 4, false>); \
        if (nwv == 16) return trw ? gow(salds::k_sa_lds_wg<DD, TT, 16, true>) : gow(salds::k_sa_lds_wg<DD, TT, 16, false>); \
        return trw ? gow(salds::k_sa_lds_wg<DD, TT, 8, true>) : gow(salds::k_sa_lds_wg<DD, TT, 8, false>);
#define MJX_LDS_WG(DD)                       \
        switch (T) {                         \
            case 2: { MJX_LDS_WG3(DD, 2) }   \
            case 3: { MJX_LDS_WG3(DD, 3) }   \
            default: { MJX_LDS_WG3(DD, 4) }  \
        }
        if (d == 3) { MJX_LDS_WG(3) }
        MJX_LDS_WG(4)
#undef MJX_LDS_WG
#undef MJX_LDS_WG3
    }
    salds::Geo g2;
    if (!(st.opt_flags & (MJX_SA_LDS_SERIAL | MJX_SA_LDS_SINGLE)) && (d == 3 || d == 4) && T <= 4 &&
        salds::geometry(n, d, T, &g2, 2)) {
        auto gop = [&](auto kern) -> int {
            MJX_HIP(set_max_lds(kern, g2.bytes), "sa_lds lds");
            kern<<<(unsigned)R, 64, (size_t)g2.bytes, hs>>>(adj, n, R, W, (u64*)s, st, nsteps, par_a, par_b, a_cap,
                                                            b_cap, t_cap, g2);
            MJX_LAUNCH_CHECK("k_sa_lds_pair");
            return MJX_OK;
        };
        const bool trp = st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE;
#define MJX_LDS_PAIR(DD)                                                                                   \
        switch (T) {                                                                                       \
            case 1: return trp ? gop(salds::k_sa_lds_pair<DD, 1, true>) : gop(salds::k_sa_lds_pair<DD, 1, false>); \
            case 2: return trp ? gop(salds::k_sa_lds_pair<DD, 2, true>) : gop(salds::k_sa_lds_pair<DD, 2, false>); \
            case 3: return trp ? gop(salds::k_sa_lds_pair<DD, 3, true>) : gop(salds::k_sa_lds_pair<DD, 3, false>); \
            default: return trp ? gop(salds::k_sa_lds_pair<DD, 4, true>) : gop(salds::k_sa_lds_pair<DD, 4, false>); \
        }
        if (d == 3) { MJX_LDS_PAIR(3) }
        MJX_LDS_PAIR(4)
#undef MJX_LDS_PAIR
    }
    if (!(st.opt_flags & MJX_SA_LDS_SERIAL) && (d == 3 || d == 4) && T <= 4) {
        auto gof = [&](auto kern) -> int {
            MJX_HIP(set_max_lds(kern, g.bytes), "sa_lds lds");
            kern<<<(unsigned)R, 64, (size_t)g.bytes, hs>>>(adj, n, R, W, (u64*)s, st, nsteps, par_a, par_b, a_cap,
                                                           b_cap, t_cap, g);
            MJX_LAUNCH_CHECK("k_sa_lds_fast");
            return MJX_OK;
        };
        const bool tr = st.tr_i || st.tr_acc || st.tr_sum || st.tr_dE;
#define MJX_LDS_FAST(DD)                                                                                   \
        switch (T) {                                                                                       \
            case 1: return tr ? gof(salds::k_sa_lds_fast<DD, 1, true>) : gof(salds::k_sa_lds_fast<DD, 1, false>); \
            case 2: return tr ? gof(salds::k_sa_lds_fast<DD, 2, true>) : gof(salds::k_sa_lds_fast<DD, 2, false>); \
            case 3: return tr ? gof(salds::k_sa_lds_fast<DD, 3, true>) : gof(salds::k_sa_lds_fast<DD, 3, false>); \
            default: return tr ? gof(salds::k_sa_lds_fast<DD, 4, true>) : gof(salds::k_sa_lds_fast<DD, 4, false>); \
        }
        if (d == 3) { MJX_LDS_FAST(3) }
        MJX_LDS_FAST(4)
#undef MJX_LDS_FAST
    }
    switch (d) {
        case 3: return go(salds::k_sa_lds<3>);
        case 4: return go(salds::k_sa_lds<4>);
        case 6: return go(salds::k_sa_lds<6>);
        default: return go(salds::k_sa_lds<0>);
    }
}
