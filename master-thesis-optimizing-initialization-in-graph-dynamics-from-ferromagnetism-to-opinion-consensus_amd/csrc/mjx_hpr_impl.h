// History-passing reinforcement (HPR) on d-regular graphs: the edge-message
// update, node marginals and bias refresh of code/HPR_pytorch_RRG.py.
//
// Message layout (the reference's, so chi arrays are drop-in):
//   row r < E  : G.edges[r] = (u, v), message u -> v;  row r + E: v -> u
//                (code/HPR_pytorch_RRG.py:277-285)
//   column of (x_a, x_b) = idx(x_a) * 2^T + idx(x_b), idx(x) = sum_k [x_k = -1] 2^(T-1-k)
//                (order_gpu, code/HPR_pytorch_RRG.py:46-61)
//
// HPr_dp (code/HPR_pytorch_RRG.py:183-218) for the message a -> b:
//   chi_new(x_a, x_b) = w(x_a[0]) [x_a[T-1] = attr] sum_{x_k1..} prod_m M_m(x_km, x_a)
//                        * prod_t allowed_t(rho_t, x_b[t])
//   M_m(x_k, x_a) = bias_{k_m}(x_k[0]) chi^{k_m -> a}(x_k, x_a), rho_t = number of +1
//   among the d-1 incoming neighbours at time t, allowed_t = the majority /
//   always-stay trajectory condition (t < T-1) or the attractor condition
//   (t = T-1) of code/HPR_pytorch_RRG.py:14-29, w = exp(-lmbd x_a[0]/n).
//
// Evaluation here (exact rearrangement of the same sum, no approximation):
//   * the count table of the first d-2 incoming neighbours is built by direct
//     convolution in registers (base d-1 digits per time step);
//   * allowed_t is a one-sided interval in rho_t whose direction depends only on
//     x_a, so the table is turned into directional cumulative sums once per x_a;
//   * the last neighbour is folded in as out(x_b) = sum_x M_last(x) CS[corner(x, x_b)].
//   x_a is a compile-time constant per wave (template), so every index above is
//   resolved at compile time and the state never leaves VGPRs.
// Work per (edge, valid x_a) at d=4, T=4: 256 + ~220 + <=256 FMAs/adds.
//
// Kernel geometry: a workgroup owns a tile of NT = 64/d nodes; lane = one
// outgoing message (node a, neighbour slot m) of the tile; wave w handles the
// valid x_a values 2q(+1), q in [w*XPW, (w+1)*XPW).  The d incoming rows of each
// tile node (every incoming message is read once per update) are staged in LDS
// with a +1 pad per row (conflict-free strided reads).
#pragma once
#include "mjx_common.h"
#include <stdlib.h>
#include <type_traits>
#include <utility>

namespace mjx {
namespace hpr {

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

constexpr int ipow(int b, int e) { return e == 0 ? 1 : b * ipow(b, e - 1); }
// spin (+1/-1) of trajectory index x at time t (index bit = 1 means -1)
constexpr int spin(int x, int t, int T) { return ((x >> (T - 1 - t)) & 1) ? -1 : 1; }
constexpr int bit01(int x, int t, int T) { return spin(x, t, T) > 0 ? 1 : 0; }
constexpr int digit(int idx, int t, int T, int base) { return (idx / ipow(base, T - 1 - t)) % base; }
constexpr int maxdigit(int idx, int T, int base) {
    int m = 0;
    for (int t = 0; t < T; ++t) m = digit(idx, t, T, base) > m ? digit(idx, t, T, base) : m;
    return m;
}
constexpr int xoff(int x, int T, int base) {
    int o = 0;
    for (int t = 0; t < T; ++t) o += bit01(x, t, T) * ipow(base, T - 1 - t);
    return o;
}
constexpr int floor_div2(int a) { return a >= 0 ? a / 2 : -((-a + 1) / 2); }
constexpr int ceil_div2(int a) { return -floor_div2(-a); }

// target spin s_t and reference spin prev_t of the condition on time t
constexpr int cond_s(int XA, int t, int T, int P) { return t < T - 1 ? spin(XA, t + 1, T) : spin(XA, P, T); }
constexpr int cond_prev(int XA, int t, int T) { return t < T - 1 ? spin(XA, t, T) : spin(XA, T - 1, T); }

// Corner of the table box for last-neighbour trajectory x and receiver x_b, or -1
// when the box is empty.  Table digits rho_t in [0, K] count the +1 spins of the
// first K = d-2 incoming neighbours; the last one adds bit01(x, t).
// sigma_t = 2(rho_t + b) - (d-1) + y_t  (code/HPR_pytorch_RRG.py:212, rho -> 2 rho - d + 1).
constexpr int corner(int XA, int x, int XB, int T, int P, int D) {
    const int K = D - 2, base = K + 1;
    int idx = 0;
    for (int t = 0; t < T; ++t) {
        const int s = cond_s(XA, t, T, P), prev = cond_prev(XA, t, T);
        const int b = bit01(x, t, T), y = spin(XB, t, T);
        int dg = 0;
        if (s > 0) {   // sigma > 0, or sigma == 0 and prev == +1
            const int thr = prev > 0 ? 0 : 1;
            int lo = ceil_div2(D - 1 - y + thr) - b;
            if (lo > K) return -1;
            dg = lo < 0 ? 0 : lo;
        } else {       // sigma < 0, or sigma == 0 and prev == -1
            const int thr = prev < 0 ? 0 : -1;
            int hi = floor_div2(D - 1 - y + thr) - b;
            if (hi < 0) return -1;
            dg = hi > K ? K : hi;
        }
        idx += dg * ipow(base, T - 1 - t);
    }
    return idx;
}

template <typename S> struct Vec16;
template <> struct Vec16<float> { typedef float4 T; static constexpr int N = 4; };
template <> struct Vec16<double> { typedef double2 T; static constexpr int N = 2; };

template <typename S, int T, int P, int D>
struct Cfg {
    static constexpr int X = 1 << T;          // trajectories per node
    static constexpr int NC = X * X;          // columns per message row
    static constexpr int K = D - 2;           // neighbours in the register table
    static constexpr int BASE = K + 1;
    static constexpr int NS = ipow(BASE, T);  // table size
    static constexpr int NT = 64 / D;         // nodes per tile
    static constexpr int NL = NT * D;         // active lanes (messages) per tile
    static constexpr int NVALID = X / 2;      // valid x_a per attr value
    static constexpr int NW = NVALID < 4 ? NVALID : 4;
    static constexpr int XPW = NVALID / NW;   // valid x_a per wave
    static constexpr int STRIDE = NC + 1;     // padded LDS row stride (elements)
    static constexpr size_t LDS = (size_t)NL * STRIDE * sizeof(S) + (size_t)NL * 2 * sizeof(S) +
                                  (size_t)NW * 64 * sizeof(S);
};

// Compile-time index tables of one (T, P, D, XA) instance.
template <int T, int P, int D, int XA>
struct Tabs {
    static constexpr int X = 1 << T, K = D - 2, BASE = K + 1, NS = ipow(BASE, T);
    struct Data {
        int xo[X];               // table offset of a neighbour trajectory
        int maxd[NS];            // largest digit of a table index
        int dg[T][NS];           // digit t of a table index
        int dir[T];              // +1: suffix sums in dim t, -1: prefix sums
        int cn[X][X];            // corner(x, xb) or -1
    };
    static constexpr Data make() {
        Data d{};
        for (int x = 0; x < X; ++x) d.xo[x] = xoff(x, T, BASE);
        for (int i = 0; i < NS; ++i) {
            d.maxd[i] = maxdigit(i, T, BASE);
            for (int t = 0; t < T; ++t) d.dg[t][i] = digit(i, t, T, BASE);
        }
        for (int t = 0; t < T; ++t) d.dir[t] = cond_s(XA, t, T, P);
        for (int x = 0; x < X; ++x)
            for (int xb = 0; xb < X; ++xb) d.cn[x][xb] = corner(XA, x, xb, T, P, D);
        return d;
    }
    static constexpr Data v = make();
};

// out[XB] for one compile-time x_a; returns the partial row sum.
template <int D>
__device__ __forceinline__ int a_local_of(int lane) { return lane / D; }

// HALF: the buffer holds only the valid-x_a half of each incoming row,
// element x_k * 2^(T-1) + (x_a >> 1).  QL (with HALF): the rows are in the
// decay-split layout (qpos below) and the buffer holds their VV and IV
// quadrants, element (x_k valid ? 0 : H^2) + (x_k >> 1) * H + (x_a >> 1), H =
// 2^(T-1); the IV entries (x_k invalid) are stored undecayed and scaled by sc.
// BSOA > 0: the biases as two arrays, b(+1) of slot s at s and b(-1) at BSOA + s
// (else interleaved at 2s, 2s + 1).
template <typename S, int T, int P, int D, int XA, int RS = Cfg<S, T, P, D>::STRIDE, bool HALF = false,
          bool QL = false, int BSOA = 0>
__device__ __forceinline__ S xa_messages(const S* __restrict__ rows, const S* __restrict__ bias, int a_local, int m,
                                         S w, S (&out)[1 << T], S sc = S(1)) {
    using C = Cfg<S, T, P, D>;
    using TB = Tabs<T, P, D, XA>;
    constexpr int X = C::X, K = C::K, BASE = C::BASE, NS = C::NS;
    // M_j(x) = bias_{k_j}(x[0]) chi^{k_j -> a}(x, x_a) for the d-1 incoming
    // neighbours other than the receiver (slot m), read from LDS when needed:
    // the first straight into the table, the middle ones by the convolution,
    // the last one after the cumulative sums (short live ranges: VGPRs)
    auto loadM = [&](int j, S (&Mj)[X]) {
        const int slot = a_local * D + (j < m ? j : j + 1);
        const S bp = BSOA ? bias[slot] : bias[2 * slot], bm = BSOA ? bias[BSOA + slot] : bias[2 * slot + 1];
        if constexpr (QL) {
            constexpr int H = X / 2;
            const S* r = rows + slot * RS + (XA >> 1);
            const S bps = bp * sc, bms = bm * sc;
#pragma unroll
            for (int x = 0; x < X; ++x) {
                const bool valid = (x & 1) == (XA & 1);              // x_k[T-1] = attr, like x_a
                const int e = (valid ? 0 : H * H) + (x >> 1) * H;
                Mj[x] = (x < X / 2 ? (valid ? bp : bps) : (valid ? bm : bms)) * r[e];
            }
        } else {
            constexpr int CS = HALF ? X / 2 : X;          // stride between x_k
            const S* r = rows + slot * RS + (HALF ? (XA >> 1) : XA);
#pragma unroll
            for (int x = 0; x < X; ++x) Mj[x] = (x < X / 2 ? bp : bm) * r[x * CS];
        }
    };
    // count table of the first K neighbours
    S tab[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) tab[i] = S(0);
    if constexpr (K == 0) {
        tab[0] = S(1);
    } else {
        {
            S M0[X];
            loadM(0, M0);
#pragma unroll
            for (int x = 0; x < X; ++x) tab[TB::v.xo[x]] = M0[x];
        }
        // in place, sources in decreasing index: every target i + xo[x] > i has
        // already given up its own value, and the all-(-1) trajectory (xo = 0)
        // rescales the source itself (one table live instead of two: VGPRs)
#pragma unroll
        for (int j = 1; j < K; ++j) {
            S Mj[X];
            loadM(j, Mj);
#pragma unroll
            for (int i = NS - 1; i >= 0; --i) {
                if (TB::v.maxd[i] <= j) {   // table holds j neighbours: digits <= j
                    const S t = tab[i];
#pragma unroll
                    for (int x = 0; x < X; ++x) {
                        if (TB::v.xo[x] == 0) tab[i] = t * Mj[x];
                    }
#pragma unroll
                    for (int x = 0; x < X; ++x) {
                        if (TB::v.xo[x] != 0) tab[i + TB::v.xo[x]] += t * Mj[x];
                    }
                }
            }
        }
    }
    // directional cumulative sums: suffix in dims whose target spin is +1, prefix otherwise
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int wt = ipow(BASE, T - 1 - t);
        if (TB::v.dir[t] > 0) {
#pragma unroll
            for (int i = NS - 1; i >= 0; --i)
                if (TB::v.dg[t][i] < K) tab[i] += tab[i + wt];
        } else {
#pragma unroll
            for (int i = 0; i < NS; ++i)
                if (TB::v.dg[t][i] > 0) tab[i] += tab[i - wt];
        }
    }
    // fold in the last neighbour
    S Ml[X];
    __builtin_amdgcn_sched_barrier(0);
    loadM(D - 2, Ml);
    S rs = S(0);
#pragma unroll
    for (int xb = 0; xb < X; ++xb) {
        S acc = S(0);
#pragma unroll
        for (int x = 0; x < X; ++x) {
            const int cn = TB::v.cn[x][xb];
            if (cn >= 0) acc += Ml[x] * tab[cn];
        }
        acc *= w;
        out[xb] = acc;
        rs += acc;
    }
    return rs;
}

#ifdef MJX_HPR_PROF
// [0..3] k_hpr_update phases; [4..9] hpr_update_pipe phases (issue, compute,
// vmcnt wait, barrier 1, epilogue, barrier 2); [10..17] pipe compute per wave
__device__ unsigned long long mjx_hpr_prof[32];
#define MJX_PROF_MARK(k) do { const unsigned long long _c = clock64(); if ((threadIdx.x & 63) == 0) atomicAdd(&mjx_hpr_prof[k], _c - _t0); _t0 = _c; } while (0)
#else
#define MJX_PROF_MARK(k) do {} while (0)
#endif

template <typename S, int T, int P, int D>
__global__ void __launch_bounds__((64 * Cfg<S, T, P, D>::NW))
k_hpr_update(const S* __restrict__ chi_in, S* __restrict__ chi_out, const S* __restrict__ biases,
             const int32_t* __restrict__ nbr, const int32_t* __restrict__ in_row, const int32_t* __restrict__ out_row,
             int64_t n, int attr_plus, S w_plus, S w_minus, S damp) {
    using C = Cfg<S, T, P, D>;
    constexpr int X = C::X, NC = C::NC, NT = C::NT, NL = C::NL, NW = C::NW, XPW = C::XPW;
    extern __shared__ __align__(16) unsigned char smem[];
    S* rows = reinterpret_cast<S*>(smem);
    S* bias = rows + NL * C::STRIDE;
    S* red = bias + NL * 2;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int64_t a0 = (int64_t)blockIdx.x * NT;
#ifdef MJX_HPR_PROF
    unsigned long long _t0 = clock64();
#endif
    const int nt = (int)((n - a0) < NT ? (n - a0) : NT);   // nodes in this tile
    const int nl = nt * D;
    // ---- stage the incoming rows of the tile's nodes and their sources' biases.
    // Three phases so that one tile pays two memory round trips, not one per
    // row: every row index, then every 16-B row piece in flight at once (a
    // wave instruction reads a whole 1 KB row at T=4 fp32), then the LDS image.
    {
        using V = typename Vec16<S>::T;
        constexpr int VN = Vec16<S>::N;
        constexpr int VPR = NC / VN;                 // 16-B vectors per row
        constexpr int IT = (NL * VPR + 64 * NW - 1) / (64 * NW);
        // branch-free loads (indices clamped into the tile): a load under a
        // per-lane branch is followed by its own vmcnt(0) wait
        const int qmax = nl * VPR - 1;
        int64_t src[IT];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            int q = tid + k * 64 * NW;
            q = q < qmax ? q : qmax;
            src[k] = (int64_t)in_row[a0 * D + q / VPR] * NC + (q % VPR) * VN;
        }
        const int bq = tid < nl ? tid : nl - 1;
        const int64_t bsrc = nbr[a0 * D + bq];
        V buf[IT];
#pragma unroll
        for (int k = 0; k < IT; ++k) buf[k] = *reinterpret_cast<const V*>(chi_in + src[k]);
        const S bp = biases[2 * bsrc], bm = biases[2 * bsrc + 1];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int q = tid + k * 64 * NW;
            if (q <= qmax) {
                const int slot = q / VPR, v = q % VPR;
                const S* xs = reinterpret_cast<const S*>(&buf[k]);
#pragma unroll
                for (int e = 0; e < VN; ++e) rows[slot * C::STRIDE + v * VN + e] = xs[e];
            }
        }
        if (tid < nl) {
            bias[2 * tid] = bp;
            bias[2 * tid + 1] = bm;
        }
    }
    __syncthreads();
    MJX_PROF_MARK(0);
    const bool active = lane < nl;
    const int a_local = lane / D, m = lane % D;
    S out[XPW][X];
    S rs = S(0);
    if (active) {
        static_for<0, XPW>([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            // the x_a pair 2q, 2q+1 differ only in x_a[T-1]; attr picks the valid one
            static_for<0, NW>([&](auto ww) {
                constexpr int wv = decltype(ww)::value;
                constexpr int q = wv * XPW + i;
                if (wave == wv) {
                    constexpr int XP = 2 * q, XM = 2 * q + 1;      // x_a[T-1] = +1 / -1
                    const S wgt0 = (XP < X / 2) ? w_plus : w_minus;
                    if (attr_plus) rs += xa_messages<S, T, P, D, XP>(rows, bias, a_local, m, wgt0, out[i]);
                    else rs += xa_messages<S, T, P, D, XM>(rows, bias, a_local, m, wgt0, out[i]);
                }
            });
        });
    }
    MJX_PROF_MARK(1);
    red[wave * 64 + lane] = rs;
    __syncthreads();
    MJX_PROF_MARK(2);
    if (!active) return;
    S tot = S(0);
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += red[w * 64 + lane];
    // chi <- damp * chi_new / rowsum + (1 - damp) * chi_old   (code/HPR_pytorch_RRG.py:215)
    const S inv = S(1) / tot;
    const S keep = S(1) - damp;
    const int64_t orow = out_row[(a0 + a_local) * D + m];
    const S* old = chi_in + orow * NC;
    S* dst = chi_out + orow * NC;
#pragma unroll
    for (int i = 0; i < XPW; ++i) {
        const int q = wave * XPW + i;
        const int cv = (attr_plus ? 2 * q : 2 * q + 1) * X;     // valid block
        const int ci = (attr_plus ? 2 * q + 1 : 2 * q) * X;     // x_a[T-1] != attr: chi_new = 0
#pragma unroll
        for (int xb = 0; xb < X; ++xb) {
            dst[cv + xb] = damp * (out[i][xb] * inv) + keep * old[cv + xb];
            dst[ci + xb] = keep * old[ci + xb];
        }
    }
#ifdef MJX_HPR_PROF
    __builtin_amdgcn_s_waitcnt(0);
#endif
    MJX_PROF_MARK(3);
}

// ---- decay-split message layout (the HPR loop's own state) --------------------
// A row's entries with an invalid sender trajectory (x_s[T-1] != attr) are never
// produced by HPr_dp: chi_new = 0 there, so the update only damps them,
// chi_t = (1-damp)^t chi_0 (code/HPR_pytorch_RRG.py:215 with chi_mat2 = 0).  The
// loop state therefore keeps every row as four quadrants of H^2 entries (H =
// 2^(T-1); v/i = valid/invalid sender, then receiver):
//   VV | VI | IV | II,   position qpos(x_s, x_r) = quad * H^2 + (x_s >> 1) * H + (x_r >> 1)
// VV and VI (the first half) are rewritten by every update; IV and II keep the
// undecayed chi_0 and are read with the scale (1-damp)^t (device memory, one
// per iteration).  The update reads the old first half (damping), the VV and
// IV quadrants of its incoming rows (x_a valid) and writes the first half: 1.5
// instead of 3 KB per message at T = 4 fp32; the marginals weigh each product
// by scale^(number of invalid senders) (k_hpr_edge_z_q).
__host__ __device__ constexpr int qpos(int xs, int xr, int T, int pv) {
    return ((((xs & 1) != pv) ? 2 : 0) + (((xr & 1) != pv) ? 1 : 0)) * (1 << (2 * T - 2)) +
           (xs >> 1) * (1 << (T - 1)) + (xr >> 1);
}

// ---- software-pipelined form (fp32, T = 4: 1 KB message rows) ---------------
// One persistent 512-thread workgroup per CU walks tiles t = blockIdx.x,
// + gridDim.x, ...; wave w owns the valid x_a 2w(+1) (XPW = 1).  Everything a
// tile reads from HBM arrives by LDS-DMA (no VGPRs) while the previous work
// computes:
//   * the incoming rows of tile i+1, only their valid-x_a half (the update
//     reads chi^{k->a}(x_k, x_a) for x_a[T-1] = attr only: 128 of 256
//     columns), one float per lane (global_load_lds_dword), into buffer
//     (i+1)&1 with a 129-float row stride (conflict-free M reads);
//   * the old rows of tile i (damping), whole (global_load_lds_dwordx4, one
//     row per wave instruction), at a 260-float stride (conflict-free
//     16-B epilogue reads);
//   * the index rows (in_row, out_row, nbr) of tile i+2 and the sources'
//     biases of tile i+1, read back from LDS (round 5: scalar index loads
//     share lgkmcnt with the DP's LDS reads and held up its first one, and a
//     per-lane out_row load made the loop latch wait for the epilogue's
//     stores; see hpr_update_q3 below, the decay-split form).
constexpr int PIPE_HRS = 129;       // half-row stride (floats) of the incoming-row buffers
constexpr int PIPE_ORS = 260;       // old-row stride (floats): 1040 B, 16-B aligned DMA bases

template <int T, int P, int D>
struct PipeCfg {
    using C = Cfg<float, T, P, D>;
    static constexpr int NW = 8, NL = C::NL, NT = C::NT;
    static constexpr int RPW = (NL + NW - 1) / NW;            // rows per wave per tile
    static constexpr size_t BUF = (size_t)64 * PIPE_HRS;       // floats per incoming buffer
    static constexpr size_t OLD = (size_t)64 * PIPE_ORS;       // floats of the old-row buffer
    static constexpr size_t LDS = (2 * BUF + OLD + 2 * 128 + 3 * 192 + (size_t)NW * 64) * sizeof(float);
};

__device__ __forceinline__ void glds16(const float* gsrc, uint32_t lds_byte_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte_addr)
                 : "memory");
}

__device__ __forceinline__ void glds4(const float* gsrc, uint32_t lds_byte_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte_addr)
                 : "memory");
}

// The tile-index plumbing both pipelined updates share: the three index rows
// of a tile by LDS-DMA (wave 0), this wave's rows read back by LDS broadcast,
// the sources' biases by LDS-DMA from per-lane addresses (wave 1).  A slot past
// the tile, or a tile past the end, reads entry 0 (row 0, node 0): the DMA
// counts stay fixed.
template <int NT, int D, int RPW>
struct TileIdx {
    const int32_t* in_row;
    const int32_t* out_row;
    const int32_t* nbr;
    const float* biases;
    int32_t* idxb;                  // [3][3][64]: in_row, out_row, nbr per slot
    uint32_t idx_lds, bias_lds;     // bias: [2][2][64] b(+1) then b(-1) per lane
    int64_t n, ntiles;
    int wave, lane;
    __device__ int tile_nl(int64_t t) const {
        if (t >= ntiles) return 0;
        const int64_t a0 = t * NT;
        return (int)((n - a0) < NT ? (n - a0) : NT) * D;
    }
    __device__ void dma_idx(int64_t t, int s3) const {             // wave 0: 3
        const int nl = tile_nl(t);
        const int64_t e = lane < nl ? t * NT * D + lane : 0;
        const uint32_t base = idx_lds + (uint32_t)(s3 * 192 * sizeof(int32_t));
        glds4(reinterpret_cast<const float*>(in_row + e), base);
        glds4(reinterpret_cast<const float*>(out_row + e), base + 64 * sizeof(int32_t));
        glds4(reinterpret_cast<const float*>(nbr + e), base + 128 * sizeof(int32_t));
    }
    __device__ void rows_of(int s3, int which, int32_t (&r)[RPW]) const {
        const int32_t* src = idxb + s3 * 192 + which * 64 + wave * RPW;
#pragma unroll
        for (int k = 0; k < RPW; ++k) r[k] = src[k];
    }
    __device__ void dma_bias(int s3, int s) const {                // wave 1: 2
        const int32_t nb = idxb[s3 * 192 + 128 + lane];
        const float* src = biases + 2 * (int64_t)nb;
        glds4(src, bias_lds + (uint32_t)((s * 128) * sizeof(float)));
        glds4(src + 1, bias_lds + (uint32_t)((s * 128 + 64) * sizeof(float)));
    }
    __device__ int32_t orow(int s3) const { return idxb[s3 * 192 + 64 + lane]; }
};

template <int T, int P, int D>
__device__ __forceinline__ void hpr_update_pipe(const float* __restrict__ chi_in, float* __restrict__ chi_out,
                                                const float* __restrict__ biases, const int32_t* __restrict__ nbr,
                                                const int32_t* __restrict__ in_row,
                                                const int32_t* __restrict__ out_row, int64_t n, int attr_plus,
                                                float w_plus, float w_minus, float damp) {
    using PC = PipeCfg<T, P, D>;
    constexpr int X = 1 << T, NC = X * X, NT = PC::NT, NL = PC::NL, NW = PC::NW, RPW = PC::RPW;
    static_assert(NC == 256 && RPW == 8 && NL <= 64, "pipelined HPR update: 1 KB rows (T = 4, fp32), 64-lane tiles");
    static_assert(Cfg<float, T, P, D>::NVALID == NW, "one valid x_a per wave");
    extern __shared__ __align__(16) unsigned char smem[];
    float* rows = reinterpret_cast<float*>(smem);                 // [2][64][PIPE_HRS] valid halves
    float* oldb = rows + 2 * PC::BUF;                             // [64][PIPE_ORS] old rows
    float* bias = oldb + PC::OLD;                                 // [2][2][64]
    int32_t* idxb = reinterpret_cast<int32_t*>(bias + 2 * 128);   // [3][3][64]
    float* red = reinterpret_cast<float*>(idxb + 3 * 192);        // [NW][64]
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int64_t ntiles = (n + NT - 1) / NT;
    const uint32_t rows_lds = (uint32_t)(uintptr_t)rows;
    const uint32_t old_lds = (uint32_t)(uintptr_t)oldb;
    const TileIdx<NT, D, RPW> ti{in_row, out_row, nbr, biases, idxb, (uint32_t)(uintptr_t)idxb,
                                 (uint32_t)(uintptr_t)bias, n, ntiles, wave, lane};
    const float keep = 1.0f - damp;
    const int q = wave;                                           // valid x_a index
    const int cv = (attr_plus ? 2 * q : 2 * q + 1) * X;           // valid block of every row
    const int ci = (attr_plus ? 2 * q + 1 : 2 * q) * X;           // x_a[T-1] != attr: chi_new = 0
    // column of half-row element h = x_k * 8 + (x_a >> 1)
    const int hcol0 = (lane >> 3) * X + 2 * (lane & 7) + (attr_plus ? 0 : 1);

    auto dma_in = [&](const int32_t (&ri)[RPW], int b) {           // valid halves -> buffer b: 2 * RPW
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int slot = wave * RPW + k;
            const uint32_t dst = rows_lds + (uint32_t)((b * PC::BUF + (size_t)slot * PIPE_HRS) * sizeof(float));
            const float* src = chi_in + (int64_t)ri[k] * NC + hcol0;
            glds4(src, dst);                                   // x_k 0..7
            glds4(src + 8 * X, dst + 64 * sizeof(float));     // x_k 8..15
        }
    };
    auto dma_old = [&](const int32_t (&ro)[RPW]) {                // whole old rows: RPW
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int slot = wave * RPW + k;
            glds16(chi_in + (int64_t)ro[k] * NC + lane * 4,
                   old_lds + (uint32_t)((size_t)slot * PIPE_ORS * sizeof(float)));
        }
    };

    int64_t t = blockIdx.x;
    if (t >= ntiles) return;
    const int64_t G = gridDim.x;
    int32_t r[RPW];
    // ---- prologue: the indices of tiles t and t+G, tile t's rows and biases
    if (wave == 0) {
        ti.dma_idx(t, 0);
        ti.dma_idx(t + G, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    ti.rows_of(0, 0, r);
    dma_in(r, 0);
    if (wave == 1) ti.dma_bias(0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    for (int it = 0; t < ntiles; ++it, t += G) {
        const int b = it & 1, s3 = it % 3, s3n = (it + 1) % 3;
        const int nl = ti.tile_nl(t);
        const bool active = lane < nl;
        // ---- stage 1 (all DMA): next tile's valid halves, indices and biases,
        // this tile's old rows
        ti.rows_of(s3n, 0, r);
        dma_in(r, 1 - b);
        if (wave == 0) ti.dma_idx(t + 2 * G, (it + 2) % 3);
        if (wave == 1) ti.dma_bias(s3n, 1 - b);
        ti.rows_of(s3, 1, r);
        dma_old(r);
        // ---- stage 2: compute from buffer b
        const float* rb = rows + b * PC::BUF;
        const float* bb = bias + b * 128;
        float out[X];
        float rs = 0.f;
        if (active) {
            static_for<0, NW>([&](auto ww) {
                constexpr int wv = decltype(ww)::value;
                if (wave == wv) {
                    constexpr int XP = 2 * wv, XM = 2 * wv + 1;
                    const float wgt0 = (XP < X / 2) ? w_plus : w_minus;
                    if (attr_plus) rs = xa_messages<float, T, P, D, XP, PIPE_HRS, true, false, 64>(
                                         rb, bb, a_local_of<D>(lane), lane % D, wgt0, out);
                    else rs = xa_messages<float, T, P, D, XM, PIPE_HRS, true, false, 64>(
                                   rb, bb, a_local_of<D>(lane), lane % D, wgt0, out);
                }
            });
        }
        red[wave * 64 + lane] = rs;
        // every DMA of this wave landed (next halves, indices, biases, old rows)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // ---- stage 3: normalise, damp, store (code/HPR_pytorch_RRG.py:215)
        if (active) {
            float tot = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) tot += red[w * 64 + lane];
            const float inv = 1.0f / tot;
            const float* ol = oldb + lane * PIPE_ORS;
            float* dst = chi_out + (int64_t)ti.orow(s3) * NC;
#pragma unroll
            for (int k = 0; k < X / 4; ++k) {
                const float4 ov = *reinterpret_cast<const float4*>(ol + cv + 4 * k);
                const float4 oi = *reinterpret_cast<const float4*>(ol + ci + 4 * k);
                float4 v, z;
                v.x = damp * (out[4 * k] * inv) + keep * ov.x;
                v.y = damp * (out[4 * k + 1] * inv) + keep * ov.y;
                v.z = damp * (out[4 * k + 2] * inv) + keep * ov.z;
                v.w = damp * (out[4 * k + 3] * inv) + keep * ov.w;
                z.x = keep * oi.x;
                z.y = keep * oi.y;
                z.z = keep * oi.z;
                z.w = keep * oi.w;
                *reinterpret_cast<float4*>(dst + cv + 4 * k) = v;
                *reinterpret_cast<float4*>(dst + ci + 4 * k) = z;
            }
        }
        // old-row buffer and buffer b free
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
}

template <int T, int P, int D>
__global__ void __launch_bounds__(512) k_hpr_update_pipe(const float* __restrict__ chi_in, float* __restrict__ chi_out,
                                                          const float* __restrict__ biases,
                                                          const int32_t* __restrict__ nbr,
                                                          const int32_t* __restrict__ in_row,
                                                          const int32_t* __restrict__ out_row, int64_t n,
                                                          int attr_plus, float w_plus, float w_minus, float damp) {
    hpr_update_pipe<T, P, D>(chi_in, chi_out, biases, nbr, in_row, out_row, n, attr_plus, w_plus, w_minus, damp);
}

// Which valid x_a each wave of the 8-wave update takes.  A wave's DP costs a
// fixed convolution plus one FMA per non-empty corner (x, x_b) of its x_a,
// and the corner counts differ by up to 3x between x_a (d=4, p=c=2, attr +1:
// 256, 108, 144, 108, 192, 81, 192, 144).  Waves w and w+4 share a SIMD, so
// x_a is dealt heaviest-with-lightest: wave s the s-th heaviest, wave s+4 the
// s-th lightest (measured per-wave DP at C3 before: 4.4k/5.5k cycles on SIMD 0
// against 2.5k/3.0k on SIMD 1).
template <int T, int P, int D, int XA>
constexpr int xa_corners() {
    int c = 0;
    for (int x = 0; x < (1 << T); ++x)
        for (int xb = 0; xb < (1 << T); ++xb) c += Tabs<T, P, D, XA>::v.cn[x][xb] >= 0 ? 1 : 0;
    return c;
}
template <int T, int P, int D, int PV>
struct XaDeal {
    static constexpr int NW = 8;
    struct M { int q[NW]; };
    template <int... Q>
    static constexpr M make(std::integer_sequence<int, Q...>) {
        const int cost[NW] = {xa_corners<T, P, D, 2 * Q + PV>()...};
        int ord[NW] = {0, 1, 2, 3, 4, 5, 6, 7};
        for (int i = 0; i < NW; ++i)                         // by cost, heaviest first (stable)
            for (int j = i + 1; j < NW; ++j)
                if (cost[ord[j]] > cost[ord[i]]) { const int tmp = ord[i]; ord[i] = ord[j]; ord[j] = tmp; }
        M m{};
        for (int s = 0; s < NW / 2; ++s) {
            m.q[s] = ord[s];
            m.q[s + NW / 2] = ord[NW - 1 - s];
        }
        return m;
    }
    static constexpr M v = make(std::make_integer_sequence<int, NW>{});
};

constexpr int PIPE_QORS = 132;      // old half-row stride (floats): 528 B, 16-B aligned DMA bases

// The decay-split update with the epilogue of tile t-G run beside the DP of
// tile t (round 6).  Round 5's form (hpr_update_q2, in git history) separated
// the two by a barrier (the row sums of every wave), so per tile it ran DP ->
// barrier -> normalise, damp, store -> barrier.  Here the outputs of the previous tile wait in registers
// (16 floats a lane) and its row sums in a second `red` slot, and iteration i
// issues tile i+1's reads, computes tile i's DP, normalises / damps / stores
// tile i-1 and meets ONE barrier: the epilogue's arithmetic and stores
// interleave with the DP of the next tile instead of standing between two
// barriers.  Buffers: incoming halves and biases by tile parity (read by the
// DP of tile i, written for tile i+1), old half rows by tile parity (written
// for tile i, read by the epilogue of tile i one iteration later), the index
// rows in four slots (tiles i-1 .. i+2 live), row sums in two.
template <int T, int P, int D>
struct PipeQ3Cfg {
    using C = Cfg<float, T, P, D>;
    static constexpr int NW = 8, NL = C::NL, NT = C::NT;
    static constexpr int RPW = (NL + NW - 1) / NW;
    static constexpr size_t IN = (size_t)64 * PIPE_HRS;         // floats per incoming slot
    static constexpr size_t OLD = (size_t)64 * PIPE_QORS;       // floats per old-row slot
    static constexpr size_t LDS = (2 * IN + 2 * OLD + 2 * 128 + 4 * 192 + 2 * (size_t)NW * 64) * sizeof(float);
    static constexpr int N_A = 2 * RPW + RPW;                   // DMA per wave in A (+3 on wave 0, +2 on wave 1)
    static constexpr int N_E = 4;                               // 16-B stores per lane in the epilogue
};

template <int T, int P, int D>
__device__ __forceinline__ void hpr_update_q3(const float* __restrict__ chi_in, float* __restrict__ chi_out,
                                              const float* __restrict__ biases, const int32_t* __restrict__ nbr,
                                              const int32_t* __restrict__ in_row, const int32_t* __restrict__ out_row,
                                              int64_t n, int attr_plus, float w_plus, float w_minus, float damp,
                                              float sc) {
    using PC = PipeQ3Cfg<T, P, D>;
    constexpr int X = 1 << T, NC = X * X, H = X / 2, NT = PC::NT, NL = PC::NL, NW = PC::NW, RPW = PC::RPW;
    static_assert(NC == 256 && RPW == 8 && NL <= 64, "decay-split update: 1 KB rows (T = 4, fp32), 64-lane tiles");
    static_assert(Cfg<float, T, P, D>::NVALID == NW, "one valid x_a per wave");
    static_assert(2 * (H / 4) == PC::N_E, "epilogue stores per lane");
    extern __shared__ __align__(16) unsigned char smem[];
    float* inb = reinterpret_cast<float*>(smem);                  // [2][64][PIPE_HRS] VV | IV halves
    float* oldb = inb + 2 * PC::IN;                               // [2][64][PIPE_QORS] first half rows
    float* biasb = oldb + 2 * PC::OLD;                            // [2][2][64]: b(+1) then b(-1) per lane
    int32_t* idxb = reinterpret_cast<int32_t*>(biasb + 2 * 128);  // [4][3][64]: in_row, out_row, nbr per slot
    float* red = reinterpret_cast<float*>(idxb + 4 * 192);        // [2][NW][64]
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int64_t ntiles = (n + NT - 1) / NT;
    const uint32_t in_lds = (uint32_t)(uintptr_t)inb, old_lds = (uint32_t)(uintptr_t)oldb;
    const TileIdx<NT, D, RPW> ti{in_row, out_row, nbr, biases, idxb, (uint32_t)(uintptr_t)idxb,
                                 (uint32_t)(uintptr_t)biasb, n, ntiles, wave, lane};
    const float keep = 1.0f - damp;
    // valid x_a index of this wave (dealt by DP cost, see XaDeal)
    const int q = attr_plus ? XaDeal<T, P, D, 0>::v.q[wave] : XaDeal<T, P, D, 1>::v.q[wave];

    auto dma_in = [&](const int32_t (&r)[RPW], int s) {           // 2 * RPW
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int slot = wave * RPW + k;
            const uint32_t dst = in_lds + (uint32_t)((s * PC::IN + (size_t)slot * PIPE_HRS) * sizeof(float));
            const float* src = chi_in + (int64_t)r[k] * NC + lane;
            glds4(src, dst);
            glds4(src + NC / 2, dst + 64 * sizeof(float));
        }
    };
    auto dma_old = [&](const int32_t (&r)[RPW], int s) {          // RPW (lanes 0..31: 512 B)
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int slot = wave * RPW + k;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(
                old_lds + (uint32_t)((s * PC::OLD + (size_t)slot * PIPE_QORS) * sizeof(float)));
            if (lane < 32) glds16(chi_in + (int64_t)r[k] * NC + lane * 4, dst);
        }
    };

    int64_t t = blockIdx.x;
    if (t >= ntiles) return;
    const int64_t G = gridDim.x;
    int32_t r[RPW];
    // ---- prologue: indices of tiles t and t+G; tile t's incoming rows and biases
    if (wave == 0) {
        ti.dma_idx(t, 0);
        ti.dma_idx(t + G, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    ti.rows_of(0, 0, r);
    dma_in(r, 0);
    if (wave == 1) ti.dma_bias(0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    float outp[X];                 // the previous tile's outputs (this wave's x_a), kept for its epilogue
#pragma unroll
    for (int x = 0; x < X; ++x) outp[x] = 0.f;
    int64_t tp = -1;               // the previous tile (-1: none)
    for (int it = 0;; ++it, t += G) {
        const bool cur = t < ntiles;                              // (block-uniform)
        if (!cur && tp < 0) break;
        const int b = it & 1, s4 = it & 3, s4n = (it + 1) & 3, s4p = (it + 3) & 3;
        float out[X];
        if (cur) {
            // ---- A: tile t+G's incoming halves and biases, tile t+2G's indices,
            // tile t's old half rows (read by its epilogue, next iteration)
            ti.rows_of(s4n, 0, r);
            dma_in(r, 1 - b);
            if (wave == 0) ti.dma_idx(t + 2 * G, (it + 2) & 3);
            if (wave == 1) ti.dma_bias(s4n, 1 - b);
            ti.rows_of(s4, 1, r);
            dma_old(r, b);
            // ---- B: DP of tile t
            const float* rb = inb + b * PC::IN;
            const float* bb = biasb + b * 128;
            float rs = 0.f;
#pragma unroll
            for (int x = 0; x < X; ++x) out[x] = 0.f;
            if (lane < ti.tile_nl(t)) {
                static_for<0, NW>([&](auto ww) {
                    constexpr int wv = decltype(ww)::value;
                    if (wave == wv) {
                        constexpr int XP = 2 * XaDeal<T, P, D, 0>::v.q[wv], XM = 2 * XaDeal<T, P, D, 1>::v.q[wv] + 1;
                        if (attr_plus) rs = xa_messages<float, T, P, D, XP, PIPE_HRS, true, true, 64>(
                                             rb, bb, a_local_of<D>(lane), lane % D, (XP < X / 2) ? w_plus : w_minus,
                                             out, sc);
                        else rs = xa_messages<float, T, P, D, XM, PIPE_HRS, true, true, 64>(
                                       rb, bb, a_local_of<D>(lane), lane % D, (XM < X / 2) ? w_plus : w_minus, out,
                                       sc);
                    }
                });
            }
            red[b * NW * 64 + wave * 64 + lane] = rs;
        }
        // ---- E: normalise, damp (code/HPR_pytorch_RRG.py:215) and store the
        // previous tile's first half rows: sums in red[1-b], old rows in oldb[1-b]
        if (tp >= 0) {
            if (lane < ti.tile_nl(tp)) {
                float tot = 0.f;
#pragma unroll
                for (int w = 0; w < NW; ++w) tot += red[(1 - b) * NW * 64 + w * 64 + lane];
                const float inv = 1.0f / tot;
                const float* ol = oldb + (1 - b) * PC::OLD + lane * PIPE_QORS;
                float* dst = chi_out + (int64_t)ti.orow(s4p) * NC;
                // entries (x_a = this wave's valid sender, x_b): VV at q*H + (x_b>>1) for
                // valid x_b, VI at H*H + q*H + (x_b>>1) for the others
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int base = half * H * H + q * H;
#pragma unroll
                    for (int k = 0; k < H / 4; ++k) {
                        const float4 ov = *reinterpret_cast<const float4*>(ol + base + 4 * k);
                        float o[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int j = 4 * k + e;                        // x_b >> 1
                            const bool odd = (half == 0) != (attr_plus != 0);
                            o[e] = odd ? outp[2 * j + 1] : outp[2 * j];
                        }
                        float4 rr;
                        rr.x = damp * (o[0] * inv) + keep * ov.x;
                        rr.y = damp * (o[1] * inv) + keep * ov.y;
                        rr.z = damp * (o[2] * inv) + keep * ov.z;
                        rr.w = damp * (o[3] * inv) + keep * ov.w;
                        *reinterpret_cast<float4*>(dst + base + 4 * k) = rr;
                    }
                }
            }
        }
        // every read of A landed (the epilogue's stores, issued after them, may fly);
        // LDS reads of B and E done before the buffers turn over
        if (cur && tp >= 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(PC::N_E) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (!cur) break;
#pragma unroll
        for (int x = 0; x < X; ++x) outp[x] = out[x];
        tp = t;
    }
}

// the decay-split layout; scale_in = decay of chi_in's IV quadrants
template <int T, int P, int D>
__global__ void __launch_bounds__(512) k_hpr_update_q3(const float* __restrict__ chi_in, float* __restrict__ chi_out,
                                                        const float* __restrict__ biases,
                                                        const int32_t* __restrict__ nbr,
                                                        const int32_t* __restrict__ in_row,
                                                        const int32_t* __restrict__ out_row, int64_t n, int attr_plus,
                                                        float w_plus, float w_minus, float damp,
                                                        const float* __restrict__ scale_in) {
    hpr_update_q3<T, P, D>(chi_in, chi_out, biases, nbr, in_row, out_row, n, attr_plus, w_plus, w_minus, damp,
                           *scale_in);
}

// ---- marginals (code/HPR_pytorch_RRG.py:147-167) ---------------------------
// Z sums of chi^{u->v}(x_u,x_v) chi^{v->u}(x_v,x_u) by x_u[0] (row r) and by
// x_v[0] (row r+E), clamped at eps, normalised.  A group of G = X lanes per
// undirected edge: lane l reads 16-B pieces l, l+G, ... of row r (a group
// instruction reads 16*G contiguous bytes) and, for each element, the
// transposed element of row r+E by scalar loads (at T=4 fp32 a group
// instruction reads 4 whole 64-B lines); the sums need log2(G) shuffle steps.  U edge groups per lane are in flight at once (the kernel is
// a stream over chi).
template <typename S, int T>
__global__ void __launch_bounds__(256) k_hpr_edge_z(const S* __restrict__ chi, int64_t E, S eps,
                                                     S* __restrict__ zp, S* __restrict__ zm) {
    constexpr int X = 1 << T, NC = X * X;
    using V = typename Vec16<S>::T;
    constexpr int VN = Vec16<S>::N;
    constexpr int G = X < 64 ? X : 64;               // lanes per edge
    constexpr int NV = NC / (VN * G);                // 16-B pieces per lane per row
    constexpr int EPW = 64 / G;                      // edges per wave instruction
    constexpr int U = 2;                             // edge groups in flight per lane
    const int lane = threadIdx.x & 63;
    const int g = lane / G, l = lane % G;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * 256) >> 6;
    for (int64_t base = wave * EPW * U; base < E; base += nwaves * EPW * U) {
        S f[U][NV][VN], b[U][NV][VN];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = base + u * EPW + g;
            const int64_t rr = r < E ? r : E - 1;            // branch-free loads
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int j0 = (v * G + l) * VN;
                const V x = *reinterpret_cast<const V*>(chi + rr * NC + j0);
                const S* xs = reinterpret_cast<const S*>(&x);
#pragma unroll
                for (int e = 0; e < VN; ++e) {
                    f[u][v][e] = xs[e];
                    const int xu = (j0 + e) / X, xv = (j0 + e) % X;
                    b[u][v][e] = chi[(rr + E) * NC + xv * X + xu];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = base + u * EPW + g;
            S sp = 0, sm = 0, bp = 0, bm = 0;            // by x_u[0], by x_v[0]
#pragma unroll
            for (int v = 0; v < NV; ++v)
#pragma unroll
                for (int e = 0; e < VN; ++e) {
                    const int j = (v * G + l) * VN + e;
                    const int xu = j / X, xv = j % X;
                    const S z = f[u][v][e] * b[u][v][e];
                    if (xu < X / 2) sp += z; else sm += z;
                    if (xv < X / 2) bp += z; else bm += z;
                }
#pragma unroll
            for (int off = G / 2; off > 0; off >>= 1) {
                sp += __shfl_xor(sp, off, 64);
                sm += __shfl_xor(sm, off, 64);
                bp += __shfl_xor(bp, off, 64);
                bm += __shfl_xor(bm, off, 64);
            }
            if (l == 0 && r < E) {
                S fp = sp > eps ? sp : eps, fm = sm > eps ? sm : eps;
                bp = bp > eps ? bp : eps; bm = bm > eps ? bm : eps;
                const S sf = fp + fm, sb = bp + bm;
                zp[r] = fp / sf; zm[r] = fm / sf;
                zp[r + E] = bp / sb; zm[r + E] = bm / sb;
            }
        }
    }
}

// the same Z sums over rows in the decay-split layout: entry j of row r is
// (x_u, x_v) = (sender, receiver) of quadrant j / H^2, its transposed partner
// in row r+E sits in the quadrant with the two validity bits swapped, and a
// product carries scale^(number of invalid senders) (IV / II entries are
// stored undecayed).  Z+ by x_u[0] = +1 <=> (x_u >> 1) < H/2.
// IIP: the II x II products never change (both factors stay chi_0), so their
// four sums per edge come precomputed (ii[4e..4e+3] = by x_u[0] +/-, by x_v[0]
// +/-, k_hpr_q_ii) and the II pieces of both rows are not read: 1.5 instead of
// 2 KB per edge at T = 4 fp32.  Needs whole 16-B pieces per quadrant
// (q_ii_aligned).
template <typename S, int T>
struct QZ {
    static constexpr int X = 1 << T, H = X / 2, HH = H * H;
    static constexpr int VN = Vec16<S>::N, G = X < 64 ? X : 64;
    static constexpr bool ALIGNED = HH % (G * VN) == 0;
};

template <typename S, int T, bool IIP = false>
__global__ void __launch_bounds__(256) k_hpr_edge_z_q(const S* __restrict__ chi, int64_t E, S eps,
                                                       const S* __restrict__ scale, S* __restrict__ zp,
                                                       S* __restrict__ zm, const S* __restrict__ ii = nullptr) {
    constexpr int X = 1 << T, NC = X * X, H = X / 2, HH = H * H;
    using V = typename Vec16<S>::T;
    constexpr int VN = Vec16<S>::N;
    constexpr int G = X < 64 ? X : 64;               // lanes per edge
    constexpr int NV = NC / (VN * G);                // 16-B pieces per lane per row
    constexpr int EPW = 64 / G;                      // edges per wave instruction
    constexpr int U = 2;                             // edge groups in flight per lane
    static_assert(!IIP || QZ<S, T>::ALIGNED, "II skip needs whole pieces per quadrant");
    // piece v lies in quadrant v * G * VN / HH (when aligned); II = 3
    constexpr int NVR = IIP ? NV - NV / 4 : NV;       // pieces read per row
    const S s1 = *scale, s2 = s1 * s1;
    const int lane = threadIdx.x & 63;
    const int g = lane / G, l = lane % G;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * 256) >> 6;
    for (int64_t base = wave * EPW * U; base < E; base += nwaves * EPW * U) {
        S f[U][NV][VN], b[U][NV][VN];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = base + u * EPW + g;
            const int64_t rr = r < E ? r : E - 1;            // branch-free loads
#pragma unroll
            for (int v = 0; v < NVR; ++v) {
                const int j0 = (v * G + l) * VN;
                const V x = *reinterpret_cast<const V*>(chi + rr * NC + j0);
                const S* xs = reinterpret_cast<const S*>(&x);
#pragma unroll
                for (int e = 0; e < VN; ++e) {
                    const int j = j0 + e, q = j / HH, w = j % HH;
                    const int jt = (((q & 1) << 1) | (q >> 1)) * HH + (w % H) * H + w / H;
                    f[u][v][e] = xs[e];
                    b[u][v][e] = chi[(rr + E) * NC + jt];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = base + u * EPW + g;
            S sp = 0, sm = 0, bp = 0, bm = 0;            // by x_u[0], by x_v[0]
#pragma unroll
            for (int v = 0; v < NVR; ++v)
#pragma unroll
                for (int e = 0; e < VN; ++e) {
                    const int j = (v * G + l) * VN + e, q = j / HH, w = j % HH;
                    const S fac = q == 0 ? S(1) : (q == 3 ? s2 : s1);
                    const S z = fac * (f[u][v][e] * b[u][v][e]);
                    if (w / H < H / 2) sp += z; else sm += z;
                    if (w % H < H / 2) bp += z; else bm += z;
                }
#pragma unroll
            for (int off = G / 2; off > 0; off >>= 1) {
                sp += __shfl_xor(sp, off, 64);
                sm += __shfl_xor(sm, off, 64);
                bp += __shfl_xor(bp, off, 64);
                bm += __shfl_xor(bm, off, 64);
            }
            if (l == 0 && r < E) {
                if (IIP) {
                    sp += s2 * ii[4 * r]; sm += s2 * ii[4 * r + 1];
                    bp += s2 * ii[4 * r + 2]; bm += s2 * ii[4 * r + 3];
                }
                S fp = sp > eps ? sp : eps, fm = sm > eps ? sm : eps;
                bp = bp > eps ? bp : eps; bm = bm > eps ? bm : eps;
                const S sf = fp + fm, sb = bp + bm;
                zp[r] = fp / sf; zm[r] = fm / sf;
                zp[r + E] = bp / sb; zm[r + E] = bm / sb;
            }
        }
    }
}

// the four II x II sums of every edge of a decay-split chi (its chi_0 quadrants)
template <typename S, int T>
__global__ void k_hpr_q_ii(const S* __restrict__ chi, int64_t E, S* __restrict__ ii) {
    constexpr int X = 1 << T, NC = X * X, H = X / 2, HH = H * H;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < E; r += (int64_t)gridDim.x * blockDim.x) {
        S sp = 0, sm = 0, bp = 0, bm = 0;
        for (int w = 0; w < HH; ++w) {
            const S z = chi[r * NC + 3 * HH + w] * chi[(r + E) * NC + 3 * HH + (w % H) * H + w / H];
            if (w / H < H / 2) sp += z; else sm += z;
            if (w % H < H / 2) bp += z; else bm += z;
        }
        ii[4 * r] = sp; ii[4 * r + 1] = sm; ii[4 * r + 2] = bp; ii[4 * r + 3] = bm;
    }
}

// reference layout <-> decay-split layout (to_q: dst = permuted src; else dst =
// src un-permuted with the sender-invalid entries scaled)
template <typename S>
__global__ void k_hpr_qperm(const S* __restrict__ src, S* __restrict__ dst, int64_t rows, int T, int pv, int to_q,
                            S scale) {
    const int X = 1 << T, NC = X * X;
    const int64_t total = rows * NC;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / NC;
        const int col = (int)(i - r * NC), xs = col / X, xr = col % X;
        const int64_t qi = r * NC + qpos(xs, xr, T, pv);
        if (to_q) dst[qi] = src[i];
        else dst[i] = ((xs & 1) != pv) ? src[qi] * scale : src[qi];
    }
}

template <typename S>
__global__ void __launch_bounds__(256) k_hpr_node_marg(const S* __restrict__ zp, const S* __restrict__ zm,
                                                        const int32_t* __restrict__ out_row, int64_t n, int d,
                                                        S* __restrict__ marg) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    S p = 1, q = 1;
    for (int m = 0; m < d; ++m) {
        const int64_t r = out_row[i * d + m];
        p *= zp[r];
        q *= zm[r];
    }
    const S s = p + q;
    marg[2 * i] = p / s;
    marg[2 * i + 1] = q / s;
}

// new_biases_i (code/HPR_pytorch_RRG.py:137-145) with caller-supplied uniforms
template <typename S>
__global__ void __launch_bounds__(256) k_hpr_new_biases(S* __restrict__ biases, const S* __restrict__ marg,
                                                         const double* __restrict__ u, double thresh, S pie,
                                                         int64_t n, int32_t* __restrict__ s) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    S b0 = biases[2 * i], b1 = biases[2 * i + 1];
    if (u[i] < thresh) {
        const bool minus = marg[2 * i + 1] >= marg[2 * i];
        b0 = minus ? pie : S(1) - pie;
        b1 = minus ? S(1) - pie : pie;
        biases[2 * i] = b0;
        biases[2 * i + 1] = b1;
    }
    if (s) s[i] = b0 > b1 ? 1 : -1;
}

// the same with the refresh decision made on the host (refresh[i] = u_i <
// 1-(1+t)^-gamma, :142): one byte per node crosses the bus instead of a double
template <typename S>
__global__ void __launch_bounds__(256) k_hpr_new_biases_mask(S* __restrict__ biases, const S* __restrict__ marg,
                                                              const uint8_t* __restrict__ refresh, S pie, int64_t n,
                                                              int32_t* __restrict__ s) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    S b0 = biases[2 * i], b1 = biases[2 * i + 1];
    if (refresh[i]) {
        const bool minus = marg[2 * i + 1] >= marg[2 * i];
        b0 = minus ? pie : S(1) - pie;
        b1 = minus ? S(1) - pie : pie;
        biases[2 * i] = b0;
        biases[2 * i + 1] = b1;
    }
    if (s) s[i] = b0 > b1 ? 1 : -1;
}

// One node step of the main loop (code/HPR_pytorch_RRG.py:147-167 node part,
// 137-145, and the packing of s for s_endstate at :352): the node marginal from
// the edge Z sums (as k_hpr_node_marg), the bias refresh with the host- or
// device-made decision (as k_hpr_new_biases_mask), the trial configuration s,
// and s bit-packed for the rollout (bit = 1 <=> s = +1, one ballot per 64
// nodes) -- three launches of the loop in one.
template <typename S>
__global__ void __launch_bounds__(256) k_hpr_node_step(const S* __restrict__ zp, const S* __restrict__ zm,
                                                        const int32_t* __restrict__ out_row, int64_t n, int d,
                                                        S* __restrict__ marg, S* __restrict__ biases,
                                                        const uint8_t* __restrict__ refresh, S pie,
                                                        int32_t* __restrict__ s, u64* __restrict__ bits) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool plus = false;
    if (i < n) {
        S p = 1, q = 1;
        for (int m = 0; m < d; ++m) {
            const int64_t r = out_row[i * d + m];
            p *= zp[r];
            q *= zm[r];
        }
        const S sum = p + q;
        const S m0 = p / sum, m1 = q / sum;
        marg[2 * i] = m0;
        marg[2 * i + 1] = m1;
        S b0 = biases[2 * i], b1 = biases[2 * i + 1];
        if (refresh[i]) {
            const bool minus = m1 >= m0;
            b0 = minus ? pie : S(1) - pie;
            b1 = minus ? S(1) - pie : pie;
            biases[2 * i] = b0;
            biases[2 * i + 1] = b1;
        }
        plus = b0 > b1;
        s[i] = plus ? 1 : -1;
    }
    const u64 w = __ballot(plus);
    if ((threadIdx.x & 63) == 0 && i < n) bits[i >> 6] = w;
}

// ---- dispatch --------------------------------------------------------------
template <typename S, int T, int P, int D>
static int launch_update(const void* chi_in, void* chi_out, const void* biases, const int32_t* nbr,
                         const int32_t* in_row, const int32_t* out_row, int64_t n, int attr_plus, double w_plus,
                         double w_minus, double damp, hipStream_t st) {
    using C = Cfg<S, T, P, D>;
    if constexpr (C::NS > 128 || C::LDS > 160 * 1024) {
        return MJX_ERANGE;
    } else {
        const int64_t tiles = (n + C::NT - 1) / C::NT;
        if (tiles > INT32_MAX) return MJX_ERANGE;
        if constexpr (std::is_same<S, float>::value && T == 4) {
            // 1 KB rows: the software-pipelined persistent form
            {
                using PC = PipeCfg<T, P, D>;
                auto pk = k_hpr_update_pipe<T, P, D>;
                MJX_HIP(set_max_lds(pk, (int)PC::LDS), "hpr pipe set lds");
                const int per = resident_blocks_per_cu((const void*)pk, 512, PC::LDS);
                int64_t grid = (int64_t)device_cus() * (per > 0 ? per : 1);
                if (grid > tiles) grid = tiles;
                pk<<<(unsigned)grid, 512, PC::LDS, st>>>((const float*)chi_in, (float*)chi_out, (const float*)biases,
                                                         nbr, in_row, out_row, n, attr_plus, (float)w_plus,
                                                         (float)w_minus, (float)damp);
                MJX_LAUNCH_CHECK("k_hpr_update_pipe");
                return MJX_OK;
            }
        }
        auto kern = k_hpr_update<S, T, P, D>;
        MJX_HIP(set_max_lds(kern, (int)C::LDS), "hpr set lds");   // opt in to > 64 KiB dynamic LDS
        kern<<<(unsigned)tiles, 64 * C::NW, C::LDS, st>>>((const S*)chi_in, (S*)chi_out, (const S*)biases, nbr,
                                                          in_row, out_row, n, attr_plus, (S)w_plus, (S)w_minus,
                                                          (S)damp);
        MJX_LAUNCH_CHECK("k_hpr_update");
        return MJX_OK;
    }
}

// the decay-split update (fp32, T = 4, register table: d <= 4)
template <int T, int P, int D>
static int launch_update_q(const void* chi_in, void* chi_out, const void* biases, const int32_t* nbr,
                           const int32_t* in_row, const int32_t* out_row, int64_t n, int attr_plus, double w_plus,
                           double w_minus, double damp, const float* scale_in, hipStream_t st) {
    using C = Cfg<float, T, P, D>;
    using PC = PipeCfg<T, P, D>;
    if constexpr (T != 4 || C::NS > 128 || PC::LDS > 160 * 1024) {
        return MJX_ERANGE;
    } else {
        const int64_t tiles = (n + C::NT - 1) / C::NT;
        if (tiles > INT32_MAX) return MJX_ERANGE;
        using PQ = PipeQ3Cfg<T, P, D>;
        auto pk = k_hpr_update_q3<T, P, D>;
        static_assert(PQ::LDS <= 160 * 1024, "decay-split update LDS");
        MJX_HIP(set_max_lds(pk, (int)PQ::LDS), "hpr update q set lds");
        const int per = resident_blocks_per_cu((const void*)pk, 512, PQ::LDS);
        int64_t grid = (int64_t)device_cus() * (per > 0 ? per : 1);
        if (grid > tiles) grid = tiles;
        pk<<<(unsigned)grid, 512, PQ::LDS, st>>>((const float*)chi_in, (float*)chi_out, (const float*)biases, nbr,
                                                 in_row, out_row, n, attr_plus, (float)w_plus, (float)w_minus,
                                                 (float)damp, scale_in);
        MJX_LAUNCH_CHECK("k_hpr_update_q");
        return MJX_OK;
    }
}

template <typename S, int T, int P>
static int dispatch_d(int d, const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir,
                      const int32_t* orr, int64_t n, int ap, double wp, double wm, double dp, hipStream_t st) {
    switch (d) {
        case 2: return launch_update<S, T, P, 2>(ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
        case 3: return launch_update<S, T, P, 3>(ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
        case 4: return launch_update<S, T, P, 4>(ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
        case 5: return launch_update<S, T, P, 5>(ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
        case 6: return launch_update<S, T, P, 6>(ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
        default: return MJX_ERANGE;
    }
}

template <typename S>
static int dispatch_tp(int p, int c, int d, const void* ci, void* co, const void* b, const int32_t* nb,
                       const int32_t* ir, const int32_t* orr, int64_t n, int ap, double wp, double wm, double dp,
                       hipStream_t st) {
    const int T = p + c;
#define MJX_TP(TT, PP) \
    if (T == TT && p == PP) return dispatch_d<S, TT, PP>(d, ci, co, b, nb, ir, orr, n, ap, wp, wm, dp, st);
    MJX_TP(2, 1) MJX_TP(3, 1) MJX_TP(3, 2) MJX_TP(4, 1) MJX_TP(4, 2) MJX_TP(4, 3)
#undef MJX_TP
    return MJX_ERANGE;
}

inline bool q_supported(int d, int p, int c) { return p >= 1 && c >= 1 && p + c == 4 && d >= 2 && d <= 4; }

// per-dtype instantiation units (mjx_hpr_f32.hip, mjx_hpr_f64.hip)
int update_q_f32(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
                 int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, const float* sc,
                 hipStream_t st);
int update_f32(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
               int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, hipStream_t st);
int update_f64(const void* ci, void* co, const void* b, const int32_t* nb, const int32_t* ir, const int32_t* orr,
               int64_t n, int d, int p, int c, int ap, double wp, double wm, double dp, hipStream_t st);

}  // namespace hpr
}  // namespace mjx
