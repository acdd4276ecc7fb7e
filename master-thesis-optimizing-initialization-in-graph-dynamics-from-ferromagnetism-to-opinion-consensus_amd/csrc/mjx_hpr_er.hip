// History-passing reinforcement on Erdos-Renyi graphs (the "general (ER)"
// variant that code/README.md:1 announces and the repository does not ship).
//
// It is HPr_dp (code/HPR_pytorch_RRG.py:183-218) with the node degree taken
// per message instead of a global d: the message a -> b has deg(a) - 1 = D
// incoming messages k -> a, and
//   chi_new(x_a, x_b) = w(x_a[0]) [x_a[T-1] = attr] sum_{x_k1..x_kD} prod_m M_m(x_km, x_a)
//                        * prod_t allowed_t(2 rho_t - D + x_b[t])
//   M_m(x_k, x_a) = bias_{k_m}(x_k[0]) chi^{k_m -> a}(x_k, x_a)   (new_biases_chi, :128-133)
//   chi <- damp * chi_new / sum chi_new + (1 - damp) * chi          (:215, Jacobi: every
//                                                                    message from the old chi)
// with the reference's HPR layout: row r < E = G.edges[r] = (u, v) as u -> v,
// row r + E = v -> u; column idx(x_a) * 2^T + idx(x_b), idx bit (T-1-t) = 1 for
// spin -1 (order_gpu, :46-61); w = exp(-lmbd x_a[0] / n) (:39).  Messages are
// grouped by D (the BDCM degree classes, nb:312-318); on a d-regular graph
// every message is in class d-1 and this is exactly HPr_dp.
//
// Evaluation: one wave per message; the count table over rho in [0..D]^T for
// every valid x_a in LDS, convolved in place one incoming message at a time
// over ALL x_k (HPR sums every sender trajectory; BDCM only attractor-ending
// ones), then directional cumulative sums, so every output is one lookup
// (the same rearrangement as mjx_bdcm.hip and mjx_hpr_impl.h).
#include "mjx_common.h"
#include <math.h>

namespace mjx {
namespace hprer {

constexpr int kMaxT = 4;
constexpr size_t kMaxLds = 160 * 1024;

struct Geo {
    int T, P, D, X, XV, B, S, ab;     // ab: index bit 0 (x_a[T-1]) of the attractor spin
    int pw[kMaxT];                    // B^(T-1-t)
};

// HPR index convention: bit (T-1-t) = 1 means spin -1
__host__ __device__ inline int hspin(int x, int t, int T) { return ((x >> (T - 1 - t)) & 1) ? -1 : 1; }
__host__ __device__ inline int fdiv2(int a) { return a >= 0 ? a / 2 : -((-a + 1) / 2); }
__host__ __device__ inline int cdiv2(int a) { return -fdiv2(-a); }

static bool make_geo(int D, int p, int c, int attr_value, Geo* g) {
    const int T = p + c;
    if (p < 1 || c < 1 || T > kMaxT || D < 0 || D > 255) return false;
    if (attr_value != 1 && attr_value != -1) return false;
    g->T = T;
    g->P = p;
    g->D = D;
    g->X = 1 << T;
    g->XV = g->X / 2;
    g->B = D + 1;
    int64_t S = 1;
    for (int t = T - 1; t >= 0; --t) {
        g->pw[t] = (int)S;
        S *= g->B;
        if (S > (1 << 22)) return false;
    }
    for (int t = T; t < kMaxT; ++t) g->pw[t] = 0;
    g->S = (int)S;
    g->ab = attr_value > 0 ? 0 : 1;
    return true;
}

template <typename S_>
static size_t tab_bytes(const Geo& g) { return (size_t)g.XV * g.S * sizeof(S_); }
template <typename S_>
static size_t m_bytes(const Geo& g) { return (size_t)g.D * g.XV * g.X * sizeof(S_); }
template <typename S_>
static size_t lds_bytes(const Geo& g) { return tab_bytes<S_>(g) + m_bytes<S_>(g); }

// the spin the condition on time t must produce, and the spin a tie keeps
// (traj_condition for t < T-1, atr_condition for t = T-1; code/HPR_pytorch_RRG.py:14-29)
__device__ inline int cond_dir(const Geo& g, int xa, int t) {
    return (t < g.T - 1) ? hspin(xa, t + 1, g.T) : hspin(xa, g.P, g.T);
}
__device__ inline int cond_prev(const Geo& g, int xa, int t) {
    return (t < g.T - 1) ? hspin(xa, t, g.T) : hspin(xa, g.T - 1, g.T);
}

// corner of the rho box allowed for (x_a, x_b), -1 when empty;
// sigma_t = 2 rho_t - D + y_t (code/HPR_pytorch_RRG.py:212, rho -> 2 rho - (d-1))
__device__ inline int corner(const Geo& g, int xa, int xb) {
    int idx = 0;
    for (int t = 0; t < g.T; ++t) {
        const int s = cond_dir(g, xa, t), prev = cond_prev(g, xa, t);
        const int y = hspin(xb, t, g.T);
        int dg;
        if (s > 0) {            // sigma > 0, or sigma == 0 and prev == +1
            const int lo = cdiv2(g.D - y + (prev > 0 ? 0 : 1));
            if (lo > g.D) return -1;
            dg = lo < 0 ? 0 : lo;
        } else {                // sigma < 0, or sigma == 0 and prev == -1
            const int hi = fdiv2(g.D - y + (prev < 0 ? 0 : -1));
            if (hi < 0) return -1;
            dg = hi > g.D ? g.D : hi;
        }
        idx += dg * g.pw[t];
    }
    return idx;
}

__device__ inline int traj_off(const Geo& g, int x) {     // table offset of one +1 count per time
    int o = 0;
    for (int t = 0; t < g.T; ++t)
        if (hspin(x, t, g.T) > 0) o += g.pw[t];
    return o;
}

template <typename S_>
__device__ inline S_ wave_sum(S_ v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// one wave per message of class D (message e0 + blockIdx.x): new row into
// chi_out.  The count table lives in LDS, or, for classes whose table exceeds
// the LDS budget (high degree, long trajectories), in a global scratch slab
// (gtab, one table per workgroup of the launch; the incoming messages stay in LDS).
template <typename S_>
__global__ void __launch_bounds__(64) k_hpr_er_edge(const S_* __restrict__ chi, S_* __restrict__ chi_out,
                                                    const S_* __restrict__ biases, const int32_t* __restrict__ rows,
                                                    const int32_t* __restrict__ inc,
                                                    const int32_t* __restrict__ inc_src, Geo g, S_ w_plus,
                                                    S_ w_minus, S_ damp, int64_t e0, S_* __restrict__ gtab) {
    extern __shared__ __align__(16) unsigned char smem_raw[];
    S_* M = reinterpret_cast<S_*>(smem_raw);
    S_* tab = gtab ? gtab + (size_t)blockIdx.x * g.XV * g.S : M + (size_t)g.D * g.XV * g.X;
    const int lane = threadIdx.x;
    const int64_t e = e0 + blockIdx.x;
    const int X = g.X, NC = X * X, XV = g.XV, S = g.S, D = g.D, ab = g.ab, T = g.T;
    // M[m][a][k] = bias_{k_m}(x_k[0]) chi^{k_m -> a}(x_k, x_a), valid x_a = 2a + ab, all x_k
    for (int q = lane; q < D * XV * X; q += 64) {
        const int m = q / (XV * X), r = q % (XV * X), a = r / X, k = r % X;
        const int64_t row = inc[e * D + m];
        const int64_t src = inc_src[e * D + m];
        const S_ b = biases[2 * src + (hspin(k, 0, T) > 0 ? 0 : 1)];
        M[q] = b * chi[row * NC + k * X + (2 * a + ab)];
    }
    for (int q = lane; q < XV * S; q += 64) tab[q] = S_(0);
    __syncthreads();
    if (D == 0) {
        if (lane < XV) tab[lane * S] = S_(1);
    } else {
        for (int q = lane; q < XV * X; q += 64) {
            const int a = q / X, k = q % X;
            tab[a * S + traj_off(g, k)] += M[q];
        }
    }
    __syncthreads();
    const int tot = XV * S;
    for (int m = 1; m < D; ++m) {
        const S_* Mm = M + m * XV * X;
        // in place, top-down: an entry only reads entries at or below itself
        for (int base = ((tot - 1) / 64) * 64; base >= 0; base -= 64) {
            const int q = base + lane;
            S_ acc = S_(0);
            if (q < tot) {
                const int a = q / S, i = q % S;
                int dg[kMaxT];
                int rem = i;
                for (int t = 0; t < T; ++t) {
                    dg[t] = rem / g.pw[t];
                    rem -= dg[t] * g.pw[t];
                }
                for (int k = X - 1; k >= 0; --k) {
                    int src = i;
                    bool ok = true;
                    for (int t = 0; t < T; ++t)
                        if (hspin(k, t, T) > 0) {
                            ok = ok && dg[t] > 0;
                            src -= g.pw[t];
                        }
                    if (ok) acc += tab[a * S + src] * Mm[a * X + k];
                }
            }
            __syncthreads();
            if (q < tot) tab[q] = acc;
            __syncthreads();
        }
    }
    // suffix sums along t where the condition needs +1, prefix sums where it needs -1
    const int lines = XV * (S / g.B);
    for (int t = 0; t < T; ++t) {
        const int step = g.pw[t], span = step * g.B;
        for (int L = lane; L < lines; L += 64) {
            const int a = L / (S / g.B), r = L % (S / g.B);
            S_* p = tab + a * S + (r / step) * span + (r % step);
            S_ run = S_(0);
            if (cond_dir(g, 2 * a + ab, t) > 0) {
                for (int j = D; j >= 0; --j) {
                    run += p[j * step];
                    p[j * step] = run;
                }
            } else {
                for (int j = 0; j <= D; ++j) {
                    run += p[j * step];
                    p[j * step] = run;
                }
            }
        }
        __syncthreads();
    }
    // outputs: every column of the row (x_a[T-1] != attr: chi_new = 0)
    constexpr int CPL = 1024 / 64;                     // NC <= 256 at T <= 4: at most 4 per lane
    S_ v[CPL / 4];
    S_ rs = S_(0);
#pragma unroll
    for (int j = 0; j < CPL / 4; ++j) {
        const int col = lane + 64 * j;
        S_ x = S_(0);
        if (col < NC) {
            const int xa = col / X, xb = col % X;
            if ((xa & 1) == ab) {
                const int cn = corner(g, xa, xb);
                if (cn >= 0) x = (hspin(xa, 0, T) > 0 ? w_plus : w_minus) * tab[(xa >> 1) * S + cn];
            }
            rs += x;
        }
        v[j] = x;
    }
    rs = wave_sum(rs);
    const int64_t row = rows[e];
    const S_ inv = S_(1) / rs;
#pragma unroll
    for (int j = 0; j < CPL / 4; ++j) {
        const int col = lane + 64 * j;
        if (col < NC) chi_out[row * NC + col] = damp * (v[j] * inv) + (S_(1) - damp) * chi[row * NC + col];
    }
}

// node marginals over CSR out-rows: marg_i(+-) = prod_m Z+-[row(i -> k_m)], normalised
// (code/HPR_pytorch_RRG.py:163-167 with a per-node degree)
template <typename S_>
__global__ void __launch_bounds__(256) k_hpr_node_marg_csr(const S_* __restrict__ zp, const S_* __restrict__ zm,
                                                            const int64_t* __restrict__ out_ptr,
                                                            const int32_t* __restrict__ out_rows, int64_t n,
                                                            S_* __restrict__ marg) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    S_ p = 1, q = 1;
    for (int64_t k = out_ptr[i]; k < out_ptr[i + 1]; ++k) {
        const int64_t r = out_rows[k];
        p *= zp[r];
        q *= zm[r];
    }
    const S_ s = p + q;
    marg[2 * i] = p / s;
    marg[2 * i + 1] = q / s;
}

template <typename S_>
static int update_impl(const void* chi_in, void* chi_out, const void* biases, const int32_t* rows, const int32_t* inc,
                       const int32_t* inc_src, int64_t m, const Geo& g, double w_plus, double w_minus, double damp,
                       void* scratch, int64_t scratch_bytes, hipStream_t st) {
    auto kern = k_hpr_er_edge<S_>;
    MJX_HIP(set_max_lds(kern, (int)kMaxLds), "hpr er set lds");   // opt in to the whole LDS (once per device)
    const bool in_lds = lds_bytes<S_>(g) <= kMaxLds;
    if (!in_lds && m_bytes<S_>(g) > kMaxLds) return MJX_ERANGE;
    // table in LDS: every message in one launch; else launches of as many
    // messages as the scratch holds tables
    const int64_t per = in_lds ? m : (scratch ? scratch_bytes / (int64_t)tab_bytes<S_>(g) : 0);
    if (per < 1) return MJX_ERANGE;
    const size_t lds = in_lds ? lds_bytes<S_>(g) : m_bytes<S_>(g);
    for (int64_t e0 = 0; e0 < m; e0 += per) {
        const int64_t cnt = (m - e0 < per) ? m - e0 : per;
        if (cnt > (int64_t)INT32_MAX) return MJX_ERANGE;
        kern<<<(unsigned)cnt, 64, lds, st>>>((const S_*)chi_in, (S_*)chi_out, (const S_*)biases, rows, inc, inc_src, g,
                                             (S_)w_plus, (S_)w_minus, (S_)damp, e0, in_lds ? nullptr : (S_*)scratch);
        MJX_LAUNCH_CHECK("k_hpr_er_edge");
    }
    return MJX_OK;
}

}  // namespace hprer
}  // namespace mjx

using namespace mjx;
using namespace mjx::hprer;

extern "C" int64_t mjx_hpr_er_scratch_bytes(int dtype, int D, int p, int c) {
    Geo g;
    if (!make_geo(D, p, c, 1, &g)) return -1;
    const size_t lds = dtype == MJX_F32 ? lds_bytes<float>(g) : lds_bytes<double>(g);
    const size_t mb = dtype == MJX_F32 ? m_bytes<float>(g) : m_bytes<double>(g);
    if (dtype != MJX_F32 && dtype != MJX_F64) return -1;
    if (lds <= kMaxLds) return 0;
    if (mb > kMaxLds) return -1;
    return (int64_t)(dtype == MJX_F32 ? tab_bytes<float>(g) : tab_bytes<double>(g));
}

extern "C" int mjx_hpr_er_update_class(int dtype, const void* chi_in, void* chi_out, const void* biases,
                                       const int32_t* rows, const int32_t* inc, const int32_t* inc_src, int64_t m,
                                       int D, int p, int c, int attr_value, double w_plus, double w_minus,
                                       double damp, void* scratch, int64_t scratch_bytes, void* stream) {
    if (m < 0) return MJX_EINVAL;
    if (m == 0) return MJX_OK;
    if (!chi_in || !chi_out || chi_in == chi_out || !biases || !rows || (D > 0 && (!inc || !inc_src)))
        return MJX_EINVAL;
    Geo g;
    if (!make_geo(D, p, c, attr_value, &g)) return MJX_ERANGE;
    hipStream_t st = as_stream(stream);
    if (dtype == MJX_F32) return update_impl<float>(chi_in, chi_out, biases, rows, inc, inc_src, m, g, w_plus, w_minus,
                                                    damp, scratch, scratch_bytes, st);
    if (dtype == MJX_F64) return update_impl<double>(chi_in, chi_out, biases, rows, inc, inc_src, m, g, w_plus,
                                                     w_minus, damp, scratch, scratch_bytes, st);
    return MJX_EINVAL;
}

extern "C" int mjx_hpr_node_marg_csr(int dtype, const void* zwork, int64_t E, const int64_t* out_ptr,
                                     const int32_t* out_rows, int64_t n, void* marg, void* stream) {
    if (n < 1 || E < 1 || !zwork || !out_ptr || !out_rows || !marg) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (dtype == MJX_F32) {
        const float* zp = (const float*)zwork;
        k_hpr_node_marg_csr<float><<<grid, 256, 0, st>>>(zp, zp + 2 * E, out_ptr, out_rows, n, (float*)marg);
    } else if (dtype == MJX_F64) {
        const double* zp = (const double*)zwork;
        k_hpr_node_marg_csr<double><<<grid, 256, 0, st>>>(zp, zp + 2 * E, out_ptr, out_rows, n, (double*)marg);
    } else {
        return MJX_EINVAL;
    }
    MJX_LAUNCH_CHECK("k_hpr_node_marg_csr");
    return MJX_OK;
}
