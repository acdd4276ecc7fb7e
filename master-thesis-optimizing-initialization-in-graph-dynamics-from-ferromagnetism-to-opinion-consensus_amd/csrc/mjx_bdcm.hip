// Backtracking dynamical cavity method (BDCM) on Erdos-Renyi graphs: the
// per-degree-class edge-message update, leaf messages, node and edge partition
// functions and the free-entropy observables of code/ER_BDCM_entropy.ipynb
// ("nb:L" = raw JSON line L of the notebook).  float64, like the reference.
//
// Message layout (the reference's, so chi arrays are drop-in): chi[2E][2^T][2^T],
// row r < E = list(G.edges)[r] = (i, j) as the message i -> j, row r + E = j -> i
// (nb:303-314); trajectory index bit (T-1-t) = 1 means spin +1 at time t
// (the ndarray axes are indexed by itertools.product([1, 0]) values, nb:150-154).
//
// BDCM_ER for the message a -> b of edge class D = deg(a) - 1 (nb:312-318):
//   LL(x_a, rho) = sum over x_k1..x_kD ending in the attractor of prod_m chi^{k_m->a}(x_km, x_a),
//                  rho_t = number of +1 among x_k1[t]..x_kD[t]                  (nb:150-184)
//   chi2(x_a, x_b) = exp(-lmbd (2 x_a[0] - 1)) sum_rho A(x_a, x_b, rho) LL(x_a, rho)   (nb:186-191)
//   chi <- damp * normalize(max(chi2, eps)) + (1 - damp) * chi                  (nb:194-196)
// A is the majority / always-stay trajectory indicator (nb:66-111).  For a fixed
// x_a every time step restricts rho_t to a one-sided interval (a lower bound when
// the spin it must produce is +1, an upper bound when it is -1), so the sum over
// the box is one entry of the directional cumulative sums of LL: the contraction
// over (D+1)^T count vectors becomes one lookup per (x_a, x_b).  The node factor
// of Zi_ER (nb:211-276) is the same box with no receiver term.
//
// Kernel geometry: one workgroup per message (or node), one to four waves by the
// table size.  The DP table of every valid x_a lives in LDS and is convolved in
// place one neighbour at a time (top-down chunks of the workgroup's width, all
// reads of a chunk before a barrier and its writes: an entry reads only entries
// at or below itself), then turned into directional cumulative sums.
#include "mjx_common.h"
#include <math.h>

#pragma clang fp contract(off)

namespace mjx {
namespace bdcm {

constexpr int kMaxT = 4;
constexpr size_t kMaxLds = 160 * 1024;

struct Geo {
    int T, P, D, X, XV, B, S, ab;     // ab: trajectory index bit of the attractor spin at t = T-1
    int pw[kMaxT];                    // B^(T-1-t)
    int src_tab;                      // 1: the convolution's source indices are tabulated in LDS
};

__host__ __device__ inline int bspin(int x, int t, int T) { return ((x >> (T - 1 - t)) & 1) ? 1 : -1; }
__host__ __device__ inline int fdiv2(int a) { return a >= 0 ? a / 2 : -((-a + 1) / 2); }
__host__ __device__ inline int cdiv2(int a) { return -fdiv2(-a); }

static bool make_geo(int D, int p, int c, int attr_value, Geo* g) {
    const int T = p + c;
    if (p < 0 || c < 1 || T > kMaxT || D < 0 || D > 255) return false;
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
    g->ab = attr_value > 0 ? 1 : 0;
    g->src_tab = 0;
    return true;
}

static size_t tab_bytes(const Geo& g) { return (size_t)g.XV * g.S * sizeof(double); }
static size_t m_bytes(const Geo& g) { return (size_t)g.D * g.XV * g.XV * sizeof(double); }
static size_t lds_bytes(const Geo& g) { return tab_bytes(g) + m_bytes(g); }
// per table entry: the row offset a*XV of its x_a and, per x_k, the entry it
// reads in a convolution step (-1: none) -- the index arithmetic (runtime
// divisions by the mixed radix) done once per item instead of once per step
static size_t src_bytes(const Geo& g) { return (size_t)g.XV * g.S * (g.XV + 1) * sizeof(int32_t); }
constexpr size_t kSrcTabMax = 32 * 1024;

// the spin the condition on rho_t must produce, and the spin a tie keeps
// (traj_condition for t < T-1, atr_condition for t = T-1; nb:66-83)
__device__ inline int cond_dir(const Geo& g, int xa, int t) {
    return (t < g.T - 1) ? bspin(xa, t + 1, g.T) : bspin(xa, g.P, g.T);
}
__device__ inline int cond_prev(const Geo& g, int xa, int t) {
    return (t < g.T - 1) ? bspin(xa, t, g.T) : bspin(xa, g.T - 1, g.T);
}

// table index of the corner of the rho box allowed for (x_a, receiver), -1 when
// the box is empty.  sigma_t = 2 rho_t - D + y_t with y = spin of x_b (edge
// factor) or 0 (node factor, A_i_sums2).
__device__ inline int corner(const Geo& g, int xa, int xb, bool node) {
    int idx = 0;
    for (int t = 0; t < g.T; ++t) {
        const int s = cond_dir(g, xa, t), prev = cond_prev(g, xa, t);
        const int y = node ? 0 : bspin(xb, t, g.T);
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

__device__ inline int traj_off(const Geo& g, int x) {
    int o = 0;
    for (int t = 0; t < g.T; ++t)
        if (bspin(x, t, g.T) > 0) o += g.pw[t];
    return o;
}

__device__ inline double wave_sum(double v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// LL of item e for every valid x_a into tab[XV][S], then directional cumulative
// sums.  inc[e*D + m] = row of the m-th incoming message k_m -> a.
__device__ void build_table(const Geo& g, const double* __restrict__ chi, const int32_t* __restrict__ inc, int64_t e,
                            double* tab, double* M, int lane, int32_t* srct) {
    // every loop strides over the workgroup (one to four waves per item)
    const int nt = blockDim.x;
    const int X = g.X, NC = X * X, XV = g.XV, S = g.S, D = g.D, ab = g.ab, T = g.T;
    // M[m][a][k] = chi^{k_m -> a}(x_k, x_a), valid x_a = 2a+ab, x_k = 2k+ab
    for (int q = lane; q < D * XV * XV; q += nt) {
        const int m = q / (XV * XV), r = q % (XV * XV), a = r / XV, k = r % XV;
        const int64_t row = inc[e * D + m];
        M[q] = chi[row * NC + (2 * k + ab) * X + (2 * a + ab)];
    }
    for (int q = lane; q < XV * S; q += nt) tab[q] = 0.0;
    __syncthreads();
    if (D == 0) {
        if (lane < XV) tab[lane * S] = 1.0;
    } else {
        for (int q = lane; q < XV * XV; q += nt) {
            const int a = q / XV, k = q % XV;
            tab[a * S + traj_off(g, 2 * k + ab)] = M[q];
        }
    }
    const int tot = XV * S;
    if (srct && D > 1) {
        for (int q = lane; q < tot; q += nt) {
            const int a = q / S, i = q % S;
            int dg[kMaxT];
            int rem = i;
            for (int t = 0; t < T; ++t) {
                dg[t] = rem / g.pw[t];
                rem -= dg[t] * g.pw[t];
            }
            int32_t* row = srct + q * (XV + 1);
            row[0] = a * XV;
            for (int k = XV - 1; k >= 0; --k) {
                const int xk = 2 * k + ab;
                int src = i;
                bool ok = true;
                for (int t = 0; t < T; ++t)
                    if (bspin(xk, t, T) > 0) {
                        ok = ok && dg[t] > 0;
                        src -= g.pw[t];
                    }
                row[1 + k] = ok ? a * S + src : -1;
            }
        }
    }
    __syncthreads();
    for (int m = 1; m < D && srct; ++m) {
        const double* Mm = M + m * XV * XV;
        for (int base = ((tot - 1) / nt) * nt; base >= 0; base -= nt) {
            const int q = base + lane;
            double acc = 0.0;
            if (q < tot) {
                const int32_t* row = srct + q * (XV + 1);
                const double* Ma = Mm + row[0];
                for (int k = XV - 1; k >= 0; --k) {       // the same order as below
                    const int src = row[1 + k];
                    if (src >= 0) acc += tab[src] * Ma[k];
                }
            }
            __syncthreads();
            if (q < tot) tab[q] = acc;
            __syncthreads();
        }
    }
    for (int m = 1; m < D && !srct; ++m) {
        const double* Mm = M + m * XV * XV;
        // in place, top-down: an entry only reads entries at or below itself
        for (int base = ((tot - 1) / nt) * nt; base >= 0; base -= nt) {
            const int q = base + lane;
            double acc = 0.0;
            if (q < tot) {
                const int a = q / S, i = q % S;
                int dg[kMaxT];
                int rem = i;
                for (int t = 0; t < T; ++t) {
                    dg[t] = rem / g.pw[t];
                    rem -= dg[t] * g.pw[t];
                }
                for (int k = XV - 1; k >= 0; --k) {
                    const int xk = 2 * k + ab;
                    int src = i;
                    bool ok = true;
                    for (int t = 0; t < T; ++t)
                        if (bspin(xk, t, T) > 0) {
                            ok = ok && dg[t] > 0;
                            src -= g.pw[t];
                        }
                    if (ok) acc += tab[a * S + src] * Mm[a * XV + k];
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
        for (int L = lane; L < lines; L += nt) {
            const int a = L / (S / g.B), r = L % (S / g.B);
            double* p = tab + a * S + (r / step) * span + (r % step);
            double run = 0.0;
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
}

// BDCM_ER for one edge class (nb:150-196), new rows into upd[m][NC].
// damp >= 1 assigns normalize(chi2) (the leaf reset of nb:404-417 is class D = 0).
// The count table lives in LDS, or (a class whose table exceeds the LDS budget)
// in the global slab gtab, one table per workgroup of the launch; item e0 + blockIdx.x.
__global__ void __launch_bounds__(256) k_bdcm_edge(const double* __restrict__ chi, const int32_t* __restrict__ rows,
                                                  const int32_t* __restrict__ inc, Geo g, double w_plus,
                                                  double w_minus, double eps, double damp, double* __restrict__ upd,
                                                  int64_t e0, double* __restrict__ gtab,
                                                  const long long* __restrict__ gate,
                                                  const double* __restrict__ w_dev) {
    if (gate && *gate) return;                 // a converged loop replays as no-ops
    if (w_dev) {                               // lambda's weights from device memory (a captured loop)
        w_plus = w_dev[0];
        w_minus = w_dev[1];
    }
    extern __shared__ __align__(16) double sm[];
    double* M = sm;
    double* tab = gtab ? gtab + (size_t)blockIdx.x * g.XV * g.S : sm + (size_t)g.D * g.XV * g.XV;
    const int lane = threadIdx.x;
    const int64_t e = e0 + blockIdx.x;
    build_table(g, chi, inc, e, tab, M, lane,
                g.src_tab ? reinterpret_cast<int32_t*>(sm + (size_t)g.D * g.XV * g.XV + (size_t)g.XV * g.S) : nullptr);
    if (lane >= 64) return;                    // the epilogue is one wave's (no barrier follows)
    const int X = g.X, NC = X * X;
    double v[4];
    double rs = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        double x = 0.0;
        if (col < NC) {
            const int xa = col / X, xb = col % X;
            if ((xa & 1) == g.ab) {
                const int cn = corner(g, xa, xb, false);
                if (cn >= 0) x = (bspin(xa, 0, g.T) > 0 ? w_plus : w_minus) * tab[(xa >> 1) * g.S + cn];
            }
            x = (x < eps) ? eps : x;           // np.maximum(chi2, epsilon); a NaN stays NaN
            rs += x;
        }
        v[j] = x;
    }
    rs = wave_sum(rs);
    const int64_t row = rows[e];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        if (col < NC) {
            const double nv = v[j] / rs;       // normalize (nb:128-130), no epsilon
            upd[e * NC + col] = (damp >= 1.0) ? nv : damp * nv + (1.0 - damp) * chi[row * NC + col];
        }
    }
}

// scatter the class's new rows into chi; max |new - old| as double bits
__global__ void __launch_bounds__(256) k_bdcm_commit(double* __restrict__ chi, const int32_t* __restrict__ rows,
                                                     int64_t m, int NC, const double* __restrict__ upd,
                                                     unsigned long long* __restrict__ delta_bits,
                                                     const long long* __restrict__ gate) {
    if (gate && *gate) return;
    unsigned long long mx = 0;
    const int64_t total = m * NC;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
        const int64_t e = q / NC;
        const int col = (int)(q % NC);
        double* p = chi + (int64_t)rows[e] * NC + col;
        const double nv = upd[q];
        // |d| >= 0 orders like its bit pattern; a NaN (0x7ff8...) beats every number
        const unsigned long long b = (unsigned long long)__double_as_longlong(fabs(nv - *p));
        mx = b > mx ? b : mx;
        *p = nv;
    }
    if (delta_bits) {
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        if ((threadIdx.x & 63) == 0 && mx) atomicMax(delta_bits, mx);
    }
}

// the notebook's convergence loop on the device (nb:422-431):
//   while delta > eps: delta = BDCM sweep; t += 1; if t >= T_max: stop
// ctl[0] = delta bits of the running sweep, ctl[1] = stop flag, ctl[2] = t,
// ctl[3] = delta bits of the last completed sweep.  One thread, plain stores.
__global__ void k_bdcm_iter_begin(long long* __restrict__ ctl) {
    if (threadIdx.x == 0 && ctl[1] == 0) ctl[0] = 0;
}

__global__ void k_bdcm_iter_end(long long* __restrict__ ctl, double eps, long long t_max) {
    if (threadIdx.x != 0 || ctl[1] != 0) return;
    const long long bits = ctl[0];
    const double delta = __longlong_as_double(bits);
    const long long t = ctl[2] + 1;
    ctl[2] = t;
    ctl[3] = bits;
    if (!(delta > eps) || t >= t_max) ctl[1] = 1;      // NaN ends the loop too (while NaN > eps is false)
}

// Zi_ER for one node-degree class (nb:211-276): zi[node] = max(sum_xa w Ai LL, eps)
__global__ void __launch_bounds__(256) k_bdcm_node(const double* __restrict__ chi, const int32_t* __restrict__ nodes,
                                                  const int32_t* __restrict__ inc, Geo g, double w_plus,
                                                  double w_minus, double eps, double* __restrict__ zi, int64_t e0,
                                                  double* __restrict__ gtab) {
    extern __shared__ __align__(16) double sm[];
    double* M = sm;
    double* tab = gtab ? gtab + (size_t)blockIdx.x * g.XV * g.S : sm + (size_t)g.D * g.XV * g.XV;
    const int lane = threadIdx.x;
    const int64_t e = e0 + blockIdx.x;
    build_table(g, chi, inc, e, tab, M, lane,
                g.src_tab ? reinterpret_cast<int32_t*>(sm + (size_t)g.D * g.XV * g.XV + (size_t)g.XV * g.S) : nullptr);
    if (lane >= 64) return;
    double z = 0.0;
    if (lane < g.XV) {
        const int xa = 2 * lane + g.ab;
        const int cn = corner(g, xa, 0, true);
        if (cn >= 0) z = (bspin(xa, 0, g.T) > 0 ? w_plus : w_minus) * tab[lane * g.S + cn];
    }
    z = wave_sum(z);
    if (lane == 0) zi[nodes[e]] = (z < eps) ? eps : z;
}

// Zij (nb:200-209) and the per-edge m_init term (nb:379-392)
__global__ void __launch_bounds__(256) k_bdcm_edge_obs(const double* __restrict__ chi, const int32_t* __restrict__ edges,
                                                       const int32_t* __restrict__ deg, int64_t E, int T, int ab,
                                                       double eps, double* __restrict__ zij,
                                                       double* __restrict__ mterm) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const int X = 1 << T, NC = X * X, XV = X / 2;
    const double du = (double)deg[edges[2 * e]], dv = (double)deg[edges[2 * e + 1]];
    const double* f = chi + e * NC;
    const double* b = chi + (e + E) * NC;
    double z = 0.0, mt = 0.0;
    for (int a = XV - 1; a >= 0; --a) {
        const int xa = 2 * a + ab;
        const double sa = (double)bspin(xa, 0, T);
        for (int c = XV - 1; c >= 0; --c) {
            const int xb = 2 * c + ab;
            const double pr = f[xa * X + xb] * b[xb * X + xa];
            z += pr;
            mt += (sa / du + (double)bspin(xb, 0, T) / dv) * pr;
        }
    }
    z = (z < eps) ? eps : z;
    zij[e] = z;
    if (mterm) mterm[e] = mt / z;
}

// deterministic two-level sum (of logs): fixed grid, fixed tree
constexpr int kSumBlocks = 256;

__device__ inline double block_sum256(double s, double* red) {
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    return red[0];
}

__global__ void __launch_bounds__(256) k_sum_partial(const double* __restrict__ x, int64_t n, int take_log,
                                                     double* __restrict__ part) {
    __shared__ double red[256];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        s += take_log ? log(x[i]) : x[i];
    const double t = block_sum256(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void __launch_bounds__(256) k_sum_final(const double* __restrict__ part, int np, double* __restrict__ out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += 256) s += part[i];
    const double t = block_sum256(s, red);
    if (threadIdx.x == 0) out[0] = t;
}

template <typename K>
static int set_lds(K kern) {
    MJX_HIP(set_max_lds(kern, (int)kMaxLds), "bdcm set lds");   // opt in to the whole LDS (once per device)
    return MJX_OK;
}

// items per launch and dynamic LDS: everything in LDS when the table fits,
// else as many tables as the scratch slab holds (0: unsupported)
// one wave per item for small tables, up to four for the hub classes (the
// convolution is a serial chain of D-1 steps over ceil(tot / width) chunks)
static int item_threads(const Geo& g) {
    const int64_t tot = (int64_t)g.XV * g.S;
    return tot <= 128 ? 64 : (tot <= 512 ? 128 : 256);
}

static int64_t plan_launch(Geo& g, int64_t m, void* scratch, int64_t scratch_bytes, size_t* lds, bool* in_lds) {
    *in_lds = lds_bytes(g) <= kMaxLds;
    *lds = *in_lds ? lds_bytes(g) : m_bytes(g);
    g.src_tab = (*in_lds && g.D > 1 && src_bytes(g) <= kSrcTabMax && lds_bytes(g) + src_bytes(g) <= kMaxLds) ? 1 : 0;
    if (g.src_tab) *lds += src_bytes(g);
    if (!*in_lds && m_bytes(g) > kMaxLds) return 0;
    if (*in_lds) return m;
    return scratch ? scratch_bytes / (int64_t)tab_bytes(g) : 0;
}

}  // namespace bdcm
}  // namespace mjx

using namespace mjx;
using namespace mjx::bdcm;

extern "C" int64_t mjx_bdcm_lds_bytes(int D, int p, int c) {
    Geo g;
    if (!make_geo(D, p, c, 1, &g)) return -1;
    return (int64_t)lds_bytes(g);
}

extern "C" int64_t mjx_bdcm_scratch_bytes(int D, int p, int c) {
    Geo g;
    if (!make_geo(D, p, c, 1, &g)) return -1;
    if (lds_bytes(g) <= kMaxLds) return 0;
    if (m_bytes(g) > kMaxLds) return -1;
    return (int64_t)tab_bytes(g);
}

extern "C" int mjx_bdcm_update_class(double* chi, const int32_t* rows, const int32_t* inc, int64_t m, int D, int p,
                                     int c, int attr_value, double lmbd, double damp, double eps, double* upd,
                                     unsigned long long* delta_bits, const long long* gate, const double* w_dev,
                                     void* scratch, int64_t scratch_bytes, void* stream) {
    if (m < 0 || !chi) return MJX_EINVAL;
    if (m == 0) return MJX_OK;
    if (!rows || !upd || (D > 0 && !inc) || !(damp > 0.0)) return MJX_EINVAL;
    Geo g;
    if (!make_geo(D, p, c, attr_value, &g)) return MJX_ERANGE;
    size_t lds;
    bool in_lds;
    const int64_t per = plan_launch(g, m, scratch, scratch_bytes, &lds, &in_lds);
    if (per < 1) return MJX_ERANGE;
    hipStream_t st = as_stream(stream);
    int rc = set_lds(k_bdcm_edge);
    if (rc) return rc;
    // exp(-lmbd*(2 x_a[0] - 1)) for x_a[0] = +1 / -1 (nb:191)
    for (int64_t e0 = 0; e0 < m; e0 += per) {
        const int64_t cnt = (m - e0 < per) ? m - e0 : per;
        if (cnt > (int64_t)INT32_MAX) return MJX_ERANGE;
        k_bdcm_edge<<<(unsigned)cnt, item_threads(g), lds, st>>>(chi, rows, inc, g, exp(-lmbd), exp(lmbd), eps, damp, upd, e0,
                                                    in_lds ? nullptr : (double*)scratch, gate, w_dev);
        MJX_LAUNCH_CHECK("k_bdcm_edge");
    }
    const int NC = g.X * g.X;
    k_bdcm_commit<<<grid_for(m * NC), 256, 0, st>>>(chi, rows, m, NC, upd, delta_bits, gate);
    MJX_LAUNCH_CHECK("k_bdcm_commit");
    return MJX_OK;
}

extern "C" int mjx_bdcm_iter_begin(long long* ctl, void* stream) {
    if (!ctl) return MJX_EINVAL;
    k_bdcm_iter_begin<<<1, 64, 0, as_stream(stream)>>>(ctl);
    MJX_LAUNCH_CHECK("k_bdcm_iter_begin");
    return MJX_OK;
}

extern "C" int mjx_bdcm_iter_end(long long* ctl, double eps, int64_t t_max, void* stream) {
    if (!ctl) return MJX_EINVAL;
    k_bdcm_iter_end<<<1, 64, 0, as_stream(stream)>>>(ctl, eps, (long long)t_max);
    MJX_LAUNCH_CHECK("k_bdcm_iter_end");
    return MJX_OK;
}

extern "C" int mjx_bdcm_node_z(const double* chi, const int32_t* nodes, const int32_t* inc, int64_t m, int D, int p,
                               int c, int attr_value, double lmbd, double eps, double* zi, void* scratch,
                               int64_t scratch_bytes, void* stream) {
    if (m < 0 || !chi || !zi) return MJX_EINVAL;
    if (m == 0) return MJX_OK;
    if (!nodes || (D > 0 && !inc)) return MJX_EINVAL;
    Geo g;
    if (!make_geo(D, p, c, attr_value, &g)) return MJX_ERANGE;
    size_t lds;
    bool in_lds;
    const int64_t per = plan_launch(g, m, scratch, scratch_bytes, &lds, &in_lds);
    if (per < 1) return MJX_ERANGE;
    hipStream_t st = as_stream(stream);
    int rc = set_lds(k_bdcm_node);
    if (rc) return rc;
    for (int64_t e0 = 0; e0 < m; e0 += per) {
        const int64_t cnt = (m - e0 < per) ? m - e0 : per;
        if (cnt > (int64_t)INT32_MAX) return MJX_ERANGE;
        k_bdcm_node<<<(unsigned)cnt, item_threads(g), lds, st>>>(chi, nodes, inc, g, exp(-lmbd), exp(lmbd), eps, zi, e0,
                                                    in_lds ? nullptr : (double*)scratch);
        MJX_LAUNCH_CHECK("k_bdcm_node");
    }
    return MJX_OK;
}

extern "C" int mjx_bdcm_edge_obs(const double* chi, const int32_t* edges, const int32_t* deg, int64_t E, int p, int c,
                                 int attr_value, double eps, double* zij, double* m_term, void* stream) {
    if (E < 0 || p < 0 || c < 1 || p + c > kMaxT || (attr_value != 1 && attr_value != -1)) return MJX_EINVAL;
    if (E == 0) return MJX_OK;
    if (!chi || !edges || !deg || !zij) return MJX_EINVAL;
    k_bdcm_edge_obs<<<(unsigned)((E + 255) / 256), 256, 0, as_stream(stream)>>>(
        chi, edges, deg, E, p + c, attr_value > 0 ? 1 : 0, eps, zij, m_term);
    MJX_LAUNCH_CHECK("k_bdcm_edge_obs");
    return MJX_OK;
}

extern "C" int mjx_sum_f64(const double* x, int64_t n, int take_log, double* work, double* out, void* stream) {
    if (n < 0 || !work || !out || (n > 0 && !x)) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    k_sum_partial<<<kSumBlocks, 256, 0, st>>>(x, n, take_log, work);
    MJX_LAUNCH_CHECK("k_sum_partial");
    k_sum_final<<<1, 256, 0, st>>>(work, kSumBlocks, out);
    MJX_LAUNCH_CHECK("k_sum_final");
    return MJX_OK;
}
