// C ABI of the HPR kernels (code/HPR_pytorch_RRG.py:137-218); kernels in mjx_hpr_impl.h.
#include "mjx_hpr_impl.h"


using namespace mjx;
using namespace mjx::hpr;

extern "C" int mjx_hpr_update(int dtype, const void* chi_in, void* chi_out, const void* biases, const int32_t* nbr,
                              const int32_t* in_row, const int32_t* out_row, int64_t n, int d, int p, int c,
                              int attr_value, double w_plus, double w_minus, double damp, void* stream) {
    if (n < 1 || d < 2 || p < 1 || c < 1 || (attr_value != 1 && attr_value != -1)) return MJX_EINVAL;
    if (!chi_in || !chi_out || !biases || !nbr || !in_row || !out_row || chi_in == chi_out) return MJX_EINVAL;
    if (n * (int64_t)d > (int64_t)INT32_MAX) return MJX_ERANGE;
    const int ap = attr_value > 0 ? 1 : 0;
    hipStream_t st = as_stream(stream);
    if (dtype == MJX_F32)
        return update_f32(chi_in, chi_out, biases, nbr, in_row, out_row, n, d, p, c, ap, w_plus, w_minus, damp, st);
    if (dtype == MJX_F64)
        return update_f64(chi_in, chi_out, biases, nbr, in_row, out_row, n, d, p, c, ap, w_plus, w_minus, damp, st);
    return MJX_EINVAL;
}

template <typename S>
static int edge_z_impl(const void* chi, int64_t E, int T, double eps, void* zwork, hipStream_t st) {
    S* zp = (S*)zwork;
    S* zm = zp + 2 * E;
    // one grid-stride round of resident waves (a larger grid runs a partly empty second round)
#define MJX_EDGE_Z(TT)                                                                                   \
    case TT: {                                                                                           \
        auto k = k_hpr_edge_z<S, TT>;                                                                    \
        const int64_t lanes = E * (1 << TT) / 2;           /* U = 2 edge groups per lane */             \
        k<<<resident_grid(k, 256, 0, lanes), 256, 0, st>>>((const S*)chi, E, (S)eps, zp, zm);            \
        break;                                                                                           \
    }
    switch (T) {
        MJX_EDGE_Z(2) MJX_EDGE_Z(3) MJX_EDGE_Z(4) MJX_EDGE_Z(5)
        default: return MJX_ERANGE;
    }
#undef MJX_EDGE_Z
    MJX_LAUNCH_CHECK("k_hpr_edge_z");
    return MJX_OK;
}

template <typename S>
static int marginals_impl(const void* chi, const int32_t* out_row, int64_t n, int d, int T, double eps, void* zwork,
                          void* marg, hipStream_t st) {
    const int64_t E = n * (int64_t)d / 2;
    const int rc = edge_z_impl<S>(chi, E, T, eps, zwork, st);
    if (rc) return rc;
    const S* zp = (const S*)zwork;
    k_hpr_node_marg<S><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(zp, zp + 2 * E, out_row, n, d, (S*)marg);
    MJX_LAUNCH_CHECK("k_hpr_node_marg");
    return MJX_OK;
}

extern "C" int mjx_hpr_marginals(int dtype, const void* chi, const int32_t* out_row, int64_t n, int d, int p, int c,
                                 double eps, void* zwork, void* marg, void* stream) {
    if (n < 1 || d < 1 || p < 1 || c < 1 || !chi || !out_row || !zwork || !marg) return MJX_EINVAL;
    if ((n * (int64_t)d) % 2) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    if (dtype == MJX_F32) return marginals_impl<float>(chi, out_row, n, d, p + c, eps, zwork, marg, st);
    if (dtype == MJX_F64) return marginals_impl<double>(chi, out_row, n, d, p + c, eps, zwork, marg, st);
    return MJX_EINVAL;
}

extern "C" int mjx_hpr_edge_z(int dtype, const void* chi, int64_t E, int p, int c, double eps, void* zwork,
                              void* stream) {
    if (E < 1 || p < 1 || c < 1 || !chi || !zwork) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    if (dtype == MJX_F32) return edge_z_impl<float>(chi, E, p + c, eps, zwork, st);
    if (dtype == MJX_F64) return edge_z_impl<double>(chi, E, p + c, eps, zwork, st);
    return MJX_EINVAL;
}

extern "C" int mjx_hpr_new_biases(int dtype, void* biases, const void* marg, const double* u, double thresh,
                                  double pie, int64_t n, int32_t* s, void* stream) {
    if (n < 1 || !biases || !marg || !u) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (dtype == MJX_F32)
        k_hpr_new_biases<float><<<grid, 256, 0, st>>>((float*)biases, (const float*)marg, u, thresh, (float)pie, n, s);
    else if (dtype == MJX_F64)
        k_hpr_new_biases<double><<<grid, 256, 0, st>>>((double*)biases, (const double*)marg, u, thresh, pie, n, s);
    else
        return MJX_EINVAL;
    MJX_LAUNCH_CHECK("k_hpr_new_biases");
    return MJX_OK;
}

extern "C" int mjx_hpr_node_step(int dtype, const void* zwork, const int32_t* out_row, int64_t n, int d, void* marg,
                                 void* biases, const uint8_t* refresh, double pie, int32_t* s, uint64_t* bits,
                                 void* stream) {
    if (n < 1 || d < 1 || !zwork || !out_row || !marg || !biases || !refresh || !s || !bits) return MJX_EINVAL;
    if ((n * (int64_t)d) % 2) return MJX_EINVAL;
    const int64_t E = n * (int64_t)d / 2;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (dtype == MJX_F32) {
        const float* zp = (const float*)zwork;
        k_hpr_node_step<float><<<grid, 256, 0, st>>>(zp, zp + 2 * E, out_row, n, d, (float*)marg, (float*)biases,
                                                     refresh, (float)pie, s, (u64*)bits);
    } else if (dtype == MJX_F64) {
        const double* zp = (const double*)zwork;
        k_hpr_node_step<double><<<grid, 256, 0, st>>>(zp, zp + 2 * E, out_row, n, d, (double*)marg, (double*)biases,
                                                      refresh, pie, s, (u64*)bits);
    } else {
        return MJX_EINVAL;
    }
    MJX_LAUNCH_CHECK("k_hpr_node_step");
    return MJX_OK;
}

extern "C" int mjx_hpr_new_biases_mask(int dtype, void* biases, const void* marg, const uint8_t* refresh,
                                       double pie, int64_t n, int32_t* s, void* stream) {
    if (n < 1 || !biases || !marg || !refresh) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (dtype == MJX_F32)
        k_hpr_new_biases_mask<float><<<grid, 256, 0, st>>>((float*)biases, (const float*)marg, refresh, (float)pie, n, s);
    else if (dtype == MJX_F64)
        k_hpr_new_biases_mask<double><<<grid, 256, 0, st>>>((double*)biases, (const double*)marg, refresh, pie, n, s);
    else
        return MJX_EINVAL;
    MJX_LAUNCH_CHECK("k_hpr_new_biases_mask");
    return MJX_OK;
}

// per-node bias pairs out[2v + k] = src[idx[v] * stride + k * half]: the
// node-indexed biases the update kernels read, taken from the reference's
// chi-shaped biases_chi (stride = 4^T, half = 4^T / 2; code/HPR_pytorch_RRG.py:
// 120-133, first half of a row = x_k^0 = +1) or from a permuted biases_i
// (stride 2, half 1)
template <typename S>
__global__ void k_hpr_node_biases(const S* __restrict__ src, const int64_t* __restrict__ idx, int64_t stride,
                                  int64_t half, int64_t n, S* __restrict__ out) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = idx[v] * stride;
        out[2 * v] = src[a];
        out[2 * v + 1] = src[a + half];
    }
}

extern "C" int mjx_hpr_node_biases(int dtype, const void* src, const int64_t* idx, int64_t stride, int64_t half,
                                   int64_t n, void* out, void* stream) {
    if (n < 1 || stride < 1 || half < 0 || half >= stride || !src || !idx || !out) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)grid_for(n, 8);
    if (dtype == MJX_F32)
        k_hpr_node_biases<float><<<grid, 256, 0, st>>>((const float*)src, idx, stride, half, n, (float*)out);
    else if (dtype == MJX_F64)
        k_hpr_node_biases<double><<<grid, 256, 0, st>>>((const double*)src, idx, stride, half, n, (double*)out);
    else
        return MJX_EINVAL;
    MJX_LAUNCH_CHECK("k_hpr_node_biases");
    return MJX_OK;
}

// ---- the decay-split layout of the HPR loop state (see mjx_hpr_impl.h) -------
extern "C" int mjx_hpr_q_supported(int dtype, int d, int p, int c) {
    return (dtype == MJX_F32 && q_supported(d, p, c)) ? 1 : 0;
}

extern "C" int mjx_hpr_qlayout(int dtype, const void* src, void* dst, int64_t rows, int p, int c, int attr_value,
                               int to_q, double scale, void* stream) {
    const int T = p + c;
    if (rows < 0 || p < 1 || c < 1 || T > 6 || (attr_value != 1 && attr_value != -1) || src == dst) return MJX_EINVAL;
    if (rows == 0) return MJX_OK;
    if (!src || !dst) return MJX_EINVAL;
    const int pv = attr_value > 0 ? 0 : 1;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)grid_for(rows << (2 * T), 8);
    if (dtype == MJX_F32)
        k_hpr_qperm<float><<<grid, 256, 0, st>>>((const float*)src, (float*)dst, rows, T, pv, to_q, (float)scale);
    else if (dtype == MJX_F64)
        k_hpr_qperm<double><<<grid, 256, 0, st>>>((const double*)src, (double*)dst, rows, T, pv, to_q, scale);
    else
        return MJX_EINVAL;
    MJX_LAUNCH_CHECK("k_hpr_qperm");
    return MJX_OK;
}

extern "C" int mjx_hpr_update_q(int dtype, const void* chi_in, void* chi_out, const void* biases, const int32_t* nbr,
                                const int32_t* in_row, const int32_t* out_row, int64_t n, int d, int p, int c,
                                int attr_value, double w_plus, double w_minus, double damp, const void* scale_in,
                                void* stream) {
    if (n < 1 || d < 2 || p < 1 || c < 1 || (attr_value != 1 && attr_value != -1)) return MJX_EINVAL;
    if (!chi_in || !chi_out || !biases || !nbr || !in_row || !out_row || !scale_in || chi_in == chi_out)
        return MJX_EINVAL;
    if (dtype != MJX_F32) return MJX_ERANGE;
    if (n * (int64_t)d > (int64_t)INT32_MAX) return MJX_ERANGE;
    return update_q_f32(chi_in, chi_out, biases, nbr, in_row, out_row, n, d, p, c, attr_value > 0 ? 1 : 0, w_plus,
                        w_minus, damp, (const float*)scale_in, as_stream(stream));
}

template <typename S>
static int marginals_q_impl(const void* chi, const int32_t* out_row, int64_t n, int d, int T, double eps,
                            const void* scale, const void* ii, void* zwork, void* marg, hipStream_t st) {
    const int64_t E = n * (int64_t)d / 2;
    S* zp = (S*)zwork;
    S* zm = zp + 2 * E;
    // ii (nullable): precomputed II x II sums (mjx_hpr_q_ii), used where whole
    // 16-B pieces fall in one quadrant
#define MJX_EDGE_ZQ(TT)                                                                                  \
    case TT: {                                                                                           \
        const int64_t lanes = E * (1 << TT) / 2;                                                         \
        if constexpr (QZ<S, TT>::ALIGNED) {                                                              \
            if (ii) {                                                                                    \
                auto k = k_hpr_edge_z_q<S, TT, true>;                                                    \
                k<<<resident_grid(k, 256, 0, lanes), 256, 0, st>>>((const S*)chi, E, (S)eps, (const S*)scale, \
                                                                   zp, zm, (const S*)ii);                \
                break;                                                                                   \
            }                                                                                            \
        }                                                                                                \
        auto k = k_hpr_edge_z_q<S, TT, false>;                                                           \
        k<<<resident_grid(k, 256, 0, lanes), 256, 0, st>>>((const S*)chi, E, (S)eps, (const S*)scale, zp, zm, \
                                                           nullptr);                                     \
        break;                                                                                           \
    }
    switch (T) {
        MJX_EDGE_ZQ(2) MJX_EDGE_ZQ(3) MJX_EDGE_ZQ(4) MJX_EDGE_ZQ(5)
        default: return MJX_ERANGE;
    }
#undef MJX_EDGE_ZQ
    MJX_LAUNCH_CHECK("k_hpr_edge_z_q");
    if (!marg) return MJX_OK;                 // the edge sums only (mjx_hpr_node_step follows)
    k_hpr_node_marg<S><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(zp, zm, out_row, n, d, (S*)marg);
    MJX_LAUNCH_CHECK("k_hpr_node_marg");
    return MJX_OK;
}

extern "C" int mjx_hpr_marginals_q(int dtype, const void* chi, const int32_t* out_row, int64_t n, int d, int p, int c,
                                   double eps, const void* scale, const void* ii, void* zwork, void* marg,
                                   void* stream) {
    if (n < 1 || d < 1 || p < 1 || c < 1 || !chi || !out_row || !scale || !zwork) return MJX_EINVAL;
    if ((n * (int64_t)d) % 2) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    if (dtype == MJX_F32) return marginals_q_impl<float>(chi, out_row, n, d, p + c, eps, scale, ii, zwork, marg, st);
    if (dtype == MJX_F64) return marginals_q_impl<double>(chi, out_row, n, d, p + c, eps, scale, ii, zwork, marg, st);
    return MJX_EINVAL;
}

extern "C" int mjx_hpr_q_ii(int dtype, const void* chi, int64_t E, int p, int c, void* ii, void* stream) {
    if (E < 1 || p < 1 || c < 1 || !chi || !ii) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    const unsigned grid = (unsigned)grid_for(E, 8);
#define MJX_QII(TT)                                                                                      \
    case TT:                                                                                             \
        if (dtype == MJX_F32) k_hpr_q_ii<float, TT><<<grid, 256, 0, st>>>((const float*)chi, E, (float*)ii); \
        else if (dtype == MJX_F64) k_hpr_q_ii<double, TT><<<grid, 256, 0, st>>>((const double*)chi, E, (double*)ii); \
        else return MJX_EINVAL;                                                                          \
        break;
    switch (p + c) {
        MJX_QII(2) MJX_QII(3) MJX_QII(4) MJX_QII(5)
        default: return MJX_ERANGE;
    }
#undef MJX_QII
    MJX_LAUNCH_CHECK("k_hpr_q_ii");
    return MJX_OK;
}

// ---- the reference's per-iteration torch.rand(n) on the device -----------------
// new_biases_i draws torch.rand(n) on torch's CPU generator every iteration
// (code/HPR_pytorch_RRG.py:142).  That generator is an MT19937 whose float64
// uniform is ((y_hi << 32 | y_lo) & (2^53 - 1)) * 2^-53 from two consecutive
// 32-bit outputs, with the engine state (624 words, `left`, `next`: a call
// decrements left, twists when it reaches 0, then returns state[next++]
// tempered).  One workgroup continues that stream from the caller's state for k
// iterations of n uniforms and writes the refresh masks mask[j*n + i] =
// (u < thresh[j]); the state is left where the CPU generator would be.  The
// twist runs in LDS in three dependency phases (words [0,227), [227,454),
// [454,624)); each block of 624 outputs is tempered and paired in parallel.
namespace {
constexpr int kMT = 624, kMTM = 397;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__global__ void __launch_bounds__(1024) k_mt_refresh_masks(uint32_t* __restrict__ state, int32_t* __restrict__ ln,
                                                            int64_t n, int k, const double* __restrict__ thresh,
                                                            uint8_t* __restrict__ mask) {
    __shared__ uint32_t buf[2][kMT];           // the state, ping-pong across twists
    const int tid = threadIdx.x;
    for (int i = tid; i < kMT; i += blockDim.x) buf[0][i] = state[i];
    int cur = 0;
    const int left0 = ln[0], next0 = ln[1];
    __syncthreads();
    const int64_t total = 2 * n * (int64_t)k;  // 32-bit outputs to consume
    int64_t done = 0;                          // outputs consumed so far
    int pos = next0;                           // next state word to read
    int avail = left0 - 1;                     // words readable before a twist
    bool carry = false;                        // an unpaired high word from the previous block
    uint32_t cval = 0;
    while (done < total) {
        if (avail == 0) {
            // twist into the other buffer: three dependency phases, one barrier each
            const uint32_t* o = buf[cur];
            uint32_t* w = buf[cur ^ 1];
            if (tid < 227) w[tid] = mt_mix(o[tid], o[tid + 1], o[tid + kMTM]);
            __syncthreads();
            if (tid < 227) w[tid + 227] = mt_mix(o[tid + 227], o[tid + 228], w[tid]);
            __syncthreads();
            if (tid < 170) {
                const int i = tid + 454;
                w[i] = mt_mix(o[i], (i + 1 < kMT) ? o[i + 1] : w[0], w[i - 227]);
            }
            __syncthreads();
            cur ^= 1;
            pos = 0;
            avail = kMT;
        }
        const uint32_t* mt = buf[cur];
        const int64_t need = total - done;
        const int cnt = (int)((int64_t)avail < need ? (int64_t)avail : need);
        const int off = carry ? 1 : 0;
        const int have = off + cnt;
        const int pairs = have / 2;
        const int64_t d0 = (done - off) / 2;   // uniform index of this block's first pair
        const int64_t j0 = d0 / n, r0 = d0 - j0 * n;   // its iteration and node (one division per block)
        const double th0 = thresh[j0];
        for (int q = tid; q < pairs; q += blockDim.x) {
            const int w0 = 2 * q - off;        // word of the pair's high half (-1: the carried one)
            const uint32_t hi = (w0 < 0) ? cval : mt_temper(mt[pos + w0]);
            const uint32_t lo = mt_temper(mt[pos + w0 + 1]);
            const uint64_t r = ((uint64_t)hi << 32) | lo;
            const double u = (double)(r & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
            const int64_t rq = r0 + q;
            const double th = (rq < n) ? th0 : thresh[j0 + rq / n];
            mask[d0 + q] = u < th ? 1 : 0;
        }
        carry = (have & 1) != 0;
        if (carry) cval = mt_temper(mt[pos + cnt - 1]);
        done += cnt;
        pos += cnt;
        avail -= cnt;
        __syncthreads();                       // the next twist overwrites the other buffer only
    }
    for (int i = tid; i < kMT; i += blockDim.x) state[i] = buf[cur][i];
    if (tid == 0) {
        // where the CPU engine would be: `pos` words of the current state read
        // (left + next = 625 after any read; a twist pending when pos = 624)
        ln[0] = kMT + 1 - pos;
        ln[1] = pos;
    }
}
}  // namespace

extern "C" int mjx_hpr_refresh_masks(uint32_t* state, int32_t* left_next, int64_t n, int k, const double* thresh,
                                     uint8_t* mask, void* stream) {
    if (n < 1 || k < 0 || !state || !left_next || (k > 0 && (!thresh || !mask))) return MJX_EINVAL;
    if (k == 0) return MJX_OK;
    k_mt_refresh_masks<<<1, 1024, 0, as_stream(stream)>>>(state, left_next, n, k, thresh, mask);
    MJX_LAUNCH_CHECK("k_mt_refresh_masks");
    return MJX_OK;
}
