// The reference's per-iteration torch.rand(n) (code/HPR_pytorch_RRG.py:142, torch's
// CPU MT19937) on the device, in parallel: MT19937 jump-ahead.
//
// A batch of k HPR iterations consumes E = 2nk consecutive 32-bit outputs of one
// MT19937 stream.  mjx_hpr_refresh_masks (mjx_hpr.hip) walks them with one
// workgroup, 624 words per twist, ~0.9 us per block: 4.6 ms per 16 iterations at
// n = 1e5.  Here the E words are split into G chunks of L = 624 c words, chunk j
// on workgroup j, which first jumps the batch-start state ahead by j L - 1 words.
//
// Jump-ahead (the standard F2-linear method): the state is the 19937-bit window
// w_m = (upper bit of x_m, x_{m+1}, ..., x_{m+623}) of the untempered sequence x,
// and w_{m+1} = A w_m for a linear map A whose characteristic polynomial P has
// degree 19937.  With r(z) = z^J mod P(z) = sum_i r_i z^i (Cayley-Hamilton),
// w_J = sum_i r_i A^i w_0 = sum_i r_i w_i, i.e. word q of the jumped window is the
// XOR of x_{i+q} over the set bits i of r: one pass over the first 19937 + 623
// words of the stream, which the workgroup generates in LDS by ordinary twists.
// P is found once per process by Berlekamp-Massey on 2 x 19937 bits of the
// sequence, and the G-1 polynomials z^{jL-1} mod P of one (n, k) are tabulated
// once on the host (mjx_mt_jump_table) and read by every batch.
//
// Jumping to j L - 1 rather than j L: the window's word 0 carries only its upper
// bit, so the jumped window's words 1..623 are x_{jL}..x_{jL+622} (full), and
// x_{jL+623} is the twist of words 0, 1 and 397 of the window.
#include "mjx_common.h"

#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

namespace mjx {
namespace mtj {

constexpr int kN = 624, kM = 397;
constexpr int kDeg = 19937;                     // degree of P
constexpr int kPW = (kDeg + 1 + 63) / 64;       // 312 words of a polynomial of degree <= 19937
constexpr int kStream = kDeg + kN;              // stream words a jump reads: 19937 + 623 (+1 spare)

// ---------------------------------------------------------------- host: GF(2) polynomials
static uint32_t twist_word(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// characteristic polynomial of the one-word state map: bits 0..19937 (bit i = coefficient of z^i)
static std::vector<uint64_t> charpoly() {
    // sequence: the top bit of consecutive untempered words from a seeded state
    const int NB = 2 * kDeg;
    std::vector<uint32_t> x(NB + kN);
    x[0] = 5489u;
    for (int i = 1; i < kN; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
    for (int m = 0; m + kN < (int)x.size(); ++m) x[m + kN] = twist_word(x[m], x[m + 1], x[m + kM]);
    std::vector<uint8_t> s(NB);
    for (int i = 0; i < NB; ++i) s[i] = (uint8_t)(x[i + 1] >> 31);   // word 1 on: every bit a state bit
    // Berlekamp-Massey over GF(2): C(z) = 1 + c_1 z + ... + c_L z^L with
    // s_i = sum_{j=1..L} c_j s_{i-j}
    const int W = (NB + 64) / 64 + 1;
    std::vector<uint64_t> C(W, 0), B(W, 0), Tm(W, 0);
    C[0] = B[0] = 1;
    // the sequence reversed and bit-packed, R bit t = s[NB-1-t]: s_{i-j} for
    // j = 0..L is the bit run of R starting at NB-1-i, so the discrepancy is the
    // parity of (C AND that run), word-parallel
    std::vector<uint64_t> R(W + 1, 0);
    for (int t = 0; t < NB; ++t)
        if (s[NB - 1 - t]) R[t >> 6] |= 1ull << (t & 63);
    int L = 0, m = 1;
    for (int i = 0; i < NB; ++i) {
        const int o = NB - 1 - i, ow = o >> 6, ob = o & 63;
        uint64_t acc = 0;
        for (int q = 0; q <= (L >> 6) && ow + q < W; ++q) {
            uint64_t run = R[ow + q] >> ob;
            if (ob) run |= R[ow + q + 1] << (64 - ob);
            acc ^= C[q] & run;
        }
        const int d = __builtin_popcountll(acc) & 1;   // c_0 = 1 contributes s_i
        if (!d) {
            ++m;
            continue;
        }
        // C ^= B << m
        auto add_shift = [&](std::vector<uint64_t>& dst) {
            const int ws = m >> 6, bs = m & 63;
            for (int q = W - 1; q >= ws; --q) {
                uint64_t v = B[q - ws] << bs;
                if (bs && q - ws - 1 >= 0) v |= B[q - ws - 1] >> (64 - bs);
                dst[q] ^= v;
            }
        };
        if (2 * L <= i) {
            Tm = C;
            add_shift(C);
            L = i + 1 - L;
            B = Tm;
            m = 1;
        } else {
            add_shift(C);
            ++m;
        }
    }
    if (L != kDeg) return {};
    // P(z) = z^L C(1/z): coefficient of z^i is c_{L-i}
    std::vector<uint64_t> P(kPW, 0);
    for (int i = 0; i <= kDeg; ++i) {
        const int j = kDeg - i;
        if ((C[j >> 6] >> (j & 63)) & 1) P[i >> 6] |= 1ull << (i & 63);
    }
    return P;
}

static const std::vector<uint64_t>& charpoly_cached() {
    static std::once_flag once;
    static std::vector<uint64_t> P;
    std::call_once(once, [] { P = charpoly(); });
    return P;
}

// r <- r * z^sh mod P, r of degree < kDeg (kPW words); Ps[b] = P << b (b < 64)
static void mul_zpow_mod(std::vector<uint64_t>& r, int64_t sh, const std::vector<std::vector<uint64_t>>& Ps) {
    while (sh > 0) {
        const int step = (int)(sh < 4096 ? sh : 4096);
        sh -= step;
        const int ws = step >> 6, bs = step & 63;
        const int NW = kPW + ws + 2;
        std::vector<uint64_t> t(NW, 0);
        for (int q = 0; q < kPW; ++q) {
            t[q + ws] ^= r[q] << bs;
            if (bs) t[q + ws + 1] ^= r[q] >> (64 - bs);
        }
        // clear bits >= kDeg from the top
        for (int64_t b = (int64_t)NW * 64 - 1; b >= kDeg; --b) {
            if (!((t[b >> 6] >> (b & 63)) & 1)) continue;
            const int64_t s = b - kDeg;              // XOR P << s
            const int w0 = (int)(s >> 6), bb = (int)(s & 63);
            const std::vector<uint64_t>& p = Ps[bb];
            for (int q = 0; q < (int)p.size() && q + w0 < NW; ++q) t[q + w0] ^= p[q];
        }
        for (int q = 0; q < kPW; ++q) r[q] = t[q];
    }
}

struct Geo {
    int64_t E;      // words per batch
    int64_t L;      // words per chunk (multiple of 624)
    int G;          // chunks (workgroups)
};

static bool geometry(int64_t n, int k, int G, Geo* g) {
    if (n < 1 || k < 1 || G < 1 || G > 4096) return false;
    g->E = 2 * n * (int64_t)k;
    // the first word read may sit anywhere in the batch-start block: cover E + 624
    const int64_t blocks = (g->E + kN + kN - 1) / kN + 1;
    const int64_t c = (blocks + G - 1) / G;
    g->L = c * kN;
    g->G = (int)((blocks + c - 1) / c);
    return true;
}

// ---------------------------------------------------------------- device
__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t twist1(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// dst[0..624) = the 624 words after the window src[0..624) (dst may not alias src);
// three dependency phases, one barrier each
__device__ __forceinline__ void twist_block(const uint32_t* src, uint32_t* dst, int tid) {
    if (tid < 227) dst[tid] = twist1(src[tid], src[tid + 1], src[tid + kM]);
    __syncthreads();
    if (tid < 227) dst[tid + 227] = twist1(src[tid + 227], src[tid + 228], dst[tid]);
    __syncthreads();
    if (tid < 170) {
        const int i = tid + 454;
        dst[i] = twist1(src[i], (i + 1 < kN) ? src[i + 1] : dst[0], dst[i - 227]);
    }
    __syncthreads();
}

constexpr int kThreads = 640;

// Workgroup j: words [jL, (j+1)L) of the batch, counted from word 0 of the
// batch-start buffer (state_in; the first word read is 625 - left).  Pair p
// (words first + 2p, first + 2p + 1) is uniform p = iteration p / n, node p % n.
__global__ void __launch_bounds__(kThreads) k_mt_refresh_jump(const uint32_t* __restrict__ state_in,
                                                              const int32_t* __restrict__ ln_in,
                                                              uint32_t* __restrict__ state_out,
                                                              int32_t* __restrict__ ln_out, int64_t n, int64_t E,
                                                              int64_t L, const uint64_t* __restrict__ table,
                                                              const double* __restrict__ thresh,
                                                              uint8_t* __restrict__ mask) {
    extern __shared__ __align__(16) uint32_t smem[];
    uint32_t* S = smem;                       // the stream x_0 .. x_{kStream-1} (jumping workgroups)
    uint32_t* blk = smem + kStream + 1;       // two 624-word blocks, ping-pong
    const int tid = threadIdx.x;
    const int j = blockIdx.x;
    const int64_t first = kN + 1 - ln_in[0];  // word index of the first output of the batch
    const int64_t last = first + E;           // one past the last
    const int64_t w0 = (int64_t)j * L;
    const int64_t w1 = w0 + L;
    if (w0 >= last || w1 <= first) return;   // nothing of the batch here (uniform: whole workgroup)
    uint32_t* cur = blk;
    uint32_t* nxt = blk + kN;
    if (j == 0) {
        for (int q = tid; q < kN; q += kThreads) cur[q] = state_in[q];
        __syncthreads();
    } else {
        for (int q = tid; q < kN; q += kThreads) S[q] = state_in[q];
        __syncthreads();
        for (int b = kN; b < kStream; b += kN) {
            // S[b .. b+624) from S[b-624 .. b): the last block may run past kStream;
            // the buffer holds kStream + 1 + 2*624 words, so it spills into blk only
            twist_block(S + b - kN, S + b, tid);
        }
        // the jumped window (offset jL - 1): acc[q] = XOR over set bits i of the
        // table polynomial of S[i + q]
        const uint64_t* poly = table + (int64_t)(j - 1) * kPW;
        uint32_t acc = 0;
        if (tid < kN) {
            for (int wi = 0; wi < kPW; ++wi) {
                uint64_t cw = poly[wi];
                const uint32_t* sp = S + wi * 64 + tid;
                while (cw) {
                    // four set bits per round: four LDS reads in flight
                    const int b0 = __builtin_ctzll(cw);
                    cw &= cw - 1;
                    uint32_t v = sp[b0];
                    if (cw) {
                        const int b1 = __builtin_ctzll(cw);
                        cw &= cw - 1;
                        v ^= sp[b1];
                        if (cw) {
                            const int b2 = __builtin_ctzll(cw);
                            cw &= cw - 1;
                            v ^= sp[b2];
                            if (cw) {
                                const int b3 = __builtin_ctzll(cw);
                                cw &= cw - 1;
                                v ^= sp[b3];
                            }
                        }
                    }
                    acc ^= v;
                }
            }
        }
        __syncthreads();                      // every lane has read S: reuse its head
        if (tid < kN) S[tid] = acc;
        __syncthreads();
        // block at jL: words 1..623 of the window, then the twist of words 0, 1, 397
        for (int q = tid; q < kN - 1; q += kThreads) cur[q] = S[q + 1];
        if (tid == 0) cur[kN - 1] = twist1(S[0], S[1], S[kM]);
        __syncthreads();
    }
    // walk the chunk's blocks; a pair whose low word is the next block's first
    // reads it from the twisted next block
    for (int64_t b0 = w0; b0 < w1 && b0 < last; b0 += kN) {
        twist_block(cur, nxt, tid);
        const int64_t lo = b0 > first ? b0 : first;
        const int64_t hi = (b0 + kN < last) ? b0 + kN : last;
        // pairs whose high word lies in [lo, hi): high word first + 2p
        const int64_t p0 = (lo - first + 1) >> 1;            // first pair starting at or after lo
        const int64_t p1 = (hi - first + 1) >> 1;            // pairs starting before hi
        for (int64_t p = p0 + tid; p < p1; p += kThreads) {
            const int64_t wh = first + 2 * p - b0;           // in [0, 624)
            const uint32_t yh = temper(cur[wh]);
            const uint32_t yl = temper(wh + 1 < kN ? cur[wh + 1] : nxt[0]);
            const uint64_t r = ((uint64_t)yh << 32) | yl;
            const double u = (double)(r & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
            const int64_t it = p / n;
            mask[p] = u < thresh[it] ? 1 : 0;
        }
        // the engine's state after the batch: the block holding the last word read
        if (last - 1 >= b0 && last - 1 < b0 + kN) {
            for (int q = tid; q < kN; q += kThreads) state_out[q] = cur[q];
            if (tid == 0) {
                const int pos = (int)(last - b0);             // words of this block read
                ln_out[0] = kN + 1 - pos;
                ln_out[1] = pos;
            }
        }
        __syncthreads();
        uint32_t* t = cur;
        cur = nxt;
        nxt = t;
    }
}

}  // namespace mtj
}  // namespace mjx

using namespace mjx;

extern "C" int mjx_mt_jump_geometry(int64_t n, int k, int G, int64_t* L, int* G_used) {
    mtj::Geo g;
    if (!mtj::geometry(n, k, G, &g)) return MJX_EINVAL;
    if (L) *L = g.L;
    if (G_used) *G_used = g.G;
    return MJX_OK;
}

extern "C" int64_t mjx_mt_jump_table_words(int64_t n, int k, int G) {
    mtj::Geo g;
    if (!mtj::geometry(n, k, G, &g)) return -1;
    return (int64_t)(g.G > 1 ? g.G - 1 : 0) * mtj::kPW;
}

extern "C" int mjx_mt_jump_table(int64_t n, int k, int G, uint64_t* table) {
    mtj::Geo g;
    if (!mtj::geometry(n, k, G, &g) || (!table && g.G > 1)) return MJX_EINVAL;
    if (g.G <= 1) return MJX_OK;
    const std::vector<uint64_t>& P = mtj::charpoly_cached();
    if (P.empty()) return MJX_ERANGE;      // Berlekamp-Massey did not find degree 19937
    // P << b for b < 64
    std::vector<std::vector<uint64_t>> Ps(64, std::vector<uint64_t>(mtj::kPW + 1, 0));
    for (int b = 0; b < 64; ++b)
        for (int q = 0; q < mtj::kPW; ++q) {
            Ps[b][q] ^= P[q] << b;
            if (b) Ps[b][q + 1] ^= P[q] >> (64 - b);
        }
    // r_1 = z^{L-1}, r_{j+1} = r_j z^L
    std::vector<uint64_t> r(mtj::kPW, 0);
    r[0] = 1;
    mtj::mul_zpow_mod(r, g.L - 1, Ps);
    for (int j = 1; j < g.G; ++j) {
        memcpy(table + (int64_t)(j - 1) * mtj::kPW, r.data(), sizeof(uint64_t) * mtj::kPW);
        if (j + 1 < g.G) mtj::mul_zpow_mod(r, g.L, Ps);
    }
    return MJX_OK;
}

extern "C" int mjx_hpr_refresh_masks_jump(const uint32_t* state_in, const int32_t* ln_in, uint32_t* state_out,
                                          int32_t* ln_out, int64_t n, int k, int G, const uint64_t* table,
                                          const double* thresh, uint8_t* mask, void* stream) {
    if (n < 1 || k < 0 || !state_in || !ln_in || !state_out || !ln_out || state_in == state_out ||
        (k > 0 && (!thresh || !mask)))
        return MJX_EINVAL;
    if (k == 0) return MJX_OK;
    mtj::Geo g;
    if (!mtj::geometry(n, k, G, &g)) return MJX_EINVAL;
    if (g.G > 1 && !table) return MJX_EINVAL;
    const size_t lds = sizeof(uint32_t) * (size_t)(mtj::kStream + 1 + 2 * mtj::kN);
    MJX_HIP(hipFuncSetAttribute((const void*)mtj::k_mt_refresh_jump, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds),
            "mt_jump lds");
    mtj::k_mt_refresh_jump<<<(unsigned)g.G, mtj::kThreads, lds, as_stream(stream)>>>(
        state_in, ln_in, state_out, ln_out, n, g.E, g.L, table, thresh, mask);
    MJX_LAUNCH_CHECK("k_mt_refresh_jump");
    return MJX_OK;
}
