// Device graph generation and checks for the majority dynamics.
//
// Random d-regular graphs.  The reference draws them with
// networkx.random_regular_graph (code/SA_RRG.py:59, code/HPR_pytorch_RRG.py:261);
// parity with it is distributional, not bit-exact.  Configuration model: the
// n*d stubs (stub v*d+k = slot k of node v) are paired through a keyed
// pseudorandom permutation pi of [0, n*d) -- stub pi(2j) with stub pi(2j+1).
// The partner of stub s is pi(pi^-1(s) ^ 1), a pure function of (seed, s), so
// any row range of the ELL adjacency adj[v*d+k] = partner(v*d+k)/d is generated
// independently: each rank of a node-range partition builds exactly its own
// rows, with no communication.  Self-loops and multi-edges (O(d^2) of them in
// expectation, independent of n) are found by a scan of all rows on the device
// and removed by deterministic double-edge switches on the host; every rank
// computes the same switches from the same scan.
#include "mjx_common.h"
#include <algorithm>
#include <cstdlib>
#include <unordered_map>
#include <utility>
#include <vector>
#include <hipcub/hipcub.hpp>

namespace mjx {
namespace gen {

constexpr int kRounds = 4;
constexpr int kMaxD = 16;

// A keyed pseudorandom permutation of [0, M): an alternating (unbalanced)
// Feistel network on [0, 2^B), B = ceil(log2 M) split into a high part of a
// and a low part of B - a bits whose widths swap every round (an even number
// of rounds restores them), restricted to [0, M) by cycle walking (2^B < 2M:
// under two steps on average).
struct Perm {
    uint64_t M;        // domain [0, M)
    int a, b;          // widths of the high and low parts, a + b = B
    uint64_t dmul;     // ceil(2^64 / d) for the stub -> node division (0: d = 1)
    uint32_t key[kRounds];
};

__host__ __device__ inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ inline uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__host__ __device__ inline uint32_t wmask(int w) { return (w >= 32) ? 0xffffffffu : ((1u << w) - 1u); }

__host__ __device__ inline uint64_t feistel(const Perm& P, uint64_t v) {
    uint32_t hi = (uint32_t)(v >> P.b), lo = (uint32_t)v & wmask(P.b);
    int wh = P.a, wl = P.b;
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t t = hi ^ (mix32(lo ^ P.key[r]) & wmask(wh));
        hi = lo;
        lo = t;
        const int x = wh;
        wh = wl;
        wl = x;
    }
    return ((uint64_t)hi << wl) | lo;
}

__host__ __device__ inline uint64_t feistel_inv(const Perm& P, uint64_t v) {
    uint32_t hi = (uint32_t)(v >> P.b), lo = (uint32_t)v & wmask(P.b);
    int wh = P.a, wl = P.b;
    for (int r = kRounds - 1; r >= 0; --r) {
        const uint32_t ol = hi, oh = lo ^ (mix32(ol ^ P.key[r]) & wmask(wl));
        hi = oh;
        lo = ol;
        const int x = wh;
        wh = wl;
        wl = x;
    }
    return ((uint64_t)hi << wl) | lo;
}

// cycle walking restricts the permutation to [0, M)
__host__ __device__ inline uint64_t perm_fwd(const Perm& P, uint64_t v) {
    uint64_t x = feistel(P, v);
    while (x >= P.M) x = feistel(P, x);
    return x;
}

__host__ __device__ inline uint64_t perm_inv(const Perm& P, uint64_t v) {
    uint64_t x = feistel_inv(P, v);
    while (x >= P.M) x = feistel_inv(P, x);
    return x;
}

__host__ __device__ inline uint64_t partner(const Perm& P, uint64_t s) { return perm_fwd(P, perm_inv(P, s) ^ 1ull); }

// stub -> node: s / d exactly for s < 2^36 (s * ceil(2^64/d) / 2^64 is off by
// less than s / 2^64 < 1/d)
__host__ __device__ inline int64_t stub_node(const Perm& P, uint64_t s) {
#ifdef __HIP_DEVICE_COMPILE__
    return P.dmul ? (int64_t)__umul64hi(s, P.dmul) : (int64_t)s;
#else
    return P.dmul ? (int64_t)(((unsigned __int128)s * P.dmul) >> 64) : (int64_t)s;
#endif
}

static Perm make_perm(uint64_t M, uint64_t seed, int d) {
    Perm P;
    P.M = M;
    int bits = 2;
    while ((1ull << bits) < M) ++bits;
    P.a = bits / 2;
    P.b = bits - P.a;
    P.dmul = (d > 1) ? (~0ull / (uint64_t)d) + 1ull : 0ull;
    uint64_t s = seed ^ 0x6a09e667f3bcc909ull;
    for (int r = 0; r < kRounds; ++r) P.key[r] = (uint32_t)splitmix64(s);
    return P;
}

// Rows of every node are computed (the defect scan needs all of them); rows in
// [lo, hi) are stored.  defects[0] = count, then (stub, partner stub) pairs.
__global__ void __launch_bounds__(256) k_rrg_rows(Perm P, int64_t n, int d, int64_t lo, int64_t hi,
                                                  int32_t* __restrict__ adj, unsigned long long* __restrict__ defects,
                                                  int64_t cap) {
    __shared__ int32_t ws[kMaxD * 256];          // the row's neighbours
    const int tid = threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t v = (int64_t)blockIdx.x * 256 + tid; v < n; v += stride) {
        const bool mine = v >= lo && v < hi;
        for (int k = 0; k < d; ++k) {
            const uint64_t s = (uint64_t)v * d + k, p = partner(P, s);
            const int32_t w = (int32_t)stub_node(P, p);
            ws[k * 256 + tid] = w;
            if (mine) adj[(v - lo) * d + k] = w;
            if (w == v && s < p) {                         // a self-loop, recorded once
                const unsigned long long q = atomicAdd(defects, 1ull);
                if ((int64_t)q < cap) {
                    defects[1 + 2 * q] = s;
                    defects[2 + 2 * q] = p;
                }
            }
        }
        for (int k = 1; k < d; ++k) {
            const int32_t w = ws[k * 256 + tid];
            if (w == v || v >= w) continue;                // a repeated neighbour, recorded from the lower end
            bool bad = false;
            for (int j = 0; j < k; ++j) bad |= ws[j * 256 + tid] == w;
            if (bad) {
                const uint64_t s = (uint64_t)v * d + k;
                const unsigned long long q = atomicAdd(defects, 1ull);
                if ((int64_t)q < cap) {
                    defects[1 + 2 * q] = s;
                    defects[2 + 2 * q] = partner(P, s);     // (rare: recomputed)
                }
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_rrg_patch(int32_t* __restrict__ adj, int64_t stub_lo,
                                                   const long long* __restrict__ patch, int64_t np) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < np) adj[patch[2 * i] - stub_lo] = (int32_t)patch[2 * i + 1];
}

// counts[0] self-loops, [1] entries repeated within their row, [2] entries
// whose reverse multiplicity differs (or that are out of range)
__global__ void __launch_bounds__(256) k_check_ell(const int32_t* __restrict__ adj, int64_t n, int d,
                                                   unsigned long long* __restrict__ counts) {
    unsigned long long c0 = 0, c1 = 0, c2 = 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n; v += stride) {
        for (int k = 0; k < d; ++k) {
            const int64_t w = adj[v * d + k];
            if (w < 0 || w >= n) {
                ++c2;
                continue;
            }
            if (w == v) ++c0;
            int mult = 0, back = 0;
            for (int j = 0; j < d; ++j) {
                mult += adj[v * d + j] == w;
                back += adj[w * d + j] == v;
            }
            if (mult > 1) ++c1;
            if (back != mult) ++c2;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        c0 += __shfl_xor(c0, off, 64);
        c1 += __shfl_xor(c1, off, 64);
        c2 += __shfl_xor(c2, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (c0) atomicAdd(&counts[0], c0);
        if (c1) atomicAdd(&counts[1], c1);
        if (c2) atomicAdd(&counts[2], c2);
    }
}

// Host side of the repair: the pairing with the switches applied so far.
struct Pairing {
    const Perm& P;
    uint64_t d;
    std::unordered_map<uint64_t, uint64_t> ov;
    uint64_t part(uint64_t s) const {
        auto it = ov.find(s);
        return it == ov.end() ? partner(P, s) : it->second;
    }
    int64_t node(uint64_t s) const { return stub_node(P, s); }
    int mult(int64_t u, int64_t w) const {
        int m = 0;
        for (uint64_t k = 0; k < d; ++k) m += node(part((uint64_t)u * d + k)) == w;
        return m;
    }
};

// Deterministic double-edge switches (u,v),(x,y) -> (u,x),(v,y) that remove every
// recorded self-loop and repeated edge without creating new ones.
static int repair(Pairing& R, uint64_t seed, std::vector<std::pair<uint64_t, uint64_t>>& defects, int64_t* nsw) {
    std::sort(defects.begin(), defects.end());
    uint64_t rs = seed ^ 0xbb67ae8584caa73bull;
    int64_t switches = 0;
    for (const auto& ab : defects) {
        const uint64_t a = ab.first, b = ab.second;
        if (R.part(a) != b) continue;                 // this pair was already switched away
        const int64_t u = R.node(a), v = R.node(b);
        if (u != v && R.mult(u, v) < 2) continue;     // no longer a defect
        bool done = false;
        for (int attempt = 0; attempt < (1 << 20) && !done; ++attempt) {
            uint64_t x = splitmix64(rs) % R.P.M;
            uint64_t y = R.part(x);
            if (x == a || x == b || y == a || y == b) continue;
            if (splitmix64(rs) & 1ull) std::swap(x, y);
            const int64_t nx = R.node(x), ny = R.node(y);
            if (nx == u || ny == v) continue;                                  // new self-loop
            if (std::min(u, nx) == std::min(v, ny) && std::max(u, nx) == std::max(v, ny)) continue;
            if (R.mult(u, nx) > 0 || R.mult(v, ny) > 0) continue;              // new repeated edge
            R.ov[a] = x;
            R.ov[x] = a;
            R.ov[b] = y;
            R.ov[y] = b;
            ++switches;
            done = true;
        }
        if (!done) return MJX_ERANGE;
    }
    *nsw = switches;
    return MJX_OK;
}

}  // namespace gen
}  // namespace mjx

using namespace mjx;
using namespace mjx::gen;

extern "C" int64_t mjx_rrg_partner_host(int64_t n, int d, uint64_t seed, int64_t stub) {
    if (n < 2 || d < 1 || stub < 0 || stub >= n * (int64_t)d || (n * (int64_t)d) % 2) return -1;
    const Perm P = make_perm((uint64_t)n * (uint64_t)d, seed, d);
    return (int64_t)partner(P, (uint64_t)stub);
}

extern "C" int mjx_rrg_generate(int64_t n, int d, uint64_t seed, int64_t row_lo, int64_t row_hi, int32_t* adj,
                                uint64_t* work, int64_t work_words, int64_t* n_switches, void* stream) {
    if (n < 2 || d < 1 || d >= n || (n * (int64_t)d) % 2 || row_lo < 0 || row_hi > n || row_lo > row_hi)
        return MJX_EINVAL;
    if (d > kMaxD || n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if ((row_hi > row_lo && !adj) || !work || work_words < 3) return MJX_EINVAL;
    const int64_t cap = (work_words - 1) / 2;
    const Perm P = make_perm((uint64_t)n * (uint64_t)d, seed, d);
    hipStream_t st = as_stream(stream);
    MJX_HIP(hipMemsetAsync(work, 0, sizeof(uint64_t), st), "rrg memset");
    k_rrg_rows<<<grid_for(n, 8), 256, 0, st>>>(P, n, d, row_lo, row_hi, adj, (unsigned long long*)work, cap);
    MJX_LAUNCH_CHECK("k_rrg_rows");
    uint64_t cnt = 0;
    MJX_HIP(hipMemcpyAsync(&cnt, work, sizeof(uint64_t), hipMemcpyDeviceToHost, st), "rrg count");
    MJX_HIP(hipStreamSynchronize(st), "rrg sync");
    if ((int64_t)cnt > cap) return MJX_ERANGE;
    std::vector<uint64_t> raw(2 * cnt);
    if (cnt) {
        MJX_HIP(hipMemcpyAsync(raw.data(), work + 1, 16 * cnt, hipMemcpyDeviceToHost, st), "rrg defects");
        MJX_HIP(hipStreamSynchronize(st), "rrg sync");
    }
    std::vector<std::pair<uint64_t, uint64_t>> defects;
    for (uint64_t q = 0; q < cnt; ++q) defects.emplace_back(raw[2 * q], raw[2 * q + 1]);
    Pairing R{P, (uint64_t)d, {}};
    int64_t nsw = 0;
    int rc = repair(R, seed, defects, &nsw);
    if (rc) return rc;
    std::vector<long long> patch;
    const uint64_t s_lo = (uint64_t)row_lo * d, s_hi = (uint64_t)row_hi * d;
    for (const auto& kv : R.ov)
        if (kv.first >= s_lo && kv.first < s_hi) {
            patch.push_back((long long)kv.first);
            patch.push_back((long long)(kv.second / (uint64_t)d));
        }
    if (!patch.empty()) {
        if ((int64_t)patch.size() > work_words) return MJX_ERANGE;
        MJX_HIP(hipMemcpyAsync(work, patch.data(), patch.size() * sizeof(long long), hipMemcpyHostToDevice, st),
                "rrg patch upload");
        const int64_t np = (int64_t)patch.size() / 2;
        k_rrg_patch<<<(unsigned)((np + 255) / 256), 256, 0, st>>>(adj, (int64_t)s_lo, (const long long*)work, np);
        MJX_LAUNCH_CHECK("k_rrg_patch");
        MJX_HIP(hipStreamSynchronize(st), "rrg sync");
    }
    if (n_switches) *n_switches = nsw;
    return MJX_OK;
}

extern "C" int mjx_graph_check_ell(const int32_t* adj, int64_t n, int d, unsigned long long* counts, void* stream) {
    if (n < 0 || d < 0 || !counts || (n > 0 && d > 0 && !adj)) return MJX_EINVAL;
    if (n == 0 || d == 0) return MJX_OK;
    k_check_ell<<<grid_for(n, 8), 256, 0, as_stream(stream)>>>(adj, n, d, counts);
    MJX_LAUNCH_CHECK("k_check_ell");
    return MJX_OK;
}

// ===========================================================================
// Source-binned (propagation-blocking) sweep of a node-packed state (one
// replica, huge n: config C5).
//
// The gather sweep reads s[u] for n*d random u per sweep: at N=1e9, d=6 every
// 4-byte gather costs a whole cache line of a 125 MB state, so it runs at the
// random line rate (98-109 ms per sweep on one MI355X).  Here the rows*d
// (destination v, source u) slots of a rank's rows are binned once, in a static
// plan, by source block b = u >> kSrcShift (1M nodes = 128 KB of state bits,
// staged in LDS) and destination tile t = (v - lo) >> kTileShift (64K nodes,
// byte counters in LDS).  Segment (b, t) = the slots with source in block b and
// destination in tile t.  A sweep is two streaming kernels:
//   phase 1 (k_bin_msg, workgroups per source block): stage the block's state
//     bits in LDS, stream the block's source offsets (phase-1 order: b-major,
//     t inside) and write one message bit per slot;
//   phase 2 (k_bin_apply_flat, one workgroup per destination tile): stream the
//     tile's 16-bit destination offsets (phase-2 order: t-major, b inside) and
//     the segments' message bytes, count +1 neighbours in LDS (byte counters),
//     then apply the majority rule with always-stay ties (code/SA_RRG.py:19-20)
//     against the node's own bit.
// Segments start on 8-slot boundaries in BOTH orders, so the eight message bits
// of an aligned 8-slot piece of a segment are one byte of msg.
// Slot i of segment (b, t) is slot i in both orders, so the phases agree
// without a per-slot index.  Algorithmic traffic per slot: 2.5 B of source
// offset (20 bits: a 16-bit low part and a 4-bit high part) + 2 B of
// destination offset + 2/8 B of message bit (written, read back), all streamed,
// instead of one random line per slot.
//
// Plan (sizes from mjx_binned_plan_shape):
//   src_lo uint16[src_len/512*640]  the phase-1 stream, in 512-slot chunks
//                            (segment starts padded to 8 slots, block starts to
//                            512): per chunk 512 entries = each slot's source
//                            offset (20 bits within its block) >> 4, i.e. the
//                            index of the 16-bit state word that holds its bit,
//                            then 128 entries = the bit within that word
//                            (offset & 15) of slots 4i..4i+3 in entry i (nibble
//                            k = slot 4i+k): one contiguous 1280-B piece;
//   src_hi                   unused (size 0; may be NULL);
//   off   uint16[off_len] phase-2 order; segment starts padded to 8 slots;
//   index int64           blk[K+1]  phase-1 padded block starts |
//                         p1T[S]    phase-1 start of segment (b,t), at t*K+b |
//                         p2[S+1]   phase-2 padded start of segment (b,t) at
//                                   t*K+b, its pad count in the low 3 bits.
// ===========================================================================
namespace mjx {
namespace binned {

constexpr int kSrcShift = 20;
constexpr int64_t kSrc = 1ll << kSrcShift;
constexpr int kSrcWords = (int)(kSrc >> 5);     // uint32 words of one block's state bits (128 KB)
constexpr int kTileShift = 16;
constexpr int64_t kTile = 1ll << kTileShift;
constexpr int kCntWords = (int)(kTile >> 2);    // byte counters, four per LDS word (64 KB)
constexpr int kMsgThreads = 1024;
constexpr int kApplyThreads = 1024;
constexpr int kMsgSplitMax = 4;                 // phase-1 workgroups per source block (all rows of n)
constexpr int64_t kScanScratch = 64ll << 20;
constexpr int64_t kMaxBlocks = 16384;           // histogram of blocks in 64 KB of LDS

struct Shape {
    int64_t K, T, S, slots, src_len, off_len, index_len, msg_words, work_bytes;
};

inline int64_t align256(int64_t x) { return (x + 255) & ~255ll; }
constexpr int kChunk = 512;                     // phase-1 slots per wave load: 8 a lane; block starts aligned to it
__host__ __device__ inline int64_t align_chunk(int64_t x) { return (x + kChunk - 1) & ~(int64_t)(kChunk - 1); }

inline Shape shape(int64_t n, int d, int64_t rows) {
    Shape s;
    s.K = (n + kSrc - 1) >> kSrcShift;
    s.T = (rows + kTile - 1) >> kTileShift;
    s.S = s.K * s.T;
    s.slots = rows * d;
    s.src_len = align_chunk(s.slots + 7 * s.S) + kChunk * s.K;   // segments padded to 8 slots, blocks to kChunk
    s.off_len = s.slots + 8 * s.S + 8;
    s.index_len = (s.K + 1) + s.S + (s.S + 1);
    s.msg_words = s.src_len / 64 + 2;
    s.work_bytes = align256(4 * s.S) + align256(8 * s.S) + kScanScratch;
    return s;
}


// ---- plan construction (setup, once per graph) ------------------------------

// per-tile histogram over source blocks: cntB[b*T+t] (b-major) and the padded
// count into p2[t*K+b] (t-major, scanned afterwards)
__global__ void __launch_bounds__(256) k_bin_count(const int32_t* __restrict__ adj, int64_t rows, int d, int64_t n,
                                                   int64_t K, int64_t T, uint32_t* __restrict__ cntB,
                                                   long long* __restrict__ p2) {
    extern __shared__ unsigned hist[];
    const int64_t t = blockIdx.x;
    for (int64_t b = threadIdx.x; b < K; b += 256) hist[b] = 0;
    __syncthreads();
    const int64_t r1 = ((t + 1) * kTile < rows) ? (t + 1) * kTile : rows;
    for (int64_t q = t * kTile * d + threadIdx.x; q < r1 * d; q += 256) {
        const int32_t u = adj[q];
        if (u >= 0 && u < n) atomicAdd(&hist[u >> kSrcShift], 1u);
    }
    __syncthreads();
    for (int64_t b = threadIdx.x; b < K; b += 256) {
        const unsigned c = hist[b];
        cntB[b * T + t] = c;
        p2[t * K + b] = (long long)((c + 7u) & ~7u);
    }
}

// tag every phase-2 start with its segment's pad count (low 3 bits)
__global__ void k_bin_tag(const uint32_t* __restrict__ cntB, int64_t K, int64_t T, long long* __restrict__ p2) {
    const int64_t S = K * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = i / K, b = i - t * K;
        const unsigned c = cntB[b * T + t];
        p2[i] |= (long long)(((c + 7u) & ~7u) - c);
    }
}

// per source block: exclusive scan of its segment sizes over t; padded total
__global__ void __launch_bounds__(256) k_bin_blockscan(const uint32_t* __restrict__ cntB, int64_t T,
                                                       long long* __restrict__ p1, long long* __restrict__ blk) {
    __shared__ long long sh[256];
    const int64_t b = blockIdx.x;
    long long carry = 0;
    for (int64_t t0 = 0; t0 < T; t0 += 256) {
        const int64_t t = t0 + threadIdx.x;
        const long long x = (t < T) ? (long long)((cntB[b * T + t] + 7u) & ~7u) : 0;   // 8-slot aligned segments
        sh[threadIdx.x] = x;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const long long y = (threadIdx.x >= (unsigned)o) ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += y;
            __syncthreads();
        }
        if (t < T) p1[b * T + t] = carry + sh[threadIdx.x] - x;
        carry += sh[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) blk[b] = align_chunk(carry);
}

// absolute phase-1 starts (b-major, for the fill) and their t-major copy
__global__ void k_bin_finish(long long* __restrict__ p1, const long long* __restrict__ blk, int64_t K, int64_t T,
                             long long* __restrict__ p1T) {
    const int64_t S = K * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / T, t = i - b * T;
        const long long v = p1[i] + blk[b];
        p1[i] = v;
        p1T[t * K + b] = v;
    }
}

// the phase-1 stream: per 512-slot chunk 1024 B of 16-bit state-word indices
// then 256 B of 4-bit bit positions (one contiguous 1280-B piece per chunk,
// kChunkU16 entries)
constexpr int kChunkU16 = kChunk + kChunk / 4;

// Place every slot of tile t (one workgroup per tile) straight into the packed
// phase-1 stream and the phase-2 offsets.  The tile's slots are taken in
// chunks that fit the LDS; a chunk is counting-sorted by source block there
// (rank = LDS atomic, so slot order inside a segment is arbitrary: both
// layouts use the same rank), and its segment runs are written as 4-slot quads
// by consecutive lanes: a quad is four 16-bit word indices (one 8-B store), one
// 16-bit entry of four bit positions and four 16-bit destination offsets (one
// 8-B store), so no slot is scattered on its own and no int32 intermediate
// exists.  A segment's last 0-3 slots of a chunk are carried in LDS to the
// next chunk (every run starts quad-aligned); the tile's last carries and the
// segments' pad slots (zeros) are written at the end, and the last tile also
// zeroes each source block's tail up to its 512-slot chunk end.  The segment
// bases come from the t-major index (p1T, p2): one contiguous K-entry read per
// tile, kept in LDS (the per-slot reads of the b-major p1 they replace were
// ~0.77 TB of random lines at N=1e9, d=6).
constexpr int kFillThreads = 1024;
constexpr int kFillSpt = 16;                    // slots per thread per chunk (at most)
constexpr int kFillLds = 160 * 1024;

struct FillLds {
    int64_t cap, ch;                            // staging capacity and chunk slots
    int64_t bytes;
};
inline FillLds fill_lds(int64_t K) {
    FillLds f;
    // b1, b2 (8 B each), so and qo (4 B, K+1 each), 32 wave sums, carries (3 slots
    // of 6 B a segment), cc (1 B)
    const int64_t fixed = 16 * K + 8 * (K + 1) + 128 + 18 * K + K + 16;
    const int64_t cap = (kFillLds - fixed) / 6;
    int64_t ch = ((cap - 3 * K) / kFillThreads) * kFillThreads;
    if (ch > kFillSpt * kFillThreads) ch = kFillSpt * kFillThreads;
    f.ch = ch;
    f.cap = ch + 3 * K;
    f.bytes = fixed + 6 * f.cap;
    return f;
}

// exclusive scans over K <= 2048 entries by 1024 threads, two entries a
// thread: x -> xs and floor(x/4) -> ys (K+1 entries each; xs may be x: every
// thread reads its entries before the first barrier)
__device__ __forceinline__ void scan2(uint32_t* x, uint32_t* xs, uint32_t* ys, int64_t K, uint32_t* wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t i0 = 2 * (int64_t)tid;
    const uint32_t a0 = (i0 < K) ? x[i0] : 0u, a1 = (i0 + 1 < K) ? x[i0 + 1] : 0u;
    const uint32_t s = a0 + a1, q = (a0 >> 2) + (a1 >> 2);
    uint32_t is = s, iq = q;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t us = __shfl_up(is, o, 64), uq = __shfl_up(iq, o, 64);
        if (lane >= o) {
            is += us;
            iq += uq;
        }
    }
    if (lane == 63) {
        wsum[wave] = is;
        wsum[16 + wave] = iq;
    }
    __syncthreads();
    uint32_t bs = 0, bq = 0;
    for (int w = 0; w < wave; ++w) {
        bs += wsum[w];
        bq += wsum[16 + w];
    }
    const uint32_t es = bs + is - s, eq = bq + iq - q;
    if (i0 < K) {
        xs[i0] = es;
        ys[i0] = eq;
    }
    if (i0 + 1 < K) {
        xs[i0 + 1] = es + a0;
        ys[i0 + 1] = eq + (a0 >> 2);
    }
    if (tid == kFillThreads - 1) {
        xs[K] = bs + is;
        ys[K] = bq + iq;
    }
}

// one quad of phase-1 slots at global position g (a multiple of 4): the word
// indices and bit positions of four 20-bit source offsets
__device__ __forceinline__ void put_src_quad(uint16_t* __restrict__ stream, int64_t g, const uint32_t* u) {
    uint16_t* ch = stream + (g >> 9) * kChunkU16;
    const int w = (int)(g & 511);
    uint2 l;
    l.x = (u[0] >> 4) | ((u[1] >> 4) << 16);
    l.y = (u[2] >> 4) | ((u[3] >> 4) << 16);
    *reinterpret_cast<uint2*>(ch + w) = l;
    ch[kChunk + (w >> 2)] =
        (uint16_t)((u[0] & 15u) | ((u[1] & 15u) << 4) | ((u[2] & 15u) << 8) | ((u[3] & 15u) << 12));
}

__device__ __forceinline__ void put_off_quad(uint16_t* __restrict__ off, int64_t g, const uint32_t* v) {
    uint2 l;
    l.x = v[0] | (v[1] << 16);
    l.y = v[2] | (v[3] << 16);
    *reinterpret_cast<uint2*>(off + g) = l;
}

__global__ void __launch_bounds__(kFillThreads) k_bin_fill(const int32_t* __restrict__ adj, int64_t rows, int d,
                                                           int64_t n, int64_t K, int64_t T, FillLds fl,
                                                           const long long* __restrict__ p1T,
                                                           const long long* __restrict__ p2,
                                                           const uint32_t* __restrict__ cntB,
                                                           const long long* __restrict__ blk,
                                                           uint16_t* __restrict__ stream, uint16_t* __restrict__ off) {
    extern __shared__ __align__(16) unsigned char fl_raw[];
    long long* b1 = reinterpret_cast<long long*>(fl_raw);                 // next phase-1 position of (b, t)
    long long* b2 = b1 + K;                                               // next phase-2 position
    uint32_t* so = reinterpret_cast<uint32_t*>(b2 + K);                   // chunk counts, then staging starts
    uint32_t* qo = so + (K + 1);                                          // quad starts
    uint32_t* wsum = qo + (K + 1);                                        // 32 wave sums
    uint32_t* cs = wsum + 32;                                             // carried source offsets (3 a segment)
    uint32_t* ss = cs + 3 * K;                                            // staged source offsets
    uint16_t* co = reinterpret_cast<uint16_t*>(ss + fl.cap);              // carried destination offsets
    uint16_t* sv = co + 3 * K;                                            // staged destination offsets
    uint8_t* cc = reinterpret_cast<uint8_t*>(sv + fl.cap);                // carried count (0..3)
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x;
    for (int64_t b = tid; b < K; b += kFillThreads) {
        b1[b] = p1T[t * K + b];
        b2[b] = p2[t * K + b] & ~7ll;
        cc[b] = 0;
    }
    __syncthreads();
    const int64_t r1 = ((t + 1) * kTile < rows) ? (t + 1) * kTile : rows;
    const int64_t qbeg = t * kTile * d, qend = r1 * d;
    const int per = (int)(fl.ch / kFillThreads);
    for (int64_t q0 = qbeg; q0 < qend; q0 += fl.ch) {
        for (int64_t b = tid; b < K; b += kFillThreads) so[b] = cc[b];     // counts start at the carries
        __syncthreads();
        // x0 = (u & 0xfffff) | b << 20 (~0: no slot), x1 = v | rank << 16
        uint32_t x0[kFillSpt], x1[kFillSpt];
#pragma unroll
        for (int k = 0; k < kFillSpt; ++k) {
            x0[k] = 0xffffffffu;
            x1[k] = 0;
            const int64_t q = q0 + (int64_t)k * kFillThreads + tid;
            if (k < per && q < qend) {
                const int32_t u = adj[q];
                if (u >= 0 && u < n) {
                    const uint32_t b = (uint32_t)u >> kSrcShift;
                    const uint32_t r = atomicAdd(&so[b], 1u);
                    x0[k] = ((uint32_t)u & (uint32_t)(kSrc - 1)) | (b << kSrcShift);
                    x1[k] = ((uint32_t)(q - qbeg) / (uint32_t)d) | (r << 16);   // row in the tile
                }
            }
        }
        __syncthreads();
        scan2(so, so, qo, K, wsum);                  // staging starts (in place) and quad starts
        __syncthreads();
        for (int64_t b = tid; b < K; b += kFillThreads)
            for (int j = 0; j < cc[b]; ++j) {
                ss[so[b] + j] = cs[3 * b + j];
                sv[so[b] + j] = co[3 * b + j];
            }
#pragma unroll
        for (int k = 0; k < kFillSpt; ++k)
            if (x0[k] != 0xffffffffu) {
                const uint32_t b = x0[k] >> kSrcShift, at = so[b] + (x1[k] >> 16);
                ss[at] = x0[k] & (uint32_t)(kSrc - 1);
                sv[at] = (uint16_t)(x1[k] & 0xffffu);
            }
        __syncthreads();
        // the runs' whole quads: consecutive lanes take consecutive quads
        const uint32_t Q = qo[K];
        for (uint32_t qi = tid; qi < Q; qi += kFillThreads) {
            int64_t lo_b = 0, hi_b = K;                 // the last b with qo[b] <= qi
            while (hi_b - lo_b > 1) {
                const int64_t mid = (lo_b + hi_b) >> 1;
                if (qo[mid] <= qi) lo_b = mid;
                else hi_b = mid;
            }
            const int64_t b = lo_b;
            const uint32_t j = qi - qo[b], at = so[b] + 4 * j;
            uint32_t u[4], v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                u[e] = ss[at + e];
                v[e] = sv[at + e];
            }
            put_src_quad(stream, b1[b] + 4 * j, u);
            put_off_quad(off, b2[b] + 4 * j, v);
        }
        __syncthreads();
        // carries and the segments' next positions
        for (int64_t b = tid; b < K; b += kFillThreads) {
            const uint32_t L = so[b + 1] - so[b], nq = L >> 2, rem = L & 3u;
            for (uint32_t j = 0; j < rem; ++j) {
                cs[3 * b + j] = ss[so[b] + 4 * nq + j];
                co[3 * b + j] = sv[so[b] + 4 * nq + j];
            }
            cc[b] = (uint8_t)rem;
            b1[b] += 4 * (int64_t)nq;
            b2[b] += 4 * (int64_t)nq;
        }
        __syncthreads();
    }
    // the carries and the pad slots up to each segment's 8-slot end; the last
    // tile also zeroes each block's tail up to its chunk end
    for (int64_t b = tid; b < K; b += kFillThreads) {
        const int64_t c = (int64_t)cntB[b * T + t];
        const int64_t pend = p1T[t * K + b] + ((c + 7) & ~7ll);
        int64_t g1 = b1[b], g2 = b2[b];
        int j = 0;
        for (; g1 < pend; g1 += 4, g2 += 4) {
            uint32_t u[4], v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool real = j < cc[b];
                u[e] = real ? cs[3 * b + j] : 0u;
                v[e] = real ? (uint32_t)co[3 * b + j] : 0u;
                ++j;
            }
            put_src_quad(stream, g1, u);
            put_off_quad(off, g2, v);
        }
        if (t == T - 1) {
            const uint32_t z[4] = {0u, 0u, 0u, 0u};
            for (; g1 < blk[b + 1]; g1 += 4) put_src_quad(stream, g1, z);
        }
    }
}

// ---- the sweep ----------------------------------------------------------------

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// UC chunks of a wave's phase-1 stream: lane l holds slots 8l..8l+7 of each
// (one 16-B load of 16-bit word indices, one 4-B load of eight 4-bit bit
// positions; streamed once, so non-temporal)
template <int UC>
struct MsgGroup {
    static constexpr int NW = kMsgThreads / 64;
    v4u l[UC];         // eight 16-bit state-word indices
    unsigned h[UC];    // eight 4-bit bit positions
    // chunks c, c + NW, ... (clamped to the wave's last chunk: always a valid
    // load); c and last are wave-uniform, so every address is a scalar base
    // plus the lane's constant offset
    __device__ __forceinline__ void fetch(const uint16_t* __restrict__ stream, int64_t c, int64_t last, int lane) {
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const int64_t cc = (c + u * NW <= last) ? c + u * NW : last;
            const uint16_t* ch = stream + cc * kChunkU16;
            l[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(ch) + lane);
            h[u] = __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(ch + kChunk) + lane);
        }
    }
    // message bits of chunks c, c + NW, ... below a1: lane l's byte is bits
    // 8l..8l+7 of its chunk, so two DPP row shifts assemble 32-bit words in
    // lanes 0, 4, .., 60 (no ballots, no lane selects)
    __device__ __forceinline__ void emit(const uint16_t* sb16, int64_t c, int64_t a1, int lane,
                                         uint32_t* __restrict__ msg32) const {
#pragma unroll
        for (int u = 0; u < UC; ++u) {
            const unsigned hh = h[u];
            unsigned m = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned x = l[u][q];
                const unsigned v0 = sb16[x & 0xffffu], v1 = sb16[x >> 16];
                m |= (__builtin_amdgcn_ubfe(v0, (hh >> (8 * q)) & 15u, 1) << (2 * q)) |
                     (__builtin_amdgcn_ubfe(v1, (hh >> (8 * q + 4)) & 15u, 1) << (2 * q + 1));
            }
            // row_shl:k (dpp_ctrl 0x100 + k): lane i reads lane i + k of its 16-lane row
            m |= (unsigned)__builtin_amdgcn_mov_dpp((int)m, 0x101, 0xf, 0xf, true) << 8;
            m |= (unsigned)__builtin_amdgcn_mov_dpp((int)m, 0x102, 0xf, 0xf, true) << 16;
            const int64_t cc = c + u * NW;
            if ((lane & 3) == 0 && cc < a1) msg32[cc * 16 + (lane >> 2)] = m;
        }
    }
};

// phase 1: message bit of every slot of block b, in phase-1 order; `split`
// workgroups share a block (each stages the block's 128 KB of state bits).
// UC chunks per wave step, loaded unconditionally (a step's last chunks are
// clamped to the wave's last one and not stored) so that every load of a step
// is in flight before the first lookup.
template <int UC>
__global__ void __launch_bounds__(kMsgThreads) k_bin_msg(const uint16_t* __restrict__ src_lo,
                                                         const uint16_t* __restrict__ src_hi,
                                                         const long long* __restrict__ blk, int64_t n, int split,
                                                         const uint32_t* __restrict__ s32, u64* __restrict__ msg) {
    extern __shared__ uint32_t sb[];
    const int64_t b = blockIdx.x / split;
    const int part = blockIdx.x % split;
    const int64_t g0 = b * kSrcWords, nw32 = (n + 31) >> 5;
    // stage the block's state bits: every thread's eight 16-B loads in flight at once
    {
        constexpr int V = kSrcWords / 4 / kMsgThreads;
        uint4 x[V];
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const int64_t g = g0 + 4 * (threadIdx.x + (int64_t)k * kMsgThreads);
            if (g + 3 < nw32) {
                x[k] = *reinterpret_cast<const uint4*>(s32 + g);
            } else {
                x[k].x = (g < nw32) ? s32[g] : 0u;
                x[k].y = (g + 1 < nw32) ? s32[g + 1] : 0u;
                x[k].z = (g + 2 < nw32) ? s32[g + 2] : 0u;
                x[k].w = 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < V; ++k) reinterpret_cast<uint4*>(sb)[threadIdx.x + k * kMsgThreads] = x[k];
    }
    __syncthreads();
    const int64_t c0 = blk[b] / kChunk, c1 = blk[b + 1] / kChunk;   // this block's chunks
    const int64_t per = (c1 - c0 + split - 1) / split;
    const int64_t a0 = c0 + part * per;
    const int64_t a1 = (a0 + per < c1) ? a0 + per : c1;
    constexpr int NW = kMsgThreads / 64;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // this wave's chunks: a0 + wave + NW*i
    const int64_t last = (a1 - 1 - a0 - wave >= 0) ? a0 + wave + ((a1 - 1 - a0 - wave) / NW) * NW : -1;
    const uint16_t* sb16 = reinterpret_cast<const uint16_t*>(sb);
    uint32_t* msg32 = reinterpret_cast<uint32_t*>(msg);
    // two groups in flight: the loads of group i+1 are issued before the
    // lookups of group i (unrolled by two, so no register copies wait on them);
    // two 512-slot chunks a group (N=1e9, d=6, one box: UC 1 5.85-5.87 ms per
    // sweep, 2 5.57-5.58, 3 5.62-5.64, 4 5.66-5.72, 8 5.66-5.69)
    if (last < 0) return;
    MsgGroup<UC> ga, gb;
    ga.fetch(src_lo, a0 + wave, last, lane);
    for (int64_t c = a0 + wave; c < a1; c += 2 * UC * NW) {
        gb.fetch(src_lo, c + UC * NW, last, lane);
        ga.emit(sb16, c, a1, lane, msg32);
        ga.fetch(src_lo, c + 2 * UC * NW, last, lane);
        gb.emit(sb16, c + UC * NW, a1, lane, msg32);
    }
}

struct Piece {
    uint4 o;     // eight 16-bit destination offsets
    unsigned bits;
};

__device__ __forceinline__ Piece load_piece(const uint16_t* __restrict__ off, const u64* __restrict__ msg,
                                            long long s1, long long s2, int64_t len, int64_t j) {
    Piece pc;
    pc.bits = 0;
    pc.o = make_uint4(0, 0, 0, 0);
    if (j < len) {
        pc.o = *reinterpret_cast<const uint4*>(off + s2 + j);
        const int64_t p = s1 + j;
        const u64 lo = msg[p >> 6], hi = msg[(p >> 6) + 1];
        const int sh = (int)(p & 63);
        const u64 w = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
        const int64_t nb = len - j;
        pc.bits = (unsigned)(w & ((nb >= 8) ? 0xffull : ((1ull << nb) - 1)));
    }
    return pc;
}

__device__ __forceinline__ void apply_piece(uint32_t* cnt, const Piece& pc) {
    const unsigned oo[4] = {pc.o.x, pc.o.y, pc.o.z, pc.o.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if ((pc.bits >> q) & 1u) {
            const unsigned v = (oo[q >> 1] >> ((q & 1) * 16)) & 0xffffu;
            atomicAdd(&cnt[v >> 2], 1u << ((v & 3) << 3));
        }
    }
}

struct Seg {
    long long s1, s2;
    int64_t len;
};

// lane k's 64-bit value as a wave-uniform (scalar) value
__device__ __forceinline__ long long readlane64(long long x, int k) {
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)(x & 0xffffffffll), k);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)((unsigned long long)x >> 32), k);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ Seg seg_of(long long m1, long long m2, long long m2e, int k) {
    Seg s;
    s.s1 = readlane64(m1, k);
    const long long a = readlane64(m2, k), e = readlane64(m2e, k);
    s.s2 = a & ~7ll;
    s.len = (e & ~7ll) - s.s2 - (a & 7);
    return s;
}

// workgroup id -> tile, XCD-contiguous: the first (T % 8) XCDs take one extra tile
__device__ __forceinline__ int64_t xcd_tile(int64_t bid, int64_t T) {
    const int64_t x = bid & 7, i = bid >> 3, q = T >> 3, r = T & 7;
    return x * q + (x < r ? x : r) + i;
}

// the majority rule over a tile's counts: wave w takes the tile's 64-node
// words [64w, 64w + 64); lane i loads the own bits of word i once, and lane k
// keeps word k's result, so the state is read and written in coalesced 512-B runs
__device__ __forceinline__ void tile_rule(const uint32_t* cnt, int64_t t, int64_t lo, int64_t hi, int d,
                                          const uint32_t* __restrict__ s32, u64* __restrict__ s_out,
                                          unsigned long long* __restrict__ counts, unsigned long long* red,
                                          int nw) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t v0 = lo + t * kTile;                       // lo is 64-aligned: whole words
    const int64_t v1 = (v0 + kTile < hi) ? v0 + kTile : hi;
    const int64_t w0 = (v0 >> 6) + (int64_t)wave * 64, wend = (v1 + 63) >> 6;
    const int64_t wl = w0 + lane;
    const u64 own = (wl < wend) ? reinterpret_cast<const u64*>(s32)[wl] : 0ull;
    u64 mine = 0;
    unsigned long long ones = 0;
    const int nk = (wend - w0 <= 0) ? 0 : (wend - w0 < 64 ? (int)(wend - w0) : 64);
    for (int k = 0; k < nk; ++k) {
        const u64 ow = (u64)readlane64((long long)own, k);
        const int64_t v = ((w0 + k) << 6) + lane;
        bool nb = false;
        if (v < v1) {
            const int64_t lv = v - v0;
            const int c = (int)((cnt[lv >> 2] >> ((lv & 3) << 3)) & 0xffu);
            const int o = (int)((ow >> lane) & 1ull);
            nb = (2 * c > d) || ((2 * c == d) && o);         // always-stay ties (code/SA_RRG.py:19-20)
        }
        const u64 word = __ballot(nb);
        if (lane == k) mine = word;
        ones += __popcll(word);
    }
    if (wl < wend) s_out[wl] = mine;
    if (counts) {
        if (lane == 0) red[wave] = ones;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long tot = 0;
            for (int i = 0; i < nw; ++i) tot += red[i];
            if (tot) atomicAdd(counts, tot);
        }
    }
}

// phase 2: one workgroup per destination tile; U segments per step
template <int U>
__global__ void __launch_bounds__(kApplyThreads) k_bin_apply(const uint16_t* __restrict__ off,
                                                             const long long* __restrict__ p1T,
                                                             const long long* __restrict__ p2,
                                                             const u64* __restrict__ msg, int64_t K, int64_t lo,
                                                             int64_t hi, int d, const uint32_t* __restrict__ s32,
                                                             u64* __restrict__ s_out,
                                                             unsigned long long* __restrict__ counts) {
    extern __shared__ uint32_t cnt[];
    constexpr int NW = kApplyThreads / 64;
    __shared__ unsigned long long red[NW];
    // XCD-aware order: workgroups are placed round-robin on the 8 XCDs, so XCD x
    // takes the consecutive tiles [x*T/8, (x+1)*T/8) and the message lines that
    // neighbouring tiles share (segments (b,t), (b,t+1), ... are adjacent in
    // phase-1 order) are hit in that XCD's L2
    const int64_t T = gridDim.x;
    const int64_t t = xcd_tile(blockIdx.x, T);
    for (int i = threadIdx.x; i < kCntWords; i += kApplyThreads) cnt[i] = 0;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long* q1 = p1T + t * K;
    const long long* q2 = p2 + t * K;
    // segments interleaved over the waves (wave w takes g + w, g + w + NW, ...):
    // at every step the workgroup's waves read NW neighbouring segments, one
    // contiguous stretch of off[] (a wave-private run of 64 segments reads
    // 16 scattered ~1 KB pieces per step and streams ~25% slower)
    for (int64_t g = 0; g < K; g += NW * 64) {
        const int64_t mb = g + (int64_t)lane * NW + wave;
        long long m1 = 0, m2 = 0, m2e = 0;
        if (mb < K) {
            m1 = q1[mb];
            m2 = q2[mb];
            m2e = q2[mb + 1];
        }
        const int64_t left = K - g - wave;   // segments g + wave + NW*l with l < ns
        const int ns = (left <= 0) ? 0 : (int)((left + NW - 1) / NW < 64 ? (left + NW - 1) / NW : 64);
        // U segments per step: their first 512-slot pieces are all in flight
        // before any count lands in LDS
        for (int k = 0; k < ns; k += U) {
            Seg sg[U];
            Piece pc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                sg[u] = seg_of(m1, m2, m2e, (k + u < ns) ? k + u : k);
                if (k + u >= ns) sg[u].len = 0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) pc[u] = load_piece(off, msg, sg[u].s1, sg[u].s2, sg[u].len, 8 * lane);
#pragma unroll
            for (int u = 0; u < U; ++u) apply_piece(cnt, pc[u]);
#pragma unroll
            for (int u = 0; u < U; ++u)
                for (int64_t i = 512; i < sg[u].len; i += 512)
                    apply_piece(cnt, load_piece(off, msg, sg[u].s1, sg[u].s2, sg[u].len, i + 8 * lane));
        }
    }
    __syncthreads();
    tile_rule(cnt, t, lo, hi, d, s32, s_out, counts, red, NW);
}

// phase 2, flat form (K <= kFlatMaxK): the tile's segment starts (relative,
// pad count in the low 3 bits) and phase-1 positions are staged in LDS, and
// each wave streams one contiguous stretch of the tile's offsets in 512-slot
// chunks (one coalesced 1 KB load per wave instruction), finding each 8-slot
// piece's segment with a forward cursor in LDS; four chunks per step.
constexpr int kFlatMaxK = 960;      // 64 KB of counters + 12 B per segment stay within half of the CU's LDS

// one group of UC 8-slot pieces of a wave's stretch: 16-bit destination
// offsets, the pieces' message bytes and their valid-slot masks
template <int UC>
struct Group {
    uint4 o[UC];
    unsigned m[UC];
    unsigned lim[UC];
};

template <int UC>
__device__ __forceinline__ void fetch_group(Group<UC>& g, int32_t c, int32_t a1, int lane, int32_t& b,
                                            const int32_t* srel, const long long* spos, const uint16_t* offt,
                                            const uint8_t* __restrict__ msg8) {
    // positions first (LDS cursor), then every load of the group unconditionally:
    // pieces past the stretch read its last piece and get an empty mask
    const uint16_t* po[UC];
    const uint8_t* pm[UC];
#pragma unroll
    for (int u = 0; u < UC; ++u) {
        const int32_t j0 = c + u * 512 + 8 * lane;
        const bool valid = j0 < a1;
        const int32_t j = valid ? j0 : a1 - 8;
        while ((srel[b + 1] & ~7) <= j) ++b;               // forward cursor (start[K] = Lt > j)
        const int32_t sb = srel[b];
        const int32_t st0 = sb & ~7;
        const int32_t len = (srel[b + 1] & ~7) - st0 - (sb & 7);
        const int32_t rel = j - st0;
        po[u] = offt + j;
        // segments start on 8-slot boundaries in both orders: the piece's
        // eight message bits are one byte
        pm[u] = msg8 + ((spos[b] + rel) >> 3);
        const int32_t nb = len - rel;
        g.lim[u] = !valid ? 0u : ((nb >= 8) ? 0xffu : (nb > 0 ? ((1u << nb) - 1) : 0u));
    }
#pragma unroll
    for (int u = 0; u < UC; ++u) {
        g.o[u] = *reinterpret_cast<const uint4*>(po[u]);
        g.m[u] = *pm[u];
    }
}

template <int UC>
__device__ __forceinline__ void apply_group(uint32_t* cnt, const Group<UC>& g) {
#pragma unroll
    for (int u = 0; u < UC; ++u) {
        const unsigned bits = g.m[u] & g.lim[u];
        const unsigned oo[4] = {g.o[u].x, g.o[u].y, g.o[u].z, g.o[u].w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            // only +1 messages touch the LDS (adding zeros for every lane costs
            // ~2 ms per sweep at N=1e9: the LDS atomic rate is per active lane)
            if ((bits >> q) & 1u) {
                const unsigned v = (oo[q >> 1] >> ((q & 1) * 16)) & 0xffffu;
                atomicAdd(&cnt[v >> 2], 1u << ((v & 3) << 3));
            }
        }
    }
}

// UC = 2 pieces per group, two groups in flight: <= 64 VGPRs keeps two
// workgroups (8 waves per SIMD) on a CU; deeper groups (UC = 3, 4) measured slower
template <int UC>
__global__ void __launch_bounds__(kApplyThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) k_bin_apply_flat(const uint16_t* __restrict__ off,
                                                                  const long long* __restrict__ p1T,
                                                                  const long long* __restrict__ p2,
                                                                  const u64* __restrict__ msg, int64_t K, int64_t lo,
                                                                  int64_t hi, int d, const uint32_t* __restrict__ s32,
                                                                  u64* __restrict__ s_out,
                                                                  unsigned long long* __restrict__ counts) {
    extern __shared__ uint32_t cnt[];
    constexpr int NW = kApplyThreads / 64;
    __shared__ unsigned long long red[NW];
    __shared__ int32_t srel[kFlatMaxK + 1];          // segment start - tile start | pad count
    __shared__ long long spos[kFlatMaxK];            // phase-1 position of the segment
    const int64_t T = gridDim.x;
    const int64_t t = xcd_tile(blockIdx.x, T);
    const long long* q2 = p2 + t * K;
    const long long P0 = q2[0] & ~7ll;
    for (int i = threadIdx.x; i < kCntWords; i += kApplyThreads) cnt[i] = 0;
    for (int64_t b = threadIdx.x; b <= K; b += kApplyThreads) {
        const long long v = q2[b];
        srel[b] = (int32_t)(((v & ~7ll) - P0) | (b < K ? (v & 7) : 0));
        if (b < K) spos[b] = p1T[t * K + b];
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t Lt = srel[K] & ~7;
    const int32_t Lw = (((Lt + NW - 1) / NW) + 511) & ~511;   // this wave's stretch, whole chunks
    const int32_t a0 = wave * Lw;
    const int32_t a1 = (a0 + Lw < Lt) ? a0 + Lw : Lt;
    // segment of this lane's first piece: last b with start <= j (binary search)
    int32_t b = 0;
    {
        const int32_t j = a0 + 8 * lane;
        int32_t lo_b = 0, hi_b = (int32_t)K;                  // invariant: start[lo_b] <= j < start[hi_b]
        if (j < Lt) {
            while (hi_b - lo_b > 1) {
                const int32_t mid = (lo_b + hi_b) >> 1;
                if ((srel[mid] & ~7) <= j) lo_b = mid; else hi_b = mid;
            }
        }
        b = lo_b;
    }
    const uint16_t* offt = off + P0;
    const uint8_t* msg8 = reinterpret_cast<const uint8_t*>(msg);
    // two groups in flight: the loads of group i+1 are issued before the LDS
    // counts of group i
    if (a0 < a1) {
        Group<UC> ga, gb;
        fetch_group<UC>(ga, a0, a1, lane, b, srel, spos, offt, msg8);
        for (int32_t c = a0; c < a1; c += 2 * UC * 512) {
            fetch_group<UC>(gb, c + UC * 512, a1, lane, b, srel, spos, offt, msg8);
            apply_group<UC>(cnt, ga);
            fetch_group<UC>(ga, c + 2 * UC * 512, a1, lane, b, srel, spos, offt, msg8);
            apply_group<UC>(cnt, gb);
        }
    }
    __syncthreads();
    tile_rule(cnt, t, lo, hi, d, s32, s_out, counts, red, NW);
}

inline int check_range(int64_t n, int d, int64_t row_lo, int64_t row_hi) {
    if (n < 1 || d < 1 || d > 16 || row_lo < 0 || row_hi > n || row_lo > row_hi) return MJX_EINVAL;
    if ((row_lo & 63) || ((row_hi & 63) && row_hi != n)) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (((n + kSrc - 1) >> kSrcShift) > kMaxBlocks) return MJX_ERANGE;
    return MJX_OK;
}

}  // namespace binned
}  // namespace mjx

extern "C" int mjx_binned_plan_shape(int64_t n, int d, int64_t row_lo, int64_t row_hi, int64_t* sizes) {
    using namespace mjx::binned;
    if (!sizes) return MJX_EINVAL;
    const int rc = check_range(n, d, row_lo, row_hi);
    if (rc) return rc;
    const Shape s = shape(n, d, row_hi - row_lo);
    sizes[0] = s.src_len / kChunk * kChunkU16;       // the phase-1 stream (src_lo; src_hi unused)
    sizes[1] = 0;
    sizes[2] = s.off_len;
    sizes[3] = s.index_len;
    sizes[4] = s.msg_words;
    sizes[5] = s.work_bytes;
    return MJX_OK;
}

extern "C" int mjx_binned_build(const int32_t* adj, int64_t n, int d, int64_t row_lo, int64_t row_hi,
                                uint16_t* src_lo, uint16_t* src_hi, uint16_t* off, long long* index, void* work,
                                int64_t work_bytes, void* stream) {
    using namespace mjx::binned;
    const int rc = check_range(n, d, row_lo, row_hi);
    if (rc) return rc;
    const int64_t rows = row_hi - row_lo;
    if (rows == 0) return MJX_OK;
    if (!adj || !src_lo || !off || !index || !work) return MJX_EINVAL;
    const Shape s = shape(n, d, rows);
    if (work_bytes < s.work_bytes) return MJX_ERANGE;
    const int64_t K = s.K, T = s.T, S = s.S;
    uint32_t* cntB = reinterpret_cast<uint32_t*>(work);
    long long* p1 = reinterpret_cast<long long*>(static_cast<char*>(work) + align256(4 * S));
    void* scan = static_cast<char*>(work) + align256(4 * S) + align256(8 * S);
    long long* blk = index;
    long long* p1T = index + (K + 1);
    long long* p2 = p1T + S;
    hipStream_t st = mjx::as_stream(stream);
    size_t need2 = 0, needk = 0;
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need2, p2, p2, S + 1, st), "bin scan size");
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, needk, blk, blk, K + 1, st), "bin scan size");
    if ((int64_t)need2 > kScanScratch || (int64_t)needk > kScanScratch) return MJX_ERANGE;
    const FillLds fl = fill_lds(K);
    if (K > 2 * kFillThreads || fl.ch < kFillThreads) return MJX_ERANGE;     // (K <= 2048 for n <= INT32_MAX)
    MJX_HIP(hipMemsetAsync(p2 + S, 0, sizeof(long long), st), "bin memset p2");
    MJX_HIP(hipMemsetAsync(blk + K, 0, sizeof(long long), st), "bin memset blk");
    k_bin_count<<<(unsigned)T, 256, K * sizeof(unsigned), st>>>(adj, rows, d, n, K, T, cntB, p2);
    MJX_LAUNCH_CHECK("k_bin_count");
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(scan, need2, p2, p2, S + 1, st), "bin scan p2");
    k_bin_tag<<<mjx::grid_for(S), 256, 0, st>>>(cntB, K, T, p2);
    MJX_LAUNCH_CHECK("k_bin_tag");
    k_bin_blockscan<<<(unsigned)K, 256, 0, st>>>(cntB, T, p1, blk);
    MJX_LAUNCH_CHECK("k_bin_blockscan");
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(scan, needk, blk, blk, K + 1, st), "bin scan blk");
    k_bin_finish<<<mjx::grid_for(S), 256, 0, st>>>(p1, blk, K, T, p1T);
    MJX_LAUNCH_CHECK("k_bin_finish");
    MJX_HIP(mjx::set_max_lds(k_bin_fill, (int)fl.bytes), "k_bin_fill lds");
    k_bin_fill<<<(unsigned)T, kFillThreads, (size_t)fl.bytes, st>>>(adj, rows, d, n, K, T, fl, p1T, p2, cntB, blk,
                                                                     src_lo, off);
    MJX_LAUNCH_CHECK("k_bin_fill");
    return MJX_OK;
}

extern "C" int mjx_sweep_binned(const uint16_t* src_lo, const uint16_t* src_hi, const uint16_t* off,
                                const long long* index, int64_t n, int d,
                                int64_t row_lo, int64_t row_hi, const uint64_t* s_in, uint64_t* msg, uint64_t* s_out,
                                unsigned long long* counts, int apply_form, void* stream) {
    using namespace mjx::binned;
    const int rc = check_range(n, d, row_lo, row_hi);
    if (rc) return rc;
    if (apply_form < 0 || apply_form > 2) return MJX_EINVAL;
    if (row_hi == row_lo) return MJX_OK;
    if (!src_lo || !off || !index || !s_in || !msg || !s_out || s_in == s_out) return MJX_EINVAL;
    const Shape s = shape(n, d, row_hi - row_lo);
    const long long* blk = index;
    const long long* p1T = index + (s.K + 1);
    const long long* p2 = p1T + s.S;
    hipStream_t st = mjx::as_stream(stream);

    // a rank with all rows: 4 workgroups per source block (~4 per CU); with
    // fewer rows fewer, so that staging the block stays a small share
    // (2, 4 and 8 measured within 5 % of each other at N=1e9, d=6)
    const int64_t rows = row_hi - row_lo;
    int split = (int)((kMsgSplitMax * rows + n - 1) / n);
    split = split < 1 ? 1 : (split > kMsgSplitMax ? kMsgSplitMax : split);
    MJX_HIP(hipFuncSetAttribute((const void*)k_bin_msg<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kSrcWords * (int)sizeof(uint32_t)), "k_bin_msg lds");
    k_bin_msg<2><<<(unsigned)(s.K * split), kMsgThreads, kSrcWords * sizeof(uint32_t), st>>>(
        src_lo, src_hi, blk, n, split, (const uint32_t*)s_in, (mjx::u64*)msg);
    MJX_LAUNCH_CHECK("k_bin_msg");
    // the flat form streams the tile contiguously; it needs the tile's
    // segment table in LDS (K <= kFlatMaxK: n <= ~1e9); apply_form 2 asks for
    // the per-segment form (tests run both)
    if (apply_form == 1 && s.K > kFlatMaxK) return MJX_ERANGE;
    const bool flat = s.K <= kFlatMaxK && apply_form != 2;
    if (flat) {
        MJX_HIP(hipFuncSetAttribute((const void*)k_bin_apply_flat<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    kCntWords * (int)sizeof(uint32_t)), "k_bin_apply_flat lds");
        k_bin_apply_flat<2><<<(unsigned)s.T, kApplyThreads, kCntWords * sizeof(uint32_t), st>>>(
            off, p1T, p2, (const mjx::u64*)msg, s.K, row_lo, row_hi, d, (const uint32_t*)s_in, (mjx::u64*)s_out,
            counts);
        MJX_LAUNCH_CHECK("k_bin_apply_flat");
        return MJX_OK;
    }
    MJX_HIP(hipFuncSetAttribute((const void*)k_bin_apply<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kCntWords * (int)sizeof(uint32_t)), "k_bin_apply lds");
    k_bin_apply<2><<<(unsigned)s.T, kApplyThreads, kCntWords * sizeof(uint32_t), st>>>(
        off, p1T, p2, (const mjx::u64*)msg, s.K, row_lo, row_hi, d, (const uint32_t*)s_in, (mjx::u64*)s_out, counts);
    MJX_LAUNCH_CHECK("k_bin_apply");
    return MJX_OK;
}

// ===========================================================================
// Device Erdos-Renyi G(n, p) generator into CSR.
//
// The notebook draws nx.erdos_renyi_graph(n, p) (code/ER_BDCM_entropy.ipynb,
// cell 'ER graph', nb:278-282), removes isolated nodes and relabels the rest in
// increasing order (nb:283-291); its dense adj_matrix (nb:294) is O(n^2) and
// makes n = 1e7 (config C4) impossible.  Parity with networkx is
// distributional: every pair (i, j), i < j, is an edge independently with
// probability p.  Row i's upper pairs (i, j > i) are drawn by geometric
// skipping, j <- j + 1 + floor(log(u) / log(1 - p)), with the k-th uniform u
// of row i a counter-based hash of (seed, i, k): rows are independent, so the
// count pass and the fill pass regenerate the same pairs.
//   k_er_count: upper-pair count per row, degree histogram (atomics);
//   (drop isolated: keep = deg > 0, new id = exclusive scan of keep);
//   row_ptr = exclusive scan of the kept degrees;
//   k_er_fill:  the upper neighbours of row i are the last up[i] entries of
//               row i in ascending order; row i is also a lower neighbour of
//               each of them, placed through a per-row cursor;
//   k_er_sort:  each row's lower part is sorted, so the CSR (rows ascending)
//               depends on the seed only.
// Setup call: synchronises `stream` once to read the edge count.
// ===========================================================================
namespace mjx {
namespace er {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// k-th uniform of row i, in (0, 1]
__device__ __forceinline__ double uniform(uint64_t seed, int64_t i, int64_t k) {
    const uint64_t h = mix64(mix64(seed ^ 0x9e3779b97f4a7c15ull) + mix64((uint64_t)i * 0x100000001b3ull + (uint64_t)k));
    return ((double)(h >> 11) + 1.0) * 0x1.0p-53;
}

// visits the upper neighbours j > i of row i, ascending
template <class F>
__device__ __forceinline__ void row_pairs(uint64_t seed, int64_t i, int64_t n, double lq, F&& f) {
    if (lq == 0.0) return;                          // p = 0
    int64_t j = i;
    for (int64_t k = 0;; ++k) {
        const double g = floor(log(uniform(seed, i, k)) / lq);
        if (!(g < (double)(n - 1 - j))) break;      // also catches +inf
        j += 1 + (int64_t)g;
        f(j);
    }
}

__global__ void k_er_count(int64_t n, double lq, uint64_t seed, int* __restrict__ up, int* __restrict__ deg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int c = 0;
        row_pairs(seed, i, n, lq, [&](int64_t j) {
            ++c;
            atomicAdd(&deg[j], 1);
        });
        up[i] = c;
        if (c) atomicAdd(&deg[i], c);
    }
}

// keep flag (deg > 0, or every node) as the value to scan into new ids
__global__ void k_er_keep(int64_t n, int drop, const int* __restrict__ deg, int* __restrict__ keep,
                          long long* __restrict__ kdeg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        keep[i] = (!drop || deg[i] > 0) ? 1 : 0;
        kdeg[i] = deg[i];
    }
}

// row_ptr of the kept rows: scanned degrees compacted through the new ids
__global__ void k_er_rowptr(int64_t n, const int* __restrict__ keep, const int* __restrict__ newid,
                            const long long* __restrict__ sdeg, long long* __restrict__ row_ptr) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (keep[i]) row_ptr[newid[i]] = sdeg[i];
}

__global__ void k_er_fill(int64_t n, double lq, uint64_t seed, const int* __restrict__ up,
                          const int* __restrict__ keep, const int* __restrict__ newid,
                          const long long* __restrict__ row_ptr, int* __restrict__ cur, int32_t* __restrict__ col) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!up[i]) continue;
        const int32_t ni = newid[i];
        long long pos = row_ptr[ni + 1] - up[i];
        row_pairs(seed, i, n, lq, [&](int64_t j) {
            const int32_t nj = newid[j];
            col[pos++] = nj;
            const int s = atomicAdd(&cur[nj], 1);
            col[row_ptr[nj] + s] = ni;
        });
        (void)keep;
    }
}

// sort the lower part (first cur[r] entries) of every kept row
__global__ void k_er_sort(int64_t rows, const long long* __restrict__ row_ptr, const int* __restrict__ cur,
                          int32_t* __restrict__ col) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
        int32_t* a = col + row_ptr[r];
        const int m = cur[r];
        for (int x = 1; x < m; ++x) {
            const int32_t v = a[x];
            int y = x - 1;
            while (y >= 0 && a[y] > v) {
                a[y + 1] = a[y];
                --y;
            }
            a[y + 1] = v;
        }
    }
}

constexpr int64_t kScan = 16ll << 20;

inline int64_t work_bytes(int64_t n) {
    // up, deg, keep, newid, cur: int32[n] each (padded); kdeg/sdeg: int64[n+1]; scan scratch
    const int64_t a = (4 * n + 255) & ~255ll, b = (8 * (n + 1) + 255) & ~255ll;
    return 5 * a + b + kScan;
}

}  // namespace er
}  // namespace mjx

extern "C" int64_t mjx_er_work_bytes(int64_t n) { return n < 1 ? 0 : mjx::er::work_bytes(n); }

extern "C" int mjx_er_generate(int64_t n, double p, uint64_t seed, int drop_isolated, long long* row_ptr,
                               int32_t* col, int64_t col_cap, int64_t* n_out, int64_t* nnz_out, void* work,
                               int64_t work_bytes, void* stream) {
    using namespace mjx::er;
    if (n < 1 || n > (int64_t)INT32_MAX - 1 || !(p >= 0.0) || !(p < 1.0) || !row_ptr || !n_out || !nnz_out || !work)
        return MJX_EINVAL;
    if (work_bytes < mjx::er::work_bytes(n)) return MJX_ERANGE;
    hipStream_t st = mjx::as_stream(stream);
    const int64_t a = (4 * n + 255) & ~255ll;
    char* w = static_cast<char*>(work);
    int* up = reinterpret_cast<int*>(w);
    int* deg = reinterpret_cast<int*>(w + a);
    int* keep = reinterpret_cast<int*>(w + 2 * a);
    int* newid = reinterpret_cast<int*>(w + 3 * a);
    int* cur = reinterpret_cast<int*>(w + 4 * a);
    long long* kdeg = reinterpret_cast<long long*>(w + 5 * a);
    void* scan = w + 5 * a + ((8 * (n + 1) + 255) & ~255ll);
    const double lq = (p > 0.0) ? log1p(-p) : 0.0;          // 0 marks p = 0 (no pairs)
    const int grid = mjx::grid_for(n);
    MJX_HIP(hipMemsetAsync(deg, 0, sizeof(int) * n, st), "er memset");
    MJX_HIP(hipMemsetAsync(cur, 0, sizeof(int) * n, st), "er memset");
    k_er_count<<<grid, 256, 0, st>>>(n, lq, seed, up, deg);
    MJX_LAUNCH_CHECK("k_er_count");
    k_er_keep<<<grid, 256, 0, st>>>(n, drop_isolated, deg, keep, kdeg);
    MJX_LAUNCH_CHECK("k_er_keep");
    MJX_HIP(hipMemsetAsync(kdeg + n, 0, sizeof(long long), st), "er memset");
    size_t need1 = 0, need2 = 0;
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need1, keep, newid, n, st), "er scan size");
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need2, kdeg, kdeg, n + 1, st), "er scan size");
    if ((int64_t)need1 > kScan || (int64_t)need2 > kScan) return MJX_ERANGE;
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(scan, need1, keep, newid, n, st), "er scan ids");
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(scan, need2, kdeg, kdeg, n + 1, st), "er scan degrees");
    // kept count and edge total: newid[n-1] + keep[n-1], kdeg[n]
    int last[2];
    long long tot = 0;
    MJX_HIP(hipMemcpyAsync(&last[0], newid + n - 1, sizeof(int), hipMemcpyDeviceToHost, st), "er read");
    MJX_HIP(hipMemcpyAsync(&last[1], keep + n - 1, sizeof(int), hipMemcpyDeviceToHost, st), "er read");
    MJX_HIP(hipMemcpyAsync(&tot, kdeg + n, sizeof(long long), hipMemcpyDeviceToHost, st), "er read");
    MJX_HIP(hipStreamSynchronize(st), "er sync");
    const int64_t n2 = (int64_t)last[0] + last[1];
    *n_out = n2;
    *nnz_out = tot;
    if (tot > col_cap) return MJX_ERANGE;
    if (tot > 0 && !col) return MJX_EINVAL;
    k_er_rowptr<<<grid, 256, 0, st>>>(n, keep, newid, kdeg, row_ptr);
    MJX_LAUNCH_CHECK("k_er_rowptr");
    MJX_HIP(hipMemcpyAsync(row_ptr + n2, &tot, sizeof(long long), hipMemcpyHostToDevice, st), "er total");
    if (tot > 0) {
        k_er_fill<<<grid, 256, 0, st>>>(n, lq, seed, up, keep, newid, row_ptr, cur, col);
        MJX_LAUNCH_CHECK("k_er_fill");
        k_er_sort<<<mjx::grid_for(n2), 256, 0, st>>>(n2, row_ptr, cur, col);
        MJX_LAUNCH_CHECK("k_er_sort");
    }
    MJX_HIP(hipStreamSynchronize(st), "er sync");   // `tot` lives on this stack frame
    return MJX_OK;
}
