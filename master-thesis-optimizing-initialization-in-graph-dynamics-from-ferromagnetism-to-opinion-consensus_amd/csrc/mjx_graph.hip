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
#include <unordered_map>
#include <utility>
#include <vector>
#include <hipcub/hipcub.hpp>

namespace mjx {
namespace gen {

constexpr int kRounds = 6;
constexpr int kMaxD = 16;

struct Perm {
    uint64_t M;        // domain [0, M)
    uint32_t mask;     // half-width mask
    int h;             // half width in bits
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

// balanced Feistel network on [0, 2^(2h))
__host__ __device__ inline uint64_t feistel(const Perm& P, uint64_t v) {
    uint32_t L = (uint32_t)(v >> P.h), R = (uint32_t)v & P.mask;
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t t = L ^ (mix32(R ^ P.key[r]) & P.mask);
        L = R;
        R = t;
    }
    return ((uint64_t)L << P.h) | R;
}

__host__ __device__ inline uint64_t feistel_inv(const Perm& P, uint64_t v) {
    uint32_t L = (uint32_t)(v >> P.h), R = (uint32_t)v & P.mask;
    for (int r = kRounds - 1; r >= 0; --r) {
        const uint32_t t = R ^ (mix32(L ^ P.key[r]) & P.mask);
        R = L;
        L = t;
    }
    return ((uint64_t)L << P.h) | R;
}

// cycle walking restricts the permutation to [0, M) (domain < 4M, so a few steps)
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

static Perm make_perm(uint64_t M, uint64_t seed) {
    Perm P;
    P.M = M;
    int bits = 1;
    while ((1ull << bits) < M) ++bits;
    if (bits & 1) ++bits;
    P.h = bits / 2;
    P.mask = (uint32_t)((1ull << P.h) - 1ull);
    uint64_t s = seed ^ 0x6a09e667f3bcc909ull;
    for (int r = 0; r < kRounds; ++r) P.key[r] = (uint32_t)splitmix64(s);
    return P;
}

// Rows of every node are computed (the defect scan needs all of them); rows in
// [lo, hi) are stored.  defects[0] = count, then (stub, partner stub) pairs.
__global__ void __launch_bounds__(256) k_rrg_rows(Perm P, int64_t n, int d, int64_t lo, int64_t hi,
                                                  int32_t* __restrict__ adj, unsigned long long* __restrict__ defects,
                                                  int64_t cap) {
    __shared__ unsigned long long ps[kMaxD * 256];
    const int tid = threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t v = (int64_t)blockIdx.x * 256 + tid; v < n; v += stride) {
        const bool mine = v >= lo && v < hi;
        for (int k = 0; k < d; ++k) {
            const uint64_t p = partner(P, (uint64_t)v * d + k);
            ps[k * 256 + tid] = p;
            if (mine) adj[(v - lo) * d + k] = (int32_t)(p / (uint64_t)d);
        }
        for (int k = 0; k < d; ++k) {
            const uint64_t s = (uint64_t)v * d + k, p = ps[k * 256 + tid];
            const int64_t w = (int64_t)(p / (uint64_t)d);
            bool bad = false;
            if (w == v) {
                bad = s < p;                                   // self-loop, recorded once
            } else if (v < w) {                                // a repeated neighbour, recorded from the lower end
                for (int j = 0; j < k; ++j)
                    if ((int64_t)(ps[j * 256 + tid] / (uint64_t)d) == w) {
                        bad = true;
                        break;
                    }
            }
            if (bad) {
                const unsigned long long q = atomicAdd(defects, 1ull);
                if ((int64_t)q < cap) {
                    defects[1 + 2 * q] = s;
                    defects[2 + 2 * q] = p;
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
    int64_t node(uint64_t s) const { return (int64_t)(s / d); }
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
    const Perm P = make_perm((uint64_t)n * (uint64_t)d, seed);
    return (int64_t)partner(P, (uint64_t)stub);
}

extern "C" int mjx_rrg_generate(int64_t n, int d, uint64_t seed, int64_t row_lo, int64_t row_hi, int32_t* adj,
                                uint64_t* work, int64_t work_words, int64_t* n_switches, void* stream) {
    if (n < 2 || d < 1 || d >= n || (n * (int64_t)d) % 2 || row_lo < 0 || row_hi > n || row_lo > row_hi)
        return MJX_EINVAL;
    if (d > kMaxD || n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if ((row_hi > row_lo && !adj) || !work || work_words < 3) return MJX_EINVAL;
    const int64_t cap = (work_words - 1) / 2;
    const Perm P = make_perm((uint64_t)n * (uint64_t)d, seed);
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
// Source-binned sweep of a node-packed state (one replica, huge n: config C5).
//
// The gather sweep reads s[u] for 6e9 random u per sweep at N=1e9, d=6: every
// 4-byte gather costs a cache line from a 125 MB state that no L2 holds, so it
// runs at the random line rate.  Here the n*d (destination, source) slots of a
// rank's rows are binned once (a static plan) by source block b = u >> kSrcShift
// (2 MB of state bits each, L2-resident) and, inside a block, by destination
// tile t = (v - lo) >> kTileShift.  A sweep is then
//   phase 1: stream the slots block by block, read s[u] (an L2 hit: the whole
//            chip works on one or two source blocks at a time) and write one
//            message bit per slot, in slot order (coalesced);
//   phase 2: one workgroup per destination tile gathers its K contiguous
//            segments (message bits + 16-bit tile offsets), counts +1
//            neighbours per node in LDS and applies the majority rule
//            (always-stay ties, code/SA_RRG.py:19-20) against the node's own bit.
// Traffic per sweep ~ 4 + 2 bytes of static plan and 2/8 bit of messages per
// slot, all streamed, instead of a random line per slot.
// ===========================================================================
namespace mjx {
namespace binned {

constexpr int kSrcShift = 24;          // 16M nodes = 2 MB of bits per source block
constexpr int kTileShift = 13;         // 8192 destinations per tile (32 KB of LDS counters)
constexpr int kTile = 1 << kTileShift;

__host__ __device__ inline int64_t nblocks(int64_t n) { return (n + (1ll << kSrcShift) - 1) >> kSrcShift; }
__host__ __device__ inline int64_t ntiles(int64_t rows) { return (rows + kTile - 1) >> kTileShift; }

// slot counts per (block, tile): one workgroup per tile, LDS histogram over blocks
__global__ void __launch_bounds__(256) k_bin_count(const int32_t* __restrict__ adj, int64_t rows, int d, int64_t K,
                                                   int64_t T, long long* __restrict__ cnt) {
    extern __shared__ unsigned hist[];
    const int64_t t = blockIdx.x;
    for (int64_t b = threadIdx.x; b < K; b += 256) hist[b] = 0;
    __syncthreads();
    const int64_t s0 = t * kTile * d, s1 = ((t + 1) * kTile < rows ? (t + 1) * kTile : rows) * d;
    for (int64_t q = s0 + threadIdx.x; q < s1; q += 256) atomicAdd(&hist[adj[q] >> kSrcShift], 1u);
    __syncthreads();
    for (int64_t b = threadIdx.x; b < K; b += 256) cnt[b * T + t] = hist[b];
}

// place every slot at seg_ptr[b*T + t] + (its rank inside the segment; order
// inside a segment is free: phase 2 only counts)
__global__ void __launch_bounds__(256) k_bin_fill(const int32_t* __restrict__ adj, int64_t rows, int d, int64_t K,
                                                  int64_t T, const long long* __restrict__ seg_ptr,
                                                  int32_t* __restrict__ src, uint16_t* __restrict__ off) {
    extern __shared__ unsigned cur[];
    const int64_t t = blockIdx.x;
    for (int64_t b = threadIdx.x; b < K; b += 256) cur[b] = 0;
    __syncthreads();
    const int64_t s0 = t * kTile * d, s1 = ((t + 1) * kTile < rows ? (t + 1) * kTile : rows) * d;
    for (int64_t q = s0 + threadIdx.x; q < s1; q += 256) {
        const int32_t u = adj[q];
        const int64_t b = u >> kSrcShift;
        const int64_t pos = seg_ptr[b * T + t] + atomicAdd(&cur[b], 1u);
        src[pos] = u;
        off[pos] = (uint16_t)((q / d) - t * kTile);
    }
}

// phase 1: message bit of every slot, in plan order
__global__ void __launch_bounds__(256) k_bin_messages(const int32_t* __restrict__ src, int64_t slots,
                                                      const uint32_t* __restrict__ s32, u64* __restrict__ msg) {
    const int lane = threadIdx.x & 63;
    const int64_t nwords = (slots + 63) >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * 256) >> 6;
    for (int64_t w = wave; w < nwords; w += nwaves) {
        const int64_t e = (w << 6) + lane;
        bool bit = false;
        if (e < slots) {
            const int32_t u = src[e];
            bit = (s32[u >> 5] >> (u & 31)) & 1u;
        }
        const u64 word = __ballot(bit);
        if (lane == 0) msg[w] = word;
    }
}

// phase 2: one workgroup per destination tile
__global__ void __launch_bounds__(256) k_bin_update(const uint16_t* __restrict__ off,
                                                    const long long* __restrict__ seg_ptr, const u64* __restrict__ msg,
                                                    int64_t K, int64_t T, int64_t lo, int64_t hi, int d,
                                                    const uint32_t* __restrict__ s32, u64* __restrict__ s_out,
                                                    unsigned long long* __restrict__ counts) {
    __shared__ unsigned cnt[kTile];
    __shared__ unsigned long long red[4];
    const int64_t t = blockIdx.x;
    for (int i = threadIdx.x; i < kTile; i += 256) cnt[i] = 0;
    __syncthreads();
    for (int64_t b = 0; b < K; ++b) {
        const int64_t e0 = seg_ptr[b * T + t], e1 = seg_ptr[b * T + t + 1];
        for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
            const unsigned bit = (unsigned)((msg[e >> 6] >> (e & 63)) & 1ull);
            if (bit) atomicAdd(&cnt[off[e]], 1u);
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t v0 = lo + t * kTile;
    const int64_t v1 = (v0 + kTile < hi) ? v0 + kTile : hi;
    unsigned long long ones = 0;
    for (int64_t w = (v0 >> 6) + (threadIdx.x >> 6); w < ((v1 + 63) >> 6); w += 4) {
        const int64_t v = (w << 6) + lane;
        bool nb = false;
        if (v < v1) {
            const int c = (int)cnt[v - v0];
            const int own = (s32[v >> 5] >> (v & 31)) & 1u;
            nb = (2 * c > d) || ((2 * c == d) && own);
        }
        const u64 word = __ballot(nb);
        if (lane == 0) {
            s_out[w] = word;
            ones += __popcll(word);
        }
    }
    if (counts) {
        if (lane == 0) red[threadIdx.x >> 6] = ones;
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long tot = red[0] + red[1] + red[2] + red[3];
            if (tot) atomicAdd(counts, tot);
        }
    }
}

}  // namespace binned
}  // namespace mjx

extern "C" int mjx_binned_plan_shape(int64_t n, int d, int64_t row_lo, int64_t row_hi, int64_t* slots,
                                     int64_t* segments) {
    using namespace mjx::binned;
    if (n < 1 || d < 1 || d > 16 || row_lo < 0 || row_hi > n || row_lo > row_hi || !slots || !segments)
        return MJX_EINVAL;
    if ((row_lo & 63) || ((row_hi & 63) && row_hi != n)) return MJX_EINVAL;
    *slots = (row_hi - row_lo) * d;
    *segments = nblocks(n) * ntiles(row_hi - row_lo);
    return MJX_OK;
}

extern "C" int mjx_binned_build(const int32_t* adj, int64_t n, int d, int64_t row_lo, int64_t row_hi, int32_t* src,
                                uint16_t* off, long long* seg_ptr, void* work, int64_t work_bytes, void* stream) {
    using namespace mjx::binned;
    if (n < 1 || d < 1 || d > 16 || row_lo < 0 || row_hi > n || row_lo > row_hi) return MJX_EINVAL;
    if ((row_lo & 63) || ((row_hi & 63) && row_hi != n)) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    const int64_t rows = row_hi - row_lo;
    if (rows == 0) return MJX_OK;
    if (!adj || !src || !off || !seg_ptr || !work) return MJX_EINVAL;
    const int64_t K = nblocks(n), T = ntiles(rows), S = K * T;
    if (K * 4 > 64 * 1024) return MJX_ERANGE;
    hipStream_t st = as_stream(stream);
    // counts into seg_ptr[0..S), then an in-place exclusive scan -> seg_ptr[0..S]
    MJX_HIP(hipMemsetAsync(seg_ptr + S, 0, sizeof(long long), st), "bin memset");
    k_bin_count<<<(unsigned)T, 256, K * sizeof(unsigned), st>>>(adj, rows, d, K, T, seg_ptr);
    MJX_LAUNCH_CHECK("k_bin_count");
    size_t need = 0;
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, need, seg_ptr, seg_ptr, S + 1, st), "bin scan size");
    if ((int64_t)need > work_bytes) return MJX_ERANGE;
    MJX_HIP(hipcub::DeviceScan::ExclusiveSum(work, need, seg_ptr, seg_ptr, S + 1, st), "bin scan");
    k_bin_fill<<<(unsigned)T, 256, K * sizeof(unsigned), st>>>(adj, rows, d, K, T, seg_ptr, src, off);
    MJX_LAUNCH_CHECK("k_bin_fill");
    return MJX_OK;
}

extern "C" int mjx_sweep_binned(const int32_t* src, const uint16_t* off, const long long* seg_ptr, int64_t n, int d,
                                int64_t row_lo, int64_t row_hi, const uint64_t* s_in, uint64_t* msg, uint64_t* s_out,
                                unsigned long long* counts, void* stream) {
    using namespace mjx::binned;
    if (n < 1 || d < 1 || d > 16 || row_lo < 0 || row_hi > n || row_lo > row_hi) return MJX_EINVAL;
    if (row_hi == row_lo) return MJX_OK;
    if ((row_lo & 63) || ((row_hi & 63) && row_hi != n)) return MJX_EINVAL;
    if (!src || !off || !seg_ptr || !s_in || !msg || !s_out || s_in == s_out) return MJX_EINVAL;
    const int64_t rows = row_hi - row_lo, slots = rows * d;
    const int64_t K = nblocks(n), T = ntiles(rows);
    hipStream_t st = as_stream(stream);
    k_bin_messages<<<grid_for(((slots + 63) / 64) * 64), 256, 0, st>>>(src, slots, (const uint32_t*)s_in, (u64*)msg);
    MJX_LAUNCH_CHECK("k_bin_messages");
    k_bin_update<<<(unsigned)T, 256, 0, st>>>(off, seg_ptr, (const u64*)msg, K, T, row_lo, row_hi, d,
                                             (const uint32_t*)s_in, (u64*)s_out, counts);
    MJX_LAUNCH_CHECK("k_bin_update");
    return MJX_OK;
}
