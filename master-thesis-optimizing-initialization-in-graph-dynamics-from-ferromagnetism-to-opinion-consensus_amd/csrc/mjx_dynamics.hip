// Majority-rule dynamics on bit-packed spins: pack/unpack, ELL (RRG) and CSR
// (Erdos-Renyi) rollouts, fused per-replica magnetisation counts.
//
// Semantics (M1/M2 of SURVEY.md 0.1): one synchronous step sets
//   s'_i = sign(S_i) if S_i != 0 else s_i,  S_i = sum_{k in N(i)} s_k
// (code/SA_RRG.py:18-20, code/HPR_pytorch_RRG.py:169-171, nb:113-117), and a
// rollout applies p+c-1 such steps (code/SA_RRG.py:23-26).  Integer exact, so
// the only thing parity depends on is the edge set.
//
// HBM-bound by design: per node and sweep the kernels read d int32 indices,
// gather d neighbour state rows, read the node's own row and write one row.
#include "mjx_common.h"
#include <algorithm>
#include <string.h>
#include <stdio.h>
#include <mutex>
#include <atomic>
#include <unordered_map>
#include <stdlib.h>
#include <math.h>

namespace mjx {

static thread_local char g_hip_err[256] = "";

void set_hip_error(hipError_t e, const char* where) {
    snprintf(g_hip_err, sizeof(g_hip_err), "%s: %s (%d)", where, hipGetErrorString(e), (int)e);
}

// Memo tables keyed by (device, pointer, two integers), in a hash map (no
// capacity limit: the keys are the library's kernels x the sizes a process
// uses).  `get`: a value computed once under the lock, failed computations not
// kept.  `raise_to`: the LARGEST value applied so far per (device, kernel); the
// setter runs only when a larger one is asked for (the dynamic-LDS opt-in is
// an upper bound, so a smaller later launch must never lower it: ADVICE r04).
struct DevMemo {
    struct Key {
        int dev; const void* k; int64_t a, b;
        bool operator==(const Key& o) const { return dev == o.dev && k == o.k && a == o.a && b == o.b; }
    };
    struct Hash {
        size_t operator()(const Key& x) const {
            uint64_t h = (uint64_t)(uintptr_t)x.k * 0x9E3779B97F4A7C15ull;
            h ^= ((uint64_t)x.a + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2));
            h ^= ((uint64_t)x.b * 0xBF58476D1CE4E5B9ull + (h << 6) + (h >> 2));
            h ^= (uint64_t)(uint32_t)x.dev * 0x94D049BB133111EBull;
            return (size_t)h;
        }
    };
    std::mutex mu;
    std::unordered_map<Key, int, Hash> e;
    template <typename F>
    int get(int dev, const void* k, int64_t a, int64_t b, F&& compute) {
        std::lock_guard<std::mutex> lock(mu);
        const Key key{dev, k, a, b};
        auto it = e.find(key);
        if (it != e.end()) return it->second;
        bool ok = true;
        const int v = compute(ok);
        if (ok) e.emplace(key, v);
        return v;
    }
    // setter(v) -> 0 on success; returns the setter's status (0 when no call was needed)
    template <typename F>
    int raise_to(int dev, const void* k, int v, F&& setter) {
        std::lock_guard<std::mutex> lock(mu);
        const Key key{dev, k, -1, -1};
        auto it = e.find(key);
        if (it != e.end() && it->second >= v) return 0;
        const int st = setter(v);
        if (st == 0) e[key] = v;
        return st;
    }
    size_t size() {
        std::lock_guard<std::mutex> lock(mu);
        return e.size();
    }
};

static int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = 0;
    }
    return dev;
}

static DevMemo& memo() {
    static DevMemo m;
    return m;
}

// CU count per device: read lock-free on every launch (0 = not yet known)
constexpr int kMaxDevices = 64;
static std::atomic<int> g_cus[kMaxDevices];

int device_cus() {
    const int dev = current_device();
    const int slot = (dev >= 0 && dev < kMaxDevices) ? dev : -1;
    if (slot >= 0) {
        const int v = g_cus[slot].load(std::memory_order_relaxed);
        if (v > 0) return v;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) {
        (void)hipGetLastError();
        return 256;                     // a whole MI355X (8 XCDs x 32 CUs); not kept, asked again
    }
    if (slot >= 0) g_cus[slot].store(cus, std::memory_order_relaxed);
    return cus;
}

hipError_t set_max_lds(const void* kernel, int bytes) {
    const int dev = current_device();
    return (hipError_t)memo().raise_to(dev, kernel, bytes, [&](int v) {
        return (int)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, v);
    });
}

int resident_blocks_per_cu(const void* kernel, int block, size_t lds) {
    const int dev = current_device();
    return memo().get(dev, kernel, block, (int64_t)lds, [&](bool& ok) {
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, lds) != hipSuccess || per < 1) {
            (void)hipGetLastError();
            ok = false;
            per = 1;
        }
        return per;
    });
}

}  // namespace mjx

// Host-only check of the memo logic (no HIP calls; tests/test_abi.py): values
// are computed once per (device, kernel, a, b), kept apart per device, and
// failed computations are retried.  0 = pass, else the number of the failed check.
extern "C" int mjx_selftest_devmemo(void) {
    mjx::DevMemo m;
    int calls = 0;
    const int k1 = 0, k2 = 0;
    auto f = [&](int v) { return [&calls, v](bool&) { ++calls; return v; }; };
    if (m.get(0, &k1, 1, 2, f(10)) != 10 || calls != 1) return 1;
    if (m.get(0, &k1, 1, 2, f(99)) != 10 || calls != 1) return 2;     // memoised
    if (m.get(1, &k1, 1, 2, f(20)) != 20 || calls != 2) return 3;     // another device: its own entry
    if (m.get(0, &k2, 1, 2, f(30)) != 30 || calls != 3) return 4;     // another kernel
    if (m.get(0, &k1, 1, 3, f(40)) != 40 || calls != 4) return 5;     // another size
    if (m.get(1, &k1, 1, 2, f(99)) != 20 || calls != 4) return 6;
    int tries = 0;
    auto bad = [&](bool& ok) { ++tries; ok = false; return 7; };
    m.get(2, &k1, 0, 0, bad);
    m.get(2, &k1, 0, 0, bad);
    if (tries != 2) return 7;                                          // failures are not kept
    // the LDS opt-in: n = 1e4, then 1e3, then 1e4 on one kernel
    int sets = 0, last = 0;
    auto setter = [&](int v) { ++sets; last = v; return 0; };
    if (m.raise_to(0, &k2, 138000, setter) != 0 || sets != 1 || last != 138000) return 8;
    if (m.raise_to(0, &k2, 14000, setter) != 0 || sets != 1) return 9;        // smaller: never lowered
    if (m.raise_to(0, &k2, 138000, setter) != 0 || sets != 1) return 10;      // still covered
    if (m.raise_to(0, &k2, 150000, setter) != 0 || sets != 2 || last != 150000) return 11;
    if (m.raise_to(1, &k2, 14000, setter) != 0 || sets != 3) return 12;       // per device
    auto fail = [&](int) { return 5; };
    if (m.raise_to(0, &k1, 9000, fail) != 5) return 13;
    if (m.raise_to(0, &k1, 9000, setter) != 0 || sets != 4) return 14;        // a failed set is retried
    // no capacity limit: 2000 distinct keys all kept
    const size_t before = m.size();
    for (int i = 0; i < 2000; ++i) m.get(3, &k1, i, 0, f(i));
    if (m.size() != before + 2000) return 15;
    const int c0 = calls;
    for (int i = 0; i < 2000; ++i)
        if (m.get(3, &k1, i, 0, f(-1)) != i) return 16;
    if (calls != c0) return 17;
    return 0;
}

namespace mjx {

// ---------------------------------------------------------------------------
// pack / unpack
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ bool is_plus(const T* s, int64_t i) { return s[i] > 0; }

template <typename T>
__global__ void __launch_bounds__(kBlock) k_pack_np(const T* __restrict__ s, int64_t n, u64* __restrict__ bits) {
    const int lane = threadIdx.x & 63;
    const int64_t nwords = (n + 63) >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t w = wave; w < nwords; w += nwaves) {
        int64_t v = (w << 6) + lane;
        bool b = (v < n) && is_plus(s, v);
        u64 word = __ballot(b);
        if (lane == 0) bits[w] = word;
    }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) k_unpack_np(const u64* __restrict__ bits, int64_t n, T* __restrict__ s) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < n; v += stride) {
        u64 w = bits[v >> 6];
        s[v] = ((w >> (v & 63)) & 1ull) ? T(1) : T(-1);
    }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) k_pack_rp(const T* __restrict__ s, int64_t n, int64_t R, int64_t W,
                                                    u64* __restrict__ bits) {
    const int64_t total = n * W;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += stride) {
        const int64_t v = t % n, w = t / n;   // node fastest: coalesced reads of s
        u64 word = 0;
        for (int b = 0; b < 64; ++b) {
            int64_t r = w * 64 + b;
            if (r < R && is_plus(s, r * n + v)) word |= (1ull << b);
        }
        bits[v * W + w] = word;
    }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) k_unpack_rp(const u64* __restrict__ bits, int64_t n, int64_t R, int64_t W,
                                                      T* __restrict__ s) {
    const int64_t total = n * W;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += stride) {
        const int64_t v = t % n, w = t / n;
        const u64 word = bits[v * W + w];
        for (int b = 0; b < 64; ++b) {
            int64_t r = w * 64 + b;
            if (r < R) s[r * n + v] = ((word >> b) & 1ull) ? T(1) : T(-1);
        }
    }
}

// ---------------------------------------------------------------------------
// per-thread vertical counter: counts, per bit position, the ones seen in the
// words added to it (bit-sliced ripple counter, KC planes, flushed to LDS
// before it can overflow).
// ---------------------------------------------------------------------------
constexpr int KC = 8;                 // planes -> up to 255 words between flushes
constexpr int kMaxLdsReplicas = 8192; // 32 KiB of LDS counters per block

template <int VW, int NK = KC>
struct VertCounter {
    static constexpr int KC = NK;
    u64 c[VW][KC];
    int added;
    __device__ __forceinline__ void reset() {
#pragma unroll
        for (int j = 0; j < VW; ++j)
#pragma unroll
            for (int p = 0; p < KC; ++p) c[j][p] = 0;
        added = 0;
    }
    __device__ __forceinline__ void add(const u64* x) {
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            u64 carry = x[j];
#pragma unroll
            for (int p = 0; p < KC; ++p) {
                u64 t = c[j][p] & carry;
                c[j][p] ^= carry;
                carry = t;
            }
        }
        ++added;
    }
    // add the per-bit counts into dst[j*64 + ((b + rot) & 63)] (LDS or global).
    // rot = the unit's index in the LDS block: lanes of consecutive units then
    // add into 64 different banks instead of all into bank b
    template <typename DST>
    __device__ __forceinline__ void flush(DST* dst, int rot = 0) {
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            for (int b = 0; b < 64; ++b) {
                unsigned cnt = 0;
#pragma unroll
                for (int p = 0; p < KC; ++p) cnt |= (unsigned)((c[j][p] >> b) & 1ull) << p;
                if (cnt) atomicAdd(&dst[j * 64 + ((b + rot) & 63)], (DST)cnt);
            }
        }
        reset();
    }
};

// ---------------------------------------------------------------------------
// node-packed (one replica) ELL sweep: a wave owns 64 consecutive nodes = one
// output word; each lane gathers its node's d neighbour bits.  Rows [v0, v1)
// are updated (v0 a multiple of 64); adj holds those rows only.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ void load_adj(const int32_t* __restrict__ adj, int64_t v, int32_t* k) {
    if constexpr (D == 4) {
        int4 a = *reinterpret_cast<const int4*>(adj + v * 4);
        k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
    } else if constexpr (D == 2) {
        int2 a = *reinterpret_cast<const int2*>(adj + v * 2);
        k[0] = a.x; k[1] = a.y;
    } else if constexpr (D == 6) {
        const int2* p = reinterpret_cast<const int2*>(adj + v * 6);
        int2 a = p[0], b = p[1], c = p[2];
        k[0] = a.x; k[1] = a.y; k[2] = b.x; k[3] = b.y; k[4] = c.x; k[5] = c.y;
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) k[j] = adj[v * D + j];
    }
}

__device__ __forceinline__ void block_count(unsigned long long ones, unsigned long long* counts) {
    __shared__ unsigned long long red[kBlock / 64];
    const int lane = threadIdx.x & 63;
    if (lane == 0) red[threadIdx.x >> 6] = ones;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < kBlock / 64; ++i) tot += red[i];
        if (tot) atomicAdd(counts, tot);
    }
}

template <int D>
__global__ void __launch_bounds__(kBlock) k_sweep_ell_np(const int32_t* __restrict__ adj, int64_t v0, int64_t v1,
                                                         const uint32_t* __restrict__ s_in32,
                                                         u64* __restrict__ s_out,
                                                         unsigned long long* __restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = v0 >> 6, w1 = (v1 + 63) >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    unsigned long long ones = 0;
    for (int64_t w = w0 + wave; w < w1; w += nwaves) {
        const int64_t v = (w << 6) + lane;
        bool nb = false;
        if (v < v1) {
            int32_t k[D];
            load_adj<D>(adj, v - v0, k);
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < D; ++j) cnt += (s_in32[k[j] >> 5] >> (k[j] & 31)) & 1u;
            const int own = (s_in32[v >> 5] >> (v & 31)) & 1u;
            nb = (2 * cnt > D) || ((2 * cnt == D) && own);
        }
        const u64 word = __ballot(nb);
        if (lane == 0) {
            s_out[w] = word;
            ones += __popcll(word);
        }
    }
    if (counts) block_count(ones, counts);
}

// runtime-degree node-packed ELL sweep (degrees other than the specialised ones)
__global__ void __launch_bounds__(kBlock) k_sweep_ell_np_dyn(const int32_t* __restrict__ adj, int64_t v0, int64_t v1,
                                                             int d, const uint32_t* __restrict__ s_in32,
                                                             u64* __restrict__ s_out,
                                                             unsigned long long* __restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = v0 >> 6, w1 = (v1 + 63) >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    unsigned long long ones = 0;
    for (int64_t w = w0 + wave; w < w1; w += nwaves) {
        const int64_t v = (w << 6) + lane;
        bool nb = false;
        if (v < v1) {
            int cnt = 0;
            for (int j = 0; j < d; ++j) {
                int32_t k = adj[(v - v0) * d + j];
                cnt += (s_in32[k >> 5] >> (k & 31)) & 1u;
            }
            const int own = (s_in32[v >> 5] >> (v & 31)) & 1u;
            nb = (2 * cnt > d) || ((2 * cnt == d) && own);
        }
        const u64 word = __ballot(nb);
        if (lane == 0) {
            s_out[w] = word;
            ones += __popcll(word);
        }
    }
    if (counts) block_count(ones, counts);
}

// node-packed CSR sweep (nb:113-117: sign(2S+s), same as always-stay)
__global__ void __launch_bounds__(kBlock) k_sweep_csr_np(const int64_t* __restrict__ row_ptr,
                                                         const int32_t* __restrict__ col, int64_t n,
                                                         const uint32_t* __restrict__ s_in32,
                                                         u64* __restrict__ s_out,
                                                         unsigned long long* __restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const int64_t nwords = (n + 63) >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    unsigned long long ones = 0;
    for (int64_t w = wave; w < nwords; w += nwaves) {
        const int64_t v = (w << 6) + lane;
        bool nb = false;
        if (v < n) {
            const int64_t b = row_ptr[v], e = row_ptr[v + 1];
            const int d = (int)(e - b);
            int cnt = 0;
            for (int64_t j = b; j < e; ++j) {
                int32_t k = col[j];
                cnt += (s_in32[k >> 5] >> (k & 31)) & 1u;
            }
            const int own = (s_in32[v >> 5] >> (v & 31)) & 1u;
            nb = (2 * cnt > d) || ((2 * cnt == d) && own);
        }
        const u64 word = __ballot(nb);
        if (lane == 0) {
            s_out[w] = word;
            ones += __popcll(word);
        }
    }
    if (counts) {
        __shared__ unsigned long long red[kBlock / 64];
        if (lane == 0) red[threadIdx.x >> 6] = ones;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long tot = 0;
            for (int i = 0; i < kBlock / 64; ++i) tot += red[i];
            if (tot) atomicAdd(counts, tot);
        }
    }
}

// ---------------------------------------------------------------------------
// replica-packed sweeps.  A node's W words are split into U = W/VW units of
// VW words (16-B loads when VW == 2).  Thread t owns unit t % U of the nodes
// slot, slot+slots, ... so its replica range is fixed (needed by the fused
// counter).
// ---------------------------------------------------------------------------
template <int VW> struct VecT;
template <> struct VecT<1> { typedef u64 T; };
template <> struct VecT<2> { typedef ulonglong2 T; };

template <int VW>
__device__ __forceinline__ void ldv(const u64* __restrict__ p, u64* x) {
    if constexpr (VW == 2) {
        ulonglong2 v = *reinterpret_cast<const ulonglong2*>(p);
        x[0] = v.x; x[1] = v.y;
    } else {
        x[0] = *p;
    }
}
template <int VW>
__device__ __forceinline__ void stv(u64* __restrict__ p, const u64* x) {
    if constexpr (VW == 2) {
        *reinterpret_cast<ulonglong2*>(p) = make_ulonglong2(x[0], x[1]);
    } else {
        *p = x[0];
    }
}

// A launch covers the units [unit0, unit0 + Us) of every node (a "slice" of
// the replicas); LDS counters are indexed relative to the slice.
template <int VW, int NK>
__device__ __forceinline__ void flush_to(VertCounter<VW, NK>& vc, int use_lds, unsigned* lds,
                                         unsigned long long* counts, int64_t unit, int64_t unit0) {
    if (use_lds) vc.flush(lds + (unit - unit0) * VW * 64, (int)((unit - unit0) & 63));
    else vc.flush(counts + unit * VW * 64);
}

template <int VW, int BS = kBlock>
__device__ __forceinline__ void lds_count_init(unsigned* lds, int64_t Us, bool use_lds) {
    if (use_lds) {
        for (int64_t r = threadIdx.x; r < Us * VW * 64; r += BS) lds[r] = 0;
        __syncthreads();
    }
}

// Shared epilogue for the fused per-replica counts.
template <int VW, bool COUNT, int BS = kBlock, int NK = KC>
__device__ __forceinline__ void count_epilogue(VertCounter<VW, NK>& vc, bool active, int64_t unit, int64_t unit0,
                                               int64_t Us, unsigned* lds, bool use_lds,
                                               unsigned long long* __restrict__ counts) {
    if constexpr (COUNT) {
        if (use_lds) {
            if (active && vc.added) vc.flush(lds + (unit - unit0) * VW * 64, (int)((unit - unit0) & 63));
            __syncthreads();  // every thread of the block reaches this (no early return)
            // undo the bank rotation; blocks start their walk at different
            // replicas so that blocks ending together do not queue their global
            // atomics on the same addresses
            const int64_t r0 = unit0 * VW * 64, tot = Us * VW * 64;
            const int64_t start = ((int64_t)blockIdx.x * BS) % tot;
            for (int64_t i = threadIdx.x; i < tot; i += BS) {
                int64_t r = start + i;
                if (r >= tot) r -= tot;
                const unsigned x = lds[r];
                if (x) {
                    const int64_t u = r / (VW * 64), rem = r - u * (VW * 64);
                    const int64_t b = ((rem & 63) - u) & 63;
                    atomicAdd(&counts[r0 + u * (VW * 64) + (rem & ~63LL) + b], (unsigned long long)x);
                }
            }
        } else {
            if (active && vc.added) vc.flush(counts + unit * VW * 64);
        }
    }
}

// BS: block size (a 1024-thread counting sweep, 4x fewer global count atomics,
// measured slower on MI355X: 537 vs 508 us at the bench size -- kept at 256).
template <int D, int VW, bool COUNT, int BS = kBlock>
__global__ void __launch_bounds__(BS) k_sweep_ell_rp(const int32_t* __restrict__ adj, int64_t n, int64_t W,
                                                     const u64* __restrict__ s_in, u64* __restrict__ s_out,
                                                     unsigned long long* __restrict__ counts, int use_lds,
                                                     int64_t unit0, int64_t Us) {
    extern __shared__ unsigned lds_cnt[];
    const int64_t t = (int64_t)blockIdx.x * BS + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * BS) / Us;
    const int64_t unit = unit0 + t % Us, slot = t / Us;
    const bool active = slot < slots;
    VertCounter<VW> vc;
    if constexpr (COUNT) {
        vc.reset();
        lds_count_init<VW, BS>(lds_cnt, Us, use_lds);
    }
    if (active) {
        for (int64_t v = slot; v < n; v += slots) {
            int32_t k[D];
            load_adj<D>(adj, v, k);
            u64 x[D][VW], own[VW], out[VW];
#pragma unroll
            for (int j = 0; j < D; ++j) ldv<VW>(s_in + (int64_t)k[j] * W + unit * VW, x[j]);
            ldv<VW>(s_in + v * W + unit * VW, own);
#pragma unroll
            for (int q = 0; q < VW; ++q) {
                u64 xs[D];
#pragma unroll
                for (int j = 0; j < D; ++j) xs[j] = x[j][q];
                out[q] = majority_fixed<D>(xs, own[q]);
            }
            stv<VW>(s_out + v * W + unit * VW, out);
            if constexpr (COUNT) {
                vc.add(out);
                if (vc.added == (1 << KC) - 1) flush_to(vc, use_lds, lds_cnt, counts, unit, unit0);
            }
        }
    }
    count_epilogue<VW, COUNT, BS>(vc, active, unit, unit0, Us, lds_cnt, use_lds, counts);
}

// runtime degree (ELL rows of length d) and CSR rows; KB counter planes
template <int VW, bool COUNT, bool CSR>
__global__ void __launch_bounds__(kBlock) k_sweep_gen_rp(const int32_t* __restrict__ adj, int d,
                                                         const int64_t* __restrict__ row_ptr,
                                                         const int32_t* __restrict__ col,
                                                         const int32_t* __restrict__ order, int64_t n, int64_t W,
                                                         const u64* __restrict__ s_in, u64* __restrict__ s_out,
                                                         unsigned long long* __restrict__ counts, int use_lds,
                                                         int64_t unit0, int64_t Us) {
    // order (nullable): node visiting order; sorted by degree it keeps the two
    // nodes a wave holds at one trip count (irregular ER rows)
    extern __shared__ unsigned lds_cnt[];
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * kBlock) / Us;
    const int64_t unit = unit0 + t % Us, slot = t / Us;
    const bool active = slot < slots;
    VertCounter<VW, 10> vc;     // up to 1023 nodes per thread between flushes (N = 1e7 rows)
    if constexpr (COUNT) {
        vc.reset();
        lds_count_init<VW>(lds_cnt, Us, use_lds);
    }
    if (active) {
        for (int64_t i = slot; i < n; i += slots) {
            const int64_t v = order ? (int64_t)order[i] : i;
            int64_t b, e;
            const int32_t* nbr;
            if constexpr (CSR) {
                b = row_ptr[v]; e = row_ptr[v + 1]; nbr = col;
            } else {
                b = v * d; e = b + d; nbr = adj;
            }
            const int deg = (int)(e - b);
            BitCounter<8> bc[VW];
#pragma unroll
            for (int q = 0; q < VW; ++q) bc[q].reset();
            // four gathers in flight per step (rows have d = 5 on average at C4)
            int64_t j = b;
            for (; j + 4 <= e; j += 4) {
                int32_t k[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) k[m] = nbr[j + m];
                u64 x[4][VW];
#pragma unroll
                for (int m = 0; m < 4; ++m) ldv<VW>(s_in + (int64_t)k[m] * W + unit * VW, x[m]);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int q = 0; q < VW; ++q) bc[q].add(x[m][q]);
            }
            if (j < e) {
                const int rest = (int)(e - j);
                int32_t k[3];
#pragma unroll
                for (int m = 0; m < 3; ++m) k[m] = m < rest ? nbr[j + m] : 0;
                u64 x[3][VW];
#pragma unroll
                for (int m = 0; m < 3; ++m)
                    if (m < rest) ldv<VW>(s_in + (int64_t)k[m] * W + unit * VW, x[m]);
#pragma unroll
                for (int m = 0; m < 3; ++m)
                    if (m < rest)
#pragma unroll
                        for (int q = 0; q < VW; ++q) bc[q].add(x[m][q]);
            }
            u64 own[VW], out[VW];
            ldv<VW>(s_in + v * W + unit * VW, own);
#pragma unroll
            for (int q = 0; q < VW; ++q) out[q] = bc[q].majority(deg, own[q]);
            stv<VW>(s_out + v * W + unit * VW, out);
            if constexpr (COUNT) {
                vc.add(out);
                if (vc.added == (1 << decltype(vc)::KC) - 1) flush_to(vc, use_lds, lds_cnt, counts, unit, unit0);
            }
        }
    }
    count_epilogue<VW, COUNT, kBlock, 10>(vc, active, unit, unit0, Us, lds_cnt, use_lds, counts);
}

// ---------------------------------------------------------------------------
// Degree-class ELL sweep: the notebook's own ER layout (nb:113-117 sums
// s[N_nodes_pos[d]] over the nodes nodes_with_d_positions[d] of each degree
// class d; nb:359-361 builds them).  One launch per class: its `cnt` nodes
// order[0..cnt) all have degree D and node order[k]'s neighbours are
// cell[k*D .. k*D+D).  Against the CSR sweep this drops the row_ptr hop (the
// chain is order/cell -> gather, as for the RRG) and, with D a template
// parameter, the runtime bit counter (88 -> fewer VGPRs, more waves in
// flight for a latency-bound gather).  D = -1: runtime degree `dd` (> 8).
// ---------------------------------------------------------------------------
// One node of a degree class: position i of the class (order = the class's
// node list, cell = its neighbour rows), new bits of this thread's unit into
// out[] and s_out.
template <int D, int VW>
__device__ __forceinline__ void cls_node(const int32_t* __restrict__ order, const int32_t* __restrict__ cell,
                                         int64_t i, int dd, int64_t W, const u64* __restrict__ s_in,
                                         u64* __restrict__ s_out, int64_t unit, u64* out) {
    const int64_t v = order[i];
    u64 own[VW];
    if constexpr (D == 0) {
        // no neighbours: S = 0, a tie, the spin stays (nb:113-117)
        ldv<VW>(s_in + v * W + unit * VW, out);
    } else if constexpr (D > 0) {
        int32_t k[D];
        load_adj<D>(cell, i, k);
        u64 x[D][VW];
#pragma unroll
        for (int j = 0; j < D; ++j) ldv<VW>(s_in + (int64_t)k[j] * W + unit * VW, x[j]);
        ldv<VW>(s_in + v * W + unit * VW, own);
#pragma unroll
        for (int q = 0; q < VW; ++q) {
            u64 xs[D];
#pragma unroll
            for (int j = 0; j < D; ++j) xs[j] = x[j][q];
            out[q] = majority_fixed<D>(xs, own[q]);
        }
    } else {
        const int32_t* row = cell + i * dd;
        BitCounter<8> bc[VW];
#pragma unroll
        for (int q = 0; q < VW; ++q) bc[q].reset();
        int j = 0;
        for (; j + 4 <= dd; j += 4) {
            int32_t k[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) k[m] = row[j + m];
            u64 x[4][VW];
#pragma unroll
            for (int m = 0; m < 4; ++m) ldv<VW>(s_in + (int64_t)k[m] * W + unit * VW, x[m]);
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int q = 0; q < VW; ++q) bc[q].add(x[m][q]);
        }
        for (; j < dd; ++j) {
            u64 x[VW];
            ldv<VW>(s_in + (int64_t)row[j] * W + unit * VW, x);
#pragma unroll
            for (int q = 0; q < VW; ++q) bc[q].add(x[q]);
        }
        ldv<VW>(s_in + v * W + unit * VW, own);
#pragma unroll
        for (int q = 0; q < VW; ++q) out[q] = bc[q].majority(dd, own[q]);
    }
    stv<VW>(s_out + v * W + unit * VW, out);
}

template <int D, int VW, bool COUNT, int NK = KC>
__global__ void __launch_bounds__(kBlock) k_sweep_cls_rp(const int32_t* __restrict__ order,
                                                         const int32_t* __restrict__ cell, int64_t cnt, int dd,
                                                         int64_t W, const u64* __restrict__ s_in,
                                                         u64* __restrict__ s_out,
                                                         unsigned long long* __restrict__ counts, int use_lds,
                                                         int64_t unit0, int64_t Us) {
    extern __shared__ unsigned lds_cnt[];
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * kBlock) / Us;
    const int64_t unit = unit0 + t % Us, slot = t / Us;
    const bool active = slot < slots;
    VertCounter<VW, NK> vc;
    if constexpr (COUNT) {
        vc.reset();
        lds_count_init<VW>(lds_cnt, Us, use_lds);
    }
    if (active) {
        for (int64_t i = slot; i < cnt; i += slots) {
            u64 out[VW];
            cls_node<D, VW>(order, cell, i, dd, W, s_in, s_out, unit, out);
            if constexpr (COUNT) {
                vc.add(out);
                if (vc.added == (1 << NK) - 1) flush_to(vc, use_lds, lds_cnt, counts, unit, unit0);
            }
        }
    }
    count_epilogue<VW, COUNT, kBlock, NK>(vc, active, unit, unit0, Us, lds_cnt, use_lds, counts);
}

// The counting sweep of a rollout over the degree classes D <= 8 in one
// launch: a thread walks its positions of the class-sorted node order with a
// forward class cursor and runs the class's node body.  The per-class launches
// each paid the count epilogue (Us*VW*64 global atomics per block, 40-100 us
// per launch at R = 4096, profiles/r04_bench_kernel_stats.csv); here it is
// paid once for them.  No runtime-degree body (the D > 8 tail keeps its own
// table launch) and 6 counter planes (a flush every 63 nodes): 90 VGPRs,
// 5 waves per SIMD (with both: 124, 4 waves).
constexpr int kMaxCls = 9;
#ifndef MJX_CLS_ALL_NK
#define MJX_CLS_ALL_NK 6
#endif
constexpr int kClsAllPlanes = MJX_CLS_ALL_NK;
struct ClsTable {
    int nc;
    int D[kMaxCls];
    int64_t i0[kMaxCls + 1];   // class c = positions [i0[c], i0[c+1]) of order
    int64_t base[kMaxCls];     // its cell rows start at cell + base[c]
};

template <int VW>
__global__ void __launch_bounds__(kBlock) k_sweep_cls_all_rp(const int32_t* __restrict__ order,
                                                             const int32_t* __restrict__ cell, ClsTable tab,
                                                             int64_t W, const u64* __restrict__ s_in,
                                                             u64* __restrict__ s_out,
                                                             unsigned long long* __restrict__ counts, int use_lds,
                                                             int64_t Us) {
    extern __shared__ unsigned lds_cnt[];
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * kBlock) / Us;
    const int64_t unit = t % Us, slot = t / Us;
    const bool active = slot < slots;
    VertCounter<VW, kClsAllPlanes> vc;
    vc.reset();
    lds_count_init<VW>(lds_cnt, Us, use_lds);
    if (active) {
        int c = 0;
        for (int64_t i = tab.i0[0] + slot; i < tab.i0[tab.nc]; i += slots) {
            while (i >= tab.i0[c + 1]) ++c;
            const int32_t* o = order + tab.i0[c];
            const int32_t* cl = cell + tab.base[c];
            const int64_t r = i - tab.i0[c];
            u64 out[VW];
            switch (tab.D[c]) {
                case 0: cls_node<0, VW>(o, cl, r, 0, W, s_in, s_out, unit, out); break;
                case 1: cls_node<1, VW>(o, cl, r, 1, W, s_in, s_out, unit, out); break;
                case 2: cls_node<2, VW>(o, cl, r, 2, W, s_in, s_out, unit, out); break;
                case 3: cls_node<3, VW>(o, cl, r, 3, W, s_in, s_out, unit, out); break;
                case 4: cls_node<4, VW>(o, cl, r, 4, W, s_in, s_out, unit, out); break;
                case 5: cls_node<5, VW>(o, cl, r, 5, W, s_in, s_out, unit, out); break;
                case 6: cls_node<6, VW>(o, cl, r, 6, W, s_in, s_out, unit, out); break;
                case 7: cls_node<7, VW>(o, cl, r, 7, W, s_in, s_out, unit, out); break;
                case 8: cls_node<8, VW>(o, cl, r, 8, W, s_in, s_out, unit, out); break;
                default: __builtin_unreachable();        // the host passes D <= 8 only
            }
            vc.add(out);
            if (vc.added == (1 << kClsAllPlanes) - 1) flush_to(vc, use_lds, lds_cnt, counts, unit, 0);
        }
    }
    count_epilogue<VW, true, kBlock, kClsAllPlanes>(vc, active, unit, 0, Us, lds_cnt, use_lds, counts);
}

// The classes above D = 8 (few nodes each: Poisson tail) in one launch: a
// table of consecutive classes, each thread walks its positions in increasing
// order with a forward class cursor.  One launch (and one count epilogue)
// instead of one per class.
constexpr int kMaxGen = 32;
struct GenTable {
    int nc;
    int D[kMaxGen];
    int64_t i0[kMaxGen + 1];   // positions relative to the first class; i0[nc] = end
    int64_t base[kMaxGen];
};

template <int VW, bool COUNT>
__global__ void __launch_bounds__(kBlock) k_sweep_cls_gen_rp(const int32_t* __restrict__ order,
                                                             const int32_t* __restrict__ cell, GenTable tab,
                                                             int64_t W, const u64* __restrict__ s_in,
                                                             u64* __restrict__ s_out,
                                                             unsigned long long* __restrict__ counts, int use_lds,
                                                             int64_t Us) {
    extern __shared__ unsigned lds_cnt[];
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * kBlock) / Us;
    const int64_t unit = t % Us, slot = t / Us;
    const bool active = slot < slots;
    VertCounter<VW> vc;
    if constexpr (COUNT) {
        vc.reset();
        lds_count_init<VW>(lds_cnt, Us, use_lds);
    }
    if (active) {
        int c = 0;
        for (int64_t i = slot; i < tab.i0[tab.nc]; i += slots) {
            while (i >= tab.i0[c + 1]) ++c;
            const int dd = tab.D[c];
            const int32_t* row = cell + tab.base[c] + (i - tab.i0[c]) * dd;
            const int64_t v = order[i];
            BitCounter<8> bc[VW];
#pragma unroll
            for (int q = 0; q < VW; ++q) bc[q].reset();
            int j = 0;
            for (; j + 4 <= dd; j += 4) {
                int32_t k[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) k[m] = row[j + m];
                u64 x[4][VW];
#pragma unroll
                for (int m = 0; m < 4; ++m) ldv<VW>(s_in + (int64_t)k[m] * W + unit * VW, x[m]);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int q = 0; q < VW; ++q) bc[q].add(x[m][q]);
            }
            for (; j < dd; ++j) {
                u64 x[VW];
                ldv<VW>(s_in + (int64_t)row[j] * W + unit * VW, x);
#pragma unroll
                for (int q = 0; q < VW; ++q) bc[q].add(x[q]);
            }
            u64 own[VW], out[VW];
            ldv<VW>(s_in + v * W + unit * VW, own);
#pragma unroll
            for (int q = 0; q < VW; ++q) out[q] = bc[q].majority(dd, own[q]);
            stv<VW>(s_out + v * W + unit * VW, out);
            if constexpr (COUNT) {
                vc.add(out);
                if (vc.added == (1 << KC) - 1) flush_to(vc, use_lds, lds_cnt, counts, unit, 0);
            }
        }
    }
    count_epilogue<VW, COUNT>(vc, active, unit, 0, Us, lds_cnt, use_lds, counts);
}

// Gather floor of the degree-class sweep (bench `er.floor_ms`, VERDICT r05
// item 5): the same positions, class-ELL rows, unit mapping and resident grid
// as the sweeps, the same rows moved -- a position's D neighbour rows, its own
// row where D is even (a tie is possible), one row written -- with no majority:
// the rows' XOR is written instead.  Eight gathers in flight per thread and
// few VGPRs (more waves than any sweep), so it is what the random 512-B rows
// of the C4 state cost on this device, not a kernel's choice.
template <int VW>
__global__ void __launch_bounds__(kBlock) k_gather_floor_cls(const int32_t* __restrict__ order,
                                                             const int32_t* __restrict__ cell, GenTable tab,
                                                             int64_t W, const u64* __restrict__ s_in,
                                                             u64* __restrict__ s_out, int64_t Us) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * kBlock) / Us;
    const int64_t unit = t % Us, slot = t / Us;
    if (slot >= slots) return;
    int c = 0;
    for (int64_t i = slot; i < tab.i0[tab.nc]; i += slots) {
        while (i >= tab.i0[c + 1]) ++c;
        const int dd = tab.D[c];
        const int32_t* row = cell + tab.base[c] + (i - tab.i0[c]) * dd;
        const int64_t v = order[i];
        u64 acc[VW];
        if (dd % 2 == 0) ldv<VW>(s_in + v * W + unit * VW, acc);
        else {
#pragma unroll
            for (int q = 0; q < VW; ++q) acc[q] = 0;
        }
        for (int j = 0; j < dd; j += 8) {
            int32_t k[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) k[m] = (j + m < dd) ? row[j + m] : -1;
            u64 x[8][VW];
#pragma unroll
            for (int m = 0; m < 8; ++m)
                if (k[m] >= 0) ldv<VW>(s_in + (int64_t)k[m] * W + unit * VW, x[m]);
#pragma unroll
            for (int m = 0; m < 8; ++m)
                if (k[m] >= 0)
#pragma unroll
                    for (int q = 0; q < VW; ++q) acc[q] ^= x[m][q];
        }
        stv<VW>(s_out + v * W + unit * VW, acc);
    }
}

// Fills the class-ELL cells of one class from CSR: cell[k*D + j] =
// col[row_ptr[order[k]] + j], k < cnt.
__global__ void __launch_bounds__(kBlock) k_class_ell_fill(const int64_t* __restrict__ row_ptr,
                                                           const int32_t* __restrict__ col,
                                                           const int32_t* __restrict__ order, int64_t cnt, int D,
                                                           int32_t* __restrict__ cell) {
    const int64_t total = cnt * D;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += (int64_t)gridDim.x * kBlock) {
        const int64_t k = e / D, j = e - k * D;
        cell[e] = col[row_ptr[order[k]] + j];
    }
}

}  // namespace mjx

// ---------------------------------------------------------------------------
// standalone per-replica popcount
// ---------------------------------------------------------------------------
namespace mjx {

__global__ void __launch_bounds__(kBlock) k_popcount_np(const u64* __restrict__ bits, int64_t n,
                                                        unsigned long long* __restrict__ counts) {
    const int64_t nwords = (n + 63) >> 6;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    unsigned long long ones = 0;
    for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < nwords; w += stride) {
        u64 x = bits[w];
        if (w == nwords - 1 && (n & 63)) x &= (1ull << (n & 63)) - 1ull;  // padding nodes
        ones += __popcll(x);
    }
    // wave reduction then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) ones += __shfl_down(ones, off, 64);
    if ((threadIdx.x & 63) == 0 && ones) atomicAdd(counts, ones);
}

template <int VW>
__global__ void __launch_bounds__(kBlock) k_popcount_rp(const u64* __restrict__ bits, int64_t n, int64_t W,
                                                        unsigned long long* __restrict__ counts, int use_lds) {
    extern __shared__ unsigned lds_cnt[];
    const int64_t U = W / VW;
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t slots = ((int64_t)gridDim.x * kBlock) / U;
    const int64_t unit = t % U, slot = t / U;
    const bool active = slot < slots;
    VertCounter<VW> vc;
    vc.reset();
    lds_count_init<VW>(lds_cnt, U, use_lds);
    if (active) {
        for (int64_t v = slot; v < n; v += slots) {
            u64 x[VW];
            ldv<VW>(bits + v * W + unit * VW, x);
            vc.add(x);
            if (vc.added == (1 << KC) - 1) flush_to(vc, use_lds, lds_cnt, counts, unit, 0);
        }
    }
    count_epilogue<VW, true>(vc, active, unit, 0, U, lds_cnt, use_lds, counts);
}

}  // namespace mjx

// ===========================================================================
// C ABI
// ===========================================================================
using namespace mjx;

extern "C" int mjx_abi_version(void) { return 2; }

extern "C" const char* mjx_strerror(int status) {
    switch (status) {
        case MJX_OK: return "ok";
        case MJX_EINVAL: return "invalid argument";
        case MJX_EHIP: return "HIP runtime error";
        case MJX_ERANGE: return "size out of supported range";
        default: return "unknown status";
    }
}

extern "C" const char* mjx_last_hip_error(void) { return g_hip_err; }

template <typename F8, typename F32, typename F64>
static int dispatch_dtype(int dtype, F8 f8, F32 f32, F64 f64) {
    switch (dtype) {
        case MJX_I8: return f8();
        case MJX_I32: return f32();
        case MJX_I64: return f64();
        default: return MJX_EINVAL;
    }
}

extern "C" int mjx_pack_np(const void* s, int dtype, int64_t n, uint64_t* bits, void* stream) {
    if (n < 0 || (n > 0 && (!s || !bits))) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    const int64_t nwords = (n + 63) / 64;
    const int grid = grid_for(nwords * 64);
    hipStream_t st = as_stream(stream);
    int rc = dispatch_dtype(dtype,
        [&] { k_pack_np<int8_t><<<grid, kBlock, 0, st>>>((const int8_t*)s, n, (u64*)bits); return 0; },
        [&] { k_pack_np<int32_t><<<grid, kBlock, 0, st>>>((const int32_t*)s, n, (u64*)bits); return 0; },
        [&] { k_pack_np<int64_t><<<grid, kBlock, 0, st>>>((const int64_t*)s, n, (u64*)bits); return 0; });
    if (rc) return rc;
    MJX_LAUNCH_CHECK("mjx_pack_np");
    return MJX_OK;
}

extern "C" int mjx_unpack_np(const uint64_t* bits, int64_t n, void* s, int dtype, void* stream) {
    if (n < 0 || (n > 0 && (!s || !bits))) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    const int grid = grid_for(n);
    hipStream_t st = as_stream(stream);
    int rc = dispatch_dtype(dtype,
        [&] { k_unpack_np<int8_t><<<grid, kBlock, 0, st>>>((const u64*)bits, n, (int8_t*)s); return 0; },
        [&] { k_unpack_np<int32_t><<<grid, kBlock, 0, st>>>((const u64*)bits, n, (int32_t*)s); return 0; },
        [&] { k_unpack_np<int64_t><<<grid, kBlock, 0, st>>>((const u64*)bits, n, (int64_t*)s); return 0; });
    if (rc) return rc;
    MJX_LAUNCH_CHECK("mjx_unpack_np");
    return MJX_OK;
}

extern "C" int mjx_pack_rp(const void* s, int dtype, int64_t n, int64_t R, uint64_t* bits, void* stream) {
    if (n < 0 || R < 1 || (n > 0 && (!s || !bits))) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    const int64_t W = (R + 63) / 64;
    const int grid = grid_for(n * W);
    hipStream_t st = as_stream(stream);
    int rc = dispatch_dtype(dtype,
        [&] { k_pack_rp<int8_t><<<grid, kBlock, 0, st>>>((const int8_t*)s, n, R, W, (u64*)bits); return 0; },
        [&] { k_pack_rp<int32_t><<<grid, kBlock, 0, st>>>((const int32_t*)s, n, R, W, (u64*)bits); return 0; },
        [&] { k_pack_rp<int64_t><<<grid, kBlock, 0, st>>>((const int64_t*)s, n, R, W, (u64*)bits); return 0; });
    if (rc) return rc;
    MJX_LAUNCH_CHECK("mjx_pack_rp");
    return MJX_OK;
}

extern "C" int mjx_unpack_rp(const uint64_t* bits, int64_t n, int64_t R, void* s, int dtype, void* stream) {
    if (n < 0 || R < 1 || (n > 0 && (!s || !bits))) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    const int64_t W = (R + 63) / 64;
    const int grid = grid_for(n * W);
    hipStream_t st = as_stream(stream);
    int rc = dispatch_dtype(dtype,
        [&] { k_unpack_rp<int8_t><<<grid, kBlock, 0, st>>>((const u64*)bits, n, R, W, (int8_t*)s); return 0; },
        [&] { k_unpack_rp<int32_t><<<grid, kBlock, 0, st>>>((const u64*)bits, n, R, W, (int32_t*)s); return 0; },
        [&] { k_unpack_rp<int64_t><<<grid, kBlock, 0, st>>>((const u64*)bits, n, R, W, (int64_t*)s); return 0; });
    if (rc) return rc;
    MJX_LAUNCH_CHECK("mjx_unpack_rp");
    return MJX_OK;
}

// ---- sweep launchers -------------------------------------------------------

static int launch_sweep_ell_np(const int32_t* adj, int64_t v0, int64_t v1, int d, const u64* in, u64* out,
                               unsigned long long* counts, hipStream_t st) {
    const int64_t nwords = ((v1 + 63) >> 6) - (v0 >> 6);
    const int grid = grid_for(nwords * 64);
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
    switch (d) {
        case 3: k_sweep_ell_np<3><<<grid, kBlock, 0, st>>>(adj, v0, v1, in32, out, counts); break;
        case 4: k_sweep_ell_np<4><<<grid, kBlock, 0, st>>>(adj, v0, v1, in32, out, counts); break;
        case 6: k_sweep_ell_np<6><<<grid, kBlock, 0, st>>>(adj, v0, v1, in32, out, counts); break;
        default: k_sweep_ell_np_dyn<<<grid, kBlock, 0, st>>>(adj, v0, v1, d, in32, out, counts); break;
    }
    MJX_LAUNCH_CHECK("sweep_ell_np");
    return MJX_OK;
}

static int launch_sweep_csr_np(const int64_t* rp, const int32_t* col, int64_t n, const u64* in, u64* out,
                               unsigned long long* counts, hipStream_t st) {
    const int64_t nwords = (n + 63) / 64;
    const int grid = grid_for(nwords * 64);
    k_sweep_csr_np<<<grid, kBlock, 0, st>>>(rp, col, n, reinterpret_cast<const uint32_t*>(in), out, counts);
    MJX_LAUNCH_CHECK("sweep_csr_np");
    return MJX_OK;
}

constexpr int kCountBlock = kBlock;

template <int VW, bool COUNT>
static void launch_ell_rp_vw(const int32_t* adj, int64_t n, int d, int64_t W, const u64* in, u64* out,
                             unsigned long long* counts, int grid, size_t lds, int use_lds, int64_t unit0,
                             int64_t Us, hipStream_t st) {
    constexpr int BS = COUNT ? kCountBlock : kBlock;
    (void)grid;
    auto ell = [&](auto kern) {
        const int g = resident_grid(kern, BS, lds, n * Us);
        kern<<<g, BS, lds, st>>>(adj, n, W, in, out, counts, use_lds, unit0, Us);
    };
    switch (d) {
        case 3: ell(k_sweep_ell_rp<3, VW, COUNT, BS>); break;
        case 4: ell(k_sweep_ell_rp<4, VW, COUNT, BS>); break;
        case 6: ell(k_sweep_ell_rp<6, VW, COUNT, BS>); break;
        default: {
            auto kern = k_sweep_gen_rp<VW, COUNT, false>;
            const int g = resident_grid(kern, kBlock, lds, n * Us);
            kern<<<g, kBlock, lds, st>>>(adj, d, nullptr, nullptr, nullptr, n, W, in, out, counts, use_lds, unit0, Us);
            break;
        }
    }
}

// Geometry of one launch over Us units (of VW words) of every node.
static int rp_geometry(int64_t n, int64_t W, int64_t Us, int* grid, int* vw, int* use_lds, size_t* lds) {
    *vw = (W % 2 == 0) ? 2 : 1;
    *grid = grid_for(n * Us);
    const int64_t threads = (int64_t)(*grid) * kBlock;
    if (threads / Us < 1) return MJX_ERANGE;
    *use_lds = (Us * (*vw) * 64 <= kMaxLdsReplicas) ? 1 : 0;
    *lds = *use_lds ? (size_t)(Us * (*vw) * 64 * sizeof(unsigned)) : 0;
    return MJX_OK;
}

// Replica slices of a replica-packed rollout: slice q covers units
// [q*U/S, (q+1)*U/S).  Replicas never interact, so a rollout can run slice by
// slice; a slice's state (n * W/S words) is small enough to stay in the 256 MB
// Infinity Cache between the sweeps that re-read it.
static int64_t units_of(int64_t W) { return (W % 2 == 0) ? W / 2 : W; }

// Measured on MI355X (tools/slice_sweep.py, profiles/r01_slice_sweep.log): at
// N=1e6, R=4096 one slice (512-B rows) runs at 6.2 TB/s, 2 slices at 6.1, 4 at
// 4.9, 8 at 2.8 -- shorter contiguous gathers cost more than the Infinity Cache
// returns -- so the automatic choice is a single slice.
static int auto_slices(int64_t, int64_t) { return 1; }

static int launch_sweep_ell_rp(const int32_t* adj, int64_t n, int d, int64_t W, const u64* in, u64* out,
                               unsigned long long* counts, int64_t unit0, int64_t Us, hipStream_t st) {
    int grid, vw, use_lds; size_t lds;
    int rc = rp_geometry(n, W, Us, &grid, &vw, &use_lds, &lds);
    if (rc) return rc;
    if (!counts) { lds = 0; use_lds = 0; }
    if (vw == 2) {
        if (counts) launch_ell_rp_vw<2, true>(adj, n, d, W, in, out, counts, grid, lds, use_lds, unit0, Us, st);
        else launch_ell_rp_vw<2, false>(adj, n, d, W, in, out, counts, grid, lds, use_lds, unit0, Us, st);
    } else {
        if (counts) launch_ell_rp_vw<1, true>(adj, n, d, W, in, out, counts, grid, lds, use_lds, unit0, Us, st);
        else launch_ell_rp_vw<1, false>(adj, n, d, W, in, out, counts, grid, lds, use_lds, unit0, Us, st);
    }
    MJX_LAUNCH_CHECK("sweep_ell_rp");
    return MJX_OK;
}

static int launch_sweep_csr_rp(const int64_t* rp, const int32_t* col, const int32_t* order, int64_t n, int64_t W,
                               const u64* in, u64* out, unsigned long long* counts, int64_t unit0, int64_t Us,
                               hipStream_t st) {
    int grid, vw, use_lds; size_t lds;
    int rc = rp_geometry(n, W, Us, &grid, &vw, &use_lds, &lds);
    if (rc) return rc;
    if (!counts) { lds = 0; use_lds = 0; }
#define MJX_CSR(VWV, C)                                                                                      \
    do {                                                                                                     \
        auto kern = k_sweep_gen_rp<VWV, C, true>;                                                            \
        grid = resident_grid(kern, kBlock, lds, n * Us);                                                     \
        kern<<<grid, kBlock, lds, st>>>(nullptr, 0, rp, col, order, n, W, in, out, counts, use_lds, unit0, Us); \
    } while (0)
    if (vw == 2) {
        if (counts) MJX_CSR(2, true); else MJX_CSR(2, false);
    } else {
        if (counts) MJX_CSR(1, true); else MJX_CSR(1, false);
    }
#undef MJX_CSR
    MJX_LAUNCH_CHECK("sweep_csr_rp");
    return MJX_OK;
}

// Runs `steps` sweeps in -> ... -> out, ping-ponging through tmp so that the
// last sweep writes `out`; the fused count rides on the last sweep.
template <typename SWEEP>
static int run_rollout(int steps, const u64* in, u64* out, u64* tmp, unsigned long long* counts, SWEEP sweep) {
    if (steps < 1) return MJX_EINVAL;
    if (steps >= 2 && !tmp) return MJX_EINVAL;
    const u64* src = in;
    for (int k = 0; k < steps; ++k) {
        u64* dst = (((steps - 1 - k) & 1) == 0) ? out : tmp;
        int rc = sweep(src, dst, (k == steps - 1) ? counts : nullptr);
        if (rc) return rc;
        src = dst;
    }
    return MJX_OK;
}

extern "C" int mjx_popcount_np(const uint64_t* bits, int64_t n, unsigned long long* counts, void* stream) {
    if (n < 0 || !counts || (n > 0 && !bits)) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    const int64_t nwords = (n + 63) / 64;
    k_popcount_np<<<grid_for(nwords), kBlock, 0, as_stream(stream)>>>((const u64*)bits, n, counts);
    MJX_LAUNCH_CHECK("mjx_popcount_np");
    return MJX_OK;
}

extern "C" int mjx_popcount_rp(const uint64_t* bits, int64_t n, int64_t words, unsigned long long* counts,
                               void* stream) {
    if (n < 0 || words < 1 || !counts || (n > 0 && !bits)) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    int grid, vw, use_lds; size_t lds;
    int rc = rp_geometry(n, words, units_of(words), &grid, &vw, &use_lds, &lds);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    if (vw == 2) k_popcount_rp<2><<<grid, kBlock, lds, st>>>((const u64*)bits, n, words, counts, use_lds);
    else k_popcount_rp<1><<<grid, kBlock, lds, st>>>((const u64*)bits, n, words, counts, use_lds);
    MJX_LAUNCH_CHECK("mjx_popcount_rp");
    return MJX_OK;
}

static bool overlaps(const void* a, const void* b) { return a && b && a == b; }

extern "C" int mjx_rollout_ell_np(const int32_t* adj, int64_t n, int d, const uint64_t* s_in, uint64_t* s_out,
                                  uint64_t* tmp, int steps, unsigned long long* counts, void* stream) {
    if (n < 0 || d < 0 || d > 255 || (n > 0 && (!adj && d > 0)) || (n > 0 && (!s_in || !s_out))) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out) || overlaps(s_in, tmp) || overlaps(s_out, tmp)) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    hipStream_t st = as_stream(stream);
    const size_t bytes = (size_t)((n + 63) / 64) * 8;
    auto sweep = [&](const u64* a, u64* b, unsigned long long* c) {
        return launch_sweep_ell_np(adj, 0, n, d, a, b, c, st);
    };
    if (steps < 0) return MJX_EINVAL;
    if (steps == 0) {
        MJX_HIP(hipMemcpyAsync(s_out, s_in, bytes, hipMemcpyDeviceToDevice, st), "rollout copy");
        return counts ? mjx_popcount_np(s_out, n, counts, stream) : MJX_OK;
    }
    return run_rollout(steps, (const u64*)s_in, (u64*)s_out, (u64*)tmp, counts, sweep);
}

extern "C" int mjx_sweep_ell_np_range(const int32_t* adj, int64_t n, int d, int64_t row_lo, int64_t row_hi,
                                      const uint64_t* s_in, uint64_t* s_out, unsigned long long* counts,
                                      void* stream) {
    if (n < 1 || d < 0 || d > 255 || row_lo < 0 || row_hi > n || row_lo > row_hi) return MJX_EINVAL;
    if (row_hi == row_lo) return MJX_OK;                       // a rank without rows
    if ((row_lo & 63) || ((row_hi & 63) && row_hi != n)) return MJX_EINVAL;
    if (!s_in || !s_out || (row_hi > row_lo && d > 0 && !adj) || overlaps(s_in, s_out)) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    return launch_sweep_ell_np(adj, row_lo, row_hi, d, (const u64*)s_in, (u64*)s_out, counts, as_stream(stream));
}

extern "C" int mjx_rollout_ell_rp_sliced(const int32_t* adj, int64_t n, int d, int64_t words, const uint64_t* s_in,
                                         uint64_t* s_out, uint64_t* tmp, int steps, int slices,
                                         unsigned long long* counts, void* stream) {
    if (n < 0 || d < 0 || d > 255 || words < 1 || slices < 0 || (n > 0 && (!s_in || !s_out || (!adj && d > 0))))
        return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out) || overlaps(s_in, tmp) || overlaps(s_out, tmp)) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    hipStream_t st = as_stream(stream);
    const size_t bytes = (size_t)n * (size_t)words * 8;
    if (steps < 0) return MJX_EINVAL;
    if (steps == 0) {
        MJX_HIP(hipMemcpyAsync(s_out, s_in, bytes, hipMemcpyDeviceToDevice, st), "rollout copy");
        return counts ? mjx_popcount_rp(s_out, n, words, counts, stream) : MJX_OK;
    }
    const int64_t U = units_of(words);
    const int S = slices ? slices : auto_slices(n, words);
    if (S < 1 || U % S) return MJX_EINVAL;
    const int64_t Us = U / S;
    for (int q = 0; q < S; ++q) {
        auto sweep = [&](const u64* a, u64* b, unsigned long long* c) {
            return launch_sweep_ell_rp(adj, n, d, words, a, b, c, q * Us, Us, st);
        };
        int rc = run_rollout(steps, (const u64*)s_in, (u64*)s_out, (u64*)tmp, counts, sweep);
        if (rc) return rc;
    }
    return MJX_OK;
}

// One synchronous sweep with a graph per replica (code/SA_RRG.py:58-62 draws a
// graph per replica; the sweep itself is code/SA_RRG.py:18-20).  Lane = replica
// r of word column w = blockIdx.y, each wave strides over nodes; a lane gathers
// the d neighbour words of ITS graph and keeps its own bit, the wave's 64 new
// bits are one ballot.  Setup-path kernel (initial levels of distinct-graph SA
// replicas): d random 8-B loads per replica-node, not the bit-parallel sweep.
template <bool COUNT>
__global__ void __launch_bounds__(kBlock) k_sweep_multi_rp(const int32_t* __restrict__ adj, int64_t n, int d,
                                                           int64_t R, int64_t W, const int32_t* __restrict__ rep_graph,
                                                           const u64* __restrict__ s_in, u64* __restrict__ s_out,
                                                           unsigned long long* __restrict__ counts) {
    const int lane = threadIdx.x & 63;
    const int64_t w = blockIdx.y;
    const int64_t r = w * 64 + lane;
    const bool live = r < R;
    const int32_t* a = adj + (live ? (int64_t)rep_graph[r] : 0) * n * d;
    const u64 bit = 1ull << lane;
    const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
    unsigned long long cnt = 0;
    for (int64_t v = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); v < n; v += waves) {
        bool nb = false;
        if (live) {
            int ones = 0;
            for (int j = 0; j < d; ++j) ones += (s_in[(int64_t)a[v * d + j] * W + w] & bit) ? 1 : 0;
            const bool own = (s_in[v * W + w] & bit) != 0;
            nb = (2 * ones > d) ? true : ((2 * ones < d) ? false : own);     // always-stay majority
        }
        const u64 word = __ballot(nb);
        if (lane == 0) s_out[v * W + w] = word;
        if constexpr (COUNT) cnt += nb ? 1 : 0;
    }
    if constexpr (COUNT) {
        if (live && cnt) atomicAdd(&counts[r], cnt);
    }
}

extern "C" int mjx_rollout_ell_rp_multi(const int32_t* adj, int64_t n, int d, int64_t R, const int32_t* rep_graph,
                                        const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp, int steps,
                                        unsigned long long* counts, void* stream) {
    if (n < 1 || d < 1 || d > 255 || R < 1 || !adj || !rep_graph || !s_in || !s_out || steps < 1) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out) || overlaps(s_in, tmp) || overlaps(s_out, tmp)) return MJX_EINVAL;
    const int64_t W = (R + 63) / 64;
    if (W > 65535) return MJX_ERANGE;
    hipStream_t st = as_stream(stream);
    int64_t gx = (n + 3) / 4;
    const int64_t cap = std::max<int64_t>(1, (int64_t)device_cus() * 8 / W);
    if (gx > cap) gx = cap;
    const dim3 grid((unsigned)gx, (unsigned)W);
    auto sweep = [&](const u64* a, u64* b, unsigned long long* c) -> int {
        if (c) k_sweep_multi_rp<true><<<grid, kBlock, 0, st>>>(adj, n, d, R, W, rep_graph, a, b, c);
        else k_sweep_multi_rp<false><<<grid, kBlock, 0, st>>>(adj, n, d, R, W, rep_graph, a, b, nullptr);
        MJX_LAUNCH_CHECK("k_sweep_multi_rp");
        return MJX_OK;
    };
    return run_rollout(steps, (const u64*)s_in, (u64*)s_out, (u64*)tmp, counts, sweep);
}

extern "C" int mjx_rollout_ell_rp(const int32_t* adj, int64_t n, int d, int64_t words, const uint64_t* s_in,
                                  uint64_t* s_out, uint64_t* tmp, int steps, unsigned long long* counts,
                                  void* stream) {
    return mjx_rollout_ell_rp_sliced(adj, n, d, words, s_in, s_out, tmp, steps, 0, counts, stream);
}

extern "C" int mjx_rollout_csr_np(const int64_t* row_ptr, const int32_t* col, int64_t n, const uint64_t* s_in,
                                  uint64_t* s_out, uint64_t* tmp, int steps, unsigned long long* counts,
                                  void* stream) {
    if (n < 0 || (n > 0 && (!row_ptr || !s_in || !s_out))) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out) || overlaps(s_in, tmp) || overlaps(s_out, tmp)) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    hipStream_t st = as_stream(stream);
    const size_t bytes = (size_t)((n + 63) / 64) * 8;
    if (steps < 0) return MJX_EINVAL;
    if (steps == 0) {
        MJX_HIP(hipMemcpyAsync(s_out, s_in, bytes, hipMemcpyDeviceToDevice, st), "rollout copy");
        return counts ? mjx_popcount_np(s_out, n, counts, stream) : MJX_OK;
    }
    auto sweep = [&](const u64* a, u64* b, unsigned long long* c) {
        return launch_sweep_csr_np(row_ptr, col, n, a, b, c, st);
    };
    return run_rollout(steps, (const u64*)s_in, (u64*)s_out, (u64*)tmp, counts, sweep);
}

extern "C" int mjx_rollout_csr_rp_ordered(const int64_t* row_ptr, const int32_t* col, const int32_t* order,
                                          int64_t n, int64_t words, const uint64_t* s_in, uint64_t* s_out,
                                          uint64_t* tmp, int steps, unsigned long long* counts, void* stream) {
    if (n < 0 || words < 1 || (n > 0 && (!row_ptr || !s_in || !s_out))) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out) || overlaps(s_in, tmp) || overlaps(s_out, tmp)) return MJX_EINVAL;
    if (n == 0) return MJX_OK;
    hipStream_t st = as_stream(stream);
    const size_t bytes = (size_t)n * (size_t)words * 8;
    if (steps < 0) return MJX_EINVAL;
    if (steps == 0) {
        MJX_HIP(hipMemcpyAsync(s_out, s_in, bytes, hipMemcpyDeviceToDevice, st), "rollout copy");
        return counts ? mjx_popcount_rp(s_out, n, words, counts, stream) : MJX_OK;
    }
    const int64_t U = units_of(words);
    const int S = auto_slices(n, words);
    const int64_t Us = U / S;
    for (int q = 0; q < S; ++q) {
        auto sweep = [&](const u64* a, u64* b, unsigned long long* c) {
            return launch_sweep_csr_rp(row_ptr, col, order, n, words, a, b, c, q * Us, Us, st);
        };
        int rc = run_rollout(steps, (const u64*)s_in, (u64*)s_out, (u64*)tmp, counts, sweep);
        if (rc) return rc;
    }
    return MJX_OK;
}

// ---- degree-class ELL ------------------------------------------------------

static int check_classes(const int64_t* classes, int nclasses, int64_t n) {
    if (nclasses < 0 || (nclasses > 0 && !classes)) return MJX_EINVAL;
    int64_t covered = 0;
    for (int c = 0; c < nclasses; ++c) {
        const int64_t i0 = classes[4 * c], cnt = classes[4 * c + 1], D = classes[4 * c + 2], base = classes[4 * c + 3];
        if (i0 < 0 || cnt < 0 || i0 + cnt > n || D < 0 || D > 255 || base < 0 || (base & 3)) return MJX_EINVAL;
        covered += cnt;
    }
    return covered == n ? MJX_OK : MJX_EINVAL;
}

extern "C" int mjx_class_ell_fill(const int64_t* row_ptr, const int32_t* col, const int32_t* order,
                                  const int64_t* classes, int nclasses, int64_t n, int32_t* cell, void* stream) {
    if (n < 0 || (n > 0 && (!row_ptr || !order))) return MJX_EINVAL;
    int rc = check_classes(classes, nclasses, n);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    for (int c = 0; c < nclasses; ++c) {
        const int64_t i0 = classes[4 * c], cnt = classes[4 * c + 1], D = classes[4 * c + 2], base = classes[4 * c + 3];
        if (cnt * D == 0) continue;
        if (!col || !cell) return MJX_EINVAL;
        k_class_ell_fill<<<grid_for(cnt * D), kBlock, 0, st>>>(row_ptr, col, order + i0, cnt, (int)D, cell + base);
        MJX_LAUNCH_CHECK("class_ell_fill");
    }
    return MJX_OK;
}

// Counting launches end with Us*VW*64 global count atomics per block (4096
// at R = 4096, ~100 us for a 2048-block grid): a small class gets at most one
// block per kClsCountNodes nodes per thread slot.
constexpr int64_t kClsCountNodes = 16;
static int64_t cls_count_threads(int64_t cnt, int64_t Us) {
    const int64_t slots = (cnt + kClsCountNodes - 1) / kClsCountNodes;
    return (slots < 1 ? 1 : slots) * Us;
}

template <int VW, bool COUNT>
static int launch_sweep_cls_gen_rp(const int32_t* order, const int32_t* cell, const GenTable& tab, int64_t W,
                                   const u64* in, u64* out, unsigned long long* counts, size_t lds, int use_lds,
                                   int64_t Us, hipStream_t st) {
    auto kern = k_sweep_cls_gen_rp<VW, COUNT>;
    const int64_t cnt = tab.i0[tab.nc];
    const int g = resident_grid(kern, kBlock, lds, COUNT ? cls_count_threads(cnt, Us) : cnt * Us);
    kern<<<g, kBlock, lds, st>>>(order, cell, tab, W, in, out, counts, use_lds, Us);
    MJX_LAUNCH_CHECK("sweep_cls_gen_rp");
    return MJX_OK;
}

template <int VW, bool COUNT>
static int launch_sweep_cls_rp(const int32_t* order, const int32_t* cell, int64_t cnt, int D, int64_t W,
                               const u64* in, u64* out, unsigned long long* counts, size_t lds, int use_lds,
                               int64_t unit0, int64_t Us, hipStream_t st) {
    auto go = [&](auto kern) {
        const int g = resident_grid(kern, kBlock, lds, COUNT ? cls_count_threads(cnt, Us) : cnt * Us);
        kern<<<g, kBlock, lds, st>>>(order, cell, cnt, D, W, in, out, counts, use_lds, unit0, Us);
    };
#define MJX_CLS(DD) go(k_sweep_cls_rp<DD, VW, COUNT>)
    switch (D) {
        case 0: MJX_CLS(0); break;
        case 1: MJX_CLS(1); break;
        case 2: MJX_CLS(2); break;
        case 3: MJX_CLS(3); break;
        case 4: MJX_CLS(4); break;
        case 5: MJX_CLS(5); break;
        case 6: MJX_CLS(6); break;
        case 7: MJX_CLS(7); break;
        case 8: MJX_CLS(8); break;
        default: MJX_CLS(-1); break;
    }
#undef MJX_CLS
    MJX_LAUNCH_CHECK("sweep_cls_rp");
    return MJX_OK;
}

extern "C" int mjx_rollout_class_rp(const int32_t* order, const int32_t* cell, const int64_t* classes,
                                    int nclasses, int64_t n, int64_t words, const uint64_t* s_in,
                                    uint64_t* s_out, uint64_t* tmp, int steps, unsigned long long* counts,
                                    void* stream) {
    if (n < 0 || words < 1 || (n > 0 && (!order || !s_in || !s_out))) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out) || overlaps(s_in, tmp) || overlaps(s_out, tmp)) return MJX_EINVAL;
    int rc = check_classes(classes, nclasses, n);
    if (rc) return rc;
    if (n == 0) return MJX_OK;
    for (int c = 0; c < nclasses; ++c)
        if (classes[4 * c + 1] * classes[4 * c + 2] > 0 && !cell) return MJX_EINVAL;
    hipStream_t st = as_stream(stream);
    if (steps < 0) return MJX_EINVAL;
    if (steps == 0) {
        MJX_HIP(hipMemcpyAsync(s_out, s_in, (size_t)n * (size_t)words * 8, hipMemcpyDeviceToDevice, st),
                "rollout copy");
        return counts ? mjx_popcount_rp(s_out, n, words, counts, stream) : MJX_OK;
    }
    const int64_t Us = units_of(words);
    int grid, vw, use_lds; size_t lds;
    rc = rp_geometry(n, words, Us, &grid, &vw, &use_lds, &lds);
    if (rc) return rc;
    // the counting sweep of the leading classes with D <= 8 that tile `order`
    // from position 0 in one launch (-DMJX_CLS_PER_LAUNCH: the per-class
    // counting launches, for timing A/B); the rest as below
    ClsTable all{};
    int lead = 0;
#ifndef MJX_CLS_PER_LAUNCH
    for (int64_t pos = 0; lead < nclasses && lead < kMaxCls; ++lead) {
        const int64_t* cl = classes + 4 * lead;
        if (cl[0] != pos || cl[2] > 8 || (cl[1] * cl[2] > 0 && !cell)) break;
        all.D[lead] = (int)cl[2];
        all.i0[lead] = cl[0];
        all.base[lead] = cl[3];
        pos = cl[0] + cl[1];
    }
#endif
    all.nc = lead;
    all.i0[lead] = lead ? all.i0[lead - 1] + classes[4 * (lead - 1) + 1] : 0;
    auto sweep = [&](const u64* a, u64* b, unsigned long long* cn) {
        const int c0 = (cn && lead >= 2) ? lead : 0;
        if (c0) {
            auto go = [&](auto kern) {
                const int g = resident_grid(kern, kBlock, lds, n * Us);
                kern<<<g, kBlock, lds, st>>>(order, cell, all, words, a, b, cn, use_lds, Us);
            };
            if (vw == 2) go(k_sweep_cls_all_rp<2>);
            else go(k_sweep_cls_all_rp<1>);
            MJX_LAUNCH_CHECK("sweep_cls_all_rp");
        }
        // runs of consecutive classes with D > 8 (adjacent in `order`) share one launch
        GenTable tab{};
        int64_t g0 = 0;
        auto flush_gen = [&]() -> int {
            if (tab.nc == 0) return MJX_OK;
            const int32_t* o = order + g0;
            int r;
            if (vw == 2) r = cn ? launch_sweep_cls_gen_rp<2, true>(o, cell, tab, words, a, b, cn, lds, use_lds, Us, st)
                                : launch_sweep_cls_gen_rp<2, false>(o, cell, tab, words, a, b, cn, 0, 0, Us, st);
            else r = cn ? launch_sweep_cls_gen_rp<1, true>(o, cell, tab, words, a, b, cn, lds, use_lds, Us, st)
                        : launch_sweep_cls_gen_rp<1, false>(o, cell, tab, words, a, b, cn, 0, 0, Us, st);
            tab.nc = 0;
            return r;
        };
        for (int c = c0; c < nclasses; ++c) {
            const int64_t i0 = classes[4 * c], cnt = classes[4 * c + 1], base = classes[4 * c + 3];
            const int D = (int)classes[4 * c + 2];
            if (cnt == 0) continue;
            if (D > 8) {
                if (tab.nc > 0 && (tab.nc == kMaxGen || g0 + tab.i0[tab.nc] != i0)) {
                    int r = flush_gen();
                    if (r) return r;
                }
                if (tab.nc == 0) { g0 = i0; tab.i0[0] = 0; }
                tab.D[tab.nc] = D;
                tab.base[tab.nc] = base;
                tab.i0[tab.nc + 1] = i0 - g0 + cnt;
                ++tab.nc;
                continue;
            }
            const int32_t* o = order + i0;
            const int32_t* cl = cell ? cell + base : nullptr;
            int r;
            if (vw == 2) r = cn ? launch_sweep_cls_rp<2, true>(o, cl, cnt, D, words, a, b, cn, lds, use_lds, 0, Us, st)
                                : launch_sweep_cls_rp<2, false>(o, cl, cnt, D, words, a, b, cn, 0, 0, 0, Us, st);
            else r = cn ? launch_sweep_cls_rp<1, true>(o, cl, cnt, D, words, a, b, cn, lds, use_lds, 0, Us, st)
                        : launch_sweep_cls_rp<1, false>(o, cl, cnt, D, words, a, b, cn, 0, 0, 0, Us, st);
            if (r) return r;
        }
        return flush_gen();
    };
    return run_rollout(steps, (const u64*)s_in, (u64*)s_out, (u64*)tmp, counts, sweep);
}

extern "C" int mjx_gather_floor_class(const int32_t* order, const int32_t* cell, const int64_t* classes,
                                      int nclasses, int64_t n, int64_t words, const uint64_t* s_in, uint64_t* s_out,
                                      void* stream) {
    if (n < 1 || words < 1 || !order || !cell || !s_in || !s_out) return MJX_EINVAL;
    if (n > (int64_t)INT32_MAX) return MJX_ERANGE;
    if (overlaps(s_in, s_out)) return MJX_EINVAL;
    int rc = check_classes(classes, nclasses, n);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    const int64_t Us = units_of(words);
    int grid, vw, use_lds; size_t lds;
    rc = rp_geometry(n, words, Us, &grid, &vw, &use_lds, &lds);
    if (rc) return rc;
    // consecutive classes (adjacent in `order`), kMaxGen at a time
    for (int c0 = 0; c0 < nclasses;) {
        GenTable tab{};
        const int64_t g0 = classes[4 * c0];
        tab.i0[0] = 0;
        int c = c0;
        for (; c < nclasses && tab.nc < kMaxGen && classes[4 * c] == g0 + tab.i0[tab.nc]; ++c) {
            tab.D[tab.nc] = (int)classes[4 * c + 2];
            tab.base[tab.nc] = classes[4 * c + 3];
            tab.i0[tab.nc + 1] = tab.i0[tab.nc] + classes[4 * c + 1];
            ++tab.nc;
        }
        auto go = [&](auto kern) {
            const int g = resident_grid(kern, kBlock, 0, tab.i0[tab.nc] * Us);
            kern<<<g, kBlock, 0, st>>>(order + g0, cell, tab, words, (const u64*)s_in, (u64*)s_out, Us);
        };
        if (vw == 2) go(k_gather_floor_cls<2>);
        else go(k_gather_floor_cls<1>);
        MJX_LAUNCH_CHECK("gather_floor_cls");
        c0 = c;
    }
    return MJX_OK;
}

extern "C" int mjx_rollout_csr_rp(const int64_t* row_ptr, const int32_t* col, int64_t n, int64_t words,
                                  const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp, int steps,
                                  unsigned long long* counts, void* stream) {
    return mjx_rollout_csr_rp_ordered(row_ptr, col, nullptr, n, words, s_in, s_out, tmp, steps, counts, stream);
}
