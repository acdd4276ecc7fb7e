// Shared helpers for the libmjx HIP translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/mjx.h"

namespace mjx {

typedef unsigned long long u64;

// Records the text of the last failing HIP call (read via mjx_last_hip_error).
void set_hip_error(hipError_t e, const char* where);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-check: kernel launches are asynchronous; only the launch itself is
// checked here (no device synchronisation inside any entry point).
#define MJX_LAUNCH_CHECK(where)                                   \
    do {                                                          \
        hipError_t _e = hipGetLastError();                        \
        if (_e != hipSuccess) { mjx::set_hip_error(_e, where); return MJX_EHIP; } \
    } while (0)

#define MJX_HIP(call, where)                                      \
    do {                                                          \
        hipError_t _e = (call);                                   \
        if (_e != hipSuccess) { mjx::set_hip_error(_e, where); return MJX_EHIP; } \
    } while (0)

constexpr int kBlock = 256;          // 4 waves of 64

// Per-device facts and one-time settings, memoised per (device, kernel, ...):
// a library caller may drive several devices (or a partitioned GPU) from one
// process, so nothing here is a process-wide constant.
int device_cus();                                        // CUs of the current device (256 on a whole MI355X)
hipError_t set_max_lds(const void* kernel, int bytes);   // opt in to `bytes` of dynamic LDS, once per device
template <typename K>
inline hipError_t set_max_lds(K* kernel, int bytes) {
    return set_max_lds(reinterpret_cast<const void*>(kernel), bytes);
}

inline int grid_for(int64_t items, int per_cu = 8) {
    int64_t g = (items + kBlock - 1) / kBlock;
    int64_t cap = (int64_t)device_cus() * per_cu;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

// Blocks of `kernel` (with `lds` dynamic LDS bytes) resident on one CU at once,
// memoised per (device, kernel, block, lds); thread-safe.
int resident_blocks_per_cu(const void* kernel, int block, size_t lds);

// Grid for a grid-stride loop over `items` threads' worth of work, capped at
// what is resident on the chip at once.  A larger grid runs in rounds over a
// fixed node partition, and the last round is partly empty: the 141-VGPR
// counting CSR sweep holds 3 waves per SIMD, so an 8-per-SIMD grid ran in
// 3 rounds (the last 2/3 full).
template <typename K>
inline int resident_grid(K* kernel, int block, size_t lds, int64_t items) {
    int per = resident_blocks_per_cu(reinterpret_cast<const void*>(kernel), block, lds);
    int64_t g = (items + block - 1) / block;
    const int64_t cap = (int64_t)device_cus() * per;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

// Bit-sliced majority with always-stay tie breaking (code/SA_RRG.py:19-20):
// new = +1 if 2*cnt > d, -1 if 2*cnt < d, old if 2*cnt == d, where cnt is the
// number of +1 neighbours.  Every bit lane of a word is an independent node
// (np layout) or replica (rp layout).
template <int D>
__device__ __forceinline__ u64 majority_fixed(const u64* x, u64 own) {
    if constexpr (D == 1) {
        return x[0];
    } else if constexpr (D == 2) {
        return (x[0] & x[1]) | ((x[0] ^ x[1]) & own);
    } else if constexpr (D == 3) {
        return (x[0] & x[1]) | (x[2] & (x[0] | x[1]));
    } else if constexpr (D == 4) {
        // ge3 = at least three ones; ge2 = at least two ones
        u64 ab_and = x[0] & x[1], ab_or = x[0] | x[1];
        u64 cd_and = x[2] & x[3], cd_or = x[2] | x[3];
        u64 ge3 = (ab_and & cd_or) | (cd_and & ab_or);
        u64 ge2 = ab_and | cd_and | (ab_or & cd_or);
        return ge3 | (ge2 & own);
    } else {
        // generic: bit-sliced ripple counter then compare with d/2
        constexpr int K = (D < 2) ? 1 : (D < 4) ? 2 : (D < 8) ? 3 : (D < 16) ? 4 : (D < 32) ? 5 : (D < 64) ? 6 : 7;
        u64 c[K];
#pragma unroll
        for (int p = 0; p < K; ++p) c[p] = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            u64 carry = x[j];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                u64 t = c[p] & carry;
                c[p] ^= carry;
                carry = t;
            }
        }
        constexpr int H = D / 2;     // compare cnt with floor(d/2)
        u64 gt = 0, eq = ~0ull;
#pragma unroll
        for (int p = K - 1; p >= 0; --p) {
            if ((H >> p) & 1) {
                eq &= c[p];
            } else {
                gt |= eq & c[p];
                eq &= ~c[p];
            }
        }
        if constexpr ((D & 1) == 0) return gt | (eq & own);
        else return gt;  // odd degree: 2*cnt == d impossible (eq means cnt == floor(d/2) -> minority)
    }
}

// Runtime-degree version for CSR rows (nb:113-117, sign(2S+s)): counter with
// KB bit planes (degree <= 2^KB - 1).
template <int KB>
struct BitCounter {
    u64 c[KB];
    __device__ __forceinline__ void reset() {
#pragma unroll
        for (int p = 0; p < KB; ++p) c[p] = 0;
    }
    __device__ __forceinline__ void add(u64 x) {
        u64 carry = x;
#pragma unroll
        for (int p = 0; p < KB; ++p) {
            u64 t = c[p] & carry;
            c[p] ^= carry;
            carry = t;
        }
    }
    // new spin word for a node of degree `deg`
    __device__ __forceinline__ u64 majority(int deg, u64 own) const {
        const int h = deg >> 1;
        u64 gt = 0, eq = ~0ull;
#pragma unroll
        for (int p = KB - 1; p >= 0; --p) {
            if ((h >> p) & 1) {
                eq &= c[p];
            } else {
                gt |= eq & c[p];
                eq &= ~c[p];
            }
        }
        // cnt == floor(d/2): for even d a tie (keep own), for odd d a loss
        return (deg & 1) ? gt : (gt | (eq & own));
    }
};

}  // namespace mjx
