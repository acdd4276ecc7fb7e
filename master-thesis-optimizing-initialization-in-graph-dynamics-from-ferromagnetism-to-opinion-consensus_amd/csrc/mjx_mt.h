// MT19937 pieces shared by the SA translation units: numpy's legacy global
// stream (np.random.seed / randint / rand / binomial) is
// replayed exactly on the device (code/SA_RRG.py:65,73,76).
#pragma once
#include "mjx_common.h"

namespace mjx {

constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr uint32_t MT_MATRIX_A = 0x9908b0dfu;
constexpr uint32_t MT_UPPER = 0x80000000u;
constexpr uint32_t MT_LOWER = 0x7fffffffu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
    uint32_t y = (cur & MT_UPPER) | (nxt & MT_LOWER);
    return far ^ (y >> 1) ^ ((y & 1u) ? MT_MATRIX_A : 0u);
}

__device__ __forceinline__ double mt_double(uint32_t w1, uint32_t w2) {
    return ((double)(w1 >> 5) * 67108864.0 + (double)(w2 >> 6)) / 9007199254740992.0;
}

// One twist of a 624-word MT19937 state held in LDS, by one wave (the three
// dependency phases of the recurrence, wave-scope fences between the reads
// and writes of a phase).
__device__ inline void lds_twist(uint32_t* buf, int lane) {
    for (int k = lane; k < MT_N - MT_M; k += 64) {
        const uint32_t v = mt_mix(buf[k], buf[k + 1], buf[k + MT_M]);
        __builtin_amdgcn_wave_barrier();
        buf[k] = v;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    for (int k = MT_N - MT_M + lane; k < 2 * (MT_N - MT_M); k += 64) {
        const uint32_t v = mt_mix(buf[k], buf[k + 1], buf[k + MT_M - MT_N]);
        __builtin_amdgcn_wave_barrier();
        buf[k] = v;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    for (int k = 2 * (MT_N - MT_M) + lane; k < MT_N - 1; k += 64) {
        const uint32_t v = mt_mix(buf[k], buf[k + 1], buf[k + MT_M - MT_N]);
        __builtin_amdgcn_wave_barrier();
        buf[k] = v;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) buf[MT_N - 1] = mt_mix(buf[MT_N - 1], buf[0], buf[MT_M - 1]);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}


}  // namespace mjx
