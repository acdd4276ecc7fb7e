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

// One twist of a 624-word MT19937 state held in LDS, by one wave.  The
// recurrence has three dependency phases (words [0, 227) read only old words,
// [227, 454) read phase 1's new words, [454, 623) phase 2's, then word 623);
// within a phase every read is issued before any write (a chunk's last lane
// reads the next chunk's first word, still old), so a phase is one LDS round
// trip of reads and one of writes.
__device__ inline void lds_twist(uint32_t* buf, int lane) {
    constexpr int P1 = MT_N - MT_M;                  // 227
    uint32_t v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = lane + 64 * c;
        if (k < P1) v[c] = mt_mix(buf[k], buf[k + 1], buf[k + MT_M]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = lane + 64 * c;
        if (k < P1) buf[k] = v[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = P1 + lane + 64 * c;
        if (k < 2 * P1) v[c] = mt_mix(buf[k], buf[k + 1], buf[k - P1]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = P1 + lane + 64 * c;
        if (k < 2 * P1) buf[k] = v[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int k = 2 * P1 + lane + 64 * c;
        if (k < MT_N - 1) v[c] = mt_mix(buf[k], buf[k + 1], buf[k - P1]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int k = 2 * P1 + lane + 64 * c;
        if (k < MT_N - 1) buf[k] = v[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) buf[MT_N - 1] = mt_mix(buf[MT_N - 1], buf[0], buf[MT_M - 1]);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// numpy's proposal draws in a window of 64 tempered words (code/SA_RRG.py:73,
// 76: randint(0, n)'s masked rejection, then rand()'s two words): a proposal
// starts at the first acceptable word at or after the previous proposal's end.
// Scanning left to right is a 3-state automaton (0 = looking for an acceptable
// word, 1 and 2 = inside rand()'s words; an acceptable word in state 0 starts a
// proposal), so the starts come from a parallel prefix of its transition
// functions (each a map {0,1,2} -> {0,1,2} packed as three 2-bit fields):
// four DPP row shifts and two row broadcasts, no serial walk.  Lane l starts a
// proposal iff the state after word l, from state 0 at the window's start, is 1.
__device__ __forceinline__ uint32_t mt_walk_compose(uint32_t g, uint32_t h) {   // x -> g(h(x))
    return ((g >> (2 * (h & 3u))) & 3u) | (((g >> (2 * ((h >> 2) & 3u))) & 3u) << 2) |
           (((g >> (2 * ((h >> 4) & 3u))) & 3u) << 4);
}
__device__ __forceinline__ unsigned long long mt_window_starts(bool ok) {
    constexpr uint32_t ID = 0u | (1u << 2) | (2u << 4);
    uint32_t f = ok ? (1u | (2u << 2)) : (2u << 2);          // ok: 0->1, 1->2, 2->0; else 0->0, 1->2, 2->0
    f = mt_walk_compose(f, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)f, 0x111, 0xf, 0xf, false));  // row_shr:1
    f = mt_walk_compose(f, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)f, 0x112, 0xf, 0xf, false));  // row_shr:2
    f = mt_walk_compose(f, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)f, 0x114, 0xf, 0xf, false));  // row_shr:4
    f = mt_walk_compose(f, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)f, 0x118, 0xf, 0xf, false));  // row_shr:8
    f = mt_walk_compose(f, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)f, 0x142, 0xa, 0xf, false));  // row_bcast:15
    f = mt_walk_compose(f, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)f, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return __ballot((f & 3u) == 1u);
}
// lane l + 1's value (wave_shl:1; lane 63 gets 0)
__device__ __forceinline__ uint32_t mt_next_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

}  // namespace mjx
