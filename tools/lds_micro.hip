// Micro-benchmarks behind the level-synchronous SA kernel's design (k_sa_lds_cu):
// the cost of a 16-wave workgroup barrier and of one dependent LDS round trip
// (read, returning atomic) on gfx950, in shader clocks (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_micro tools/lds_micro.hip   (CPU)
//   ./tools/lds_micro                                                          (GPU)
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

// mode 0: barrier only; 1: barrier + one dependent LDS read (every wave);
// 2: dependent LDS read chain, no barrier; 3: dependent returning LDS atomic chain;
// 4: barrier + a wave-0-only dependent chain of 6 reads (the others wait)
__global__ void __launch_bounds__(1024) k_micro(int mode, int nwaves, unsigned long long* out) {
    __shared__ unsigned int buf[4096];
    const int tid = threadIdx.x;
    for (int q = tid; q < 4096; q += blockDim.x) buf[q] = (unsigned)((q * 37 + 11) & 4095);
    __syncthreads();
    unsigned int x = tid & 4095;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        if (mode == 0) {
            __syncthreads();
        } else if (mode == 1) {
            x = buf[x];
            __syncthreads();
        } else if (mode == 2) {
            x = buf[x];
        } else if (mode == 3) {
            x = atomicAdd(&buf[x & 4095], 1u) & 4095u;
        } else {
            if ((tid >> 6) == 0) {
#pragma unroll
                for (int q = 0; q < 6; ++q) x = buf[x];
            }
            __syncthreads();
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) out[blockIdx.x] = t1 - t0;
    if (x == 0xffffffffu) out[1] = x;           // keep the chain live
}

int main() {
    unsigned long long* d;
    (void)hipMalloc(&d, 1024 * sizeof(unsigned long long));
    const char* names[] = {"barrier", "barrier + 1 dependent read", "dependent read", "dependent returning atomic",
                           "barrier + 6 dependent reads in wave 0"};
    for (int mode = 0; mode < 2; ++mode)
        for (int nw : {1, 2, 4, 8, 16}) {
            hipLaunchKernelGGL(k_micro, dim3(256), dim3(64 * nw), 0, 0, mode, nw, d);
            hipLaunchKernelGGL(k_micro, dim3(256), dim3(64 * nw), 0, 0, mode, nw, d);
            unsigned long long h[256];
            (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            double s = 0;
            for (int b = 0; b < 256; ++b) s += (double)h[b];
            printf("%-40s %2d waves: %.1f clocks per iteration\n", names[mode], nw, s / 256 / ITERS);
        }
    return 0;
}
