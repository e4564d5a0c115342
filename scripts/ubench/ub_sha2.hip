// ub_sha2.hip — one vs two interleaved rng_spawn chains per lane
// (hclib_amd/csrc/uts_sha1.h): cycles per SHA-1 on one wave and the chip's
// SHA-1 throughput at 1, 2 and 3 waves per SIMD. Dependent chains (each
// spawn's output is the next one's parent) as in a span-bound tree; the
// throughput rows count every lane's spawns over the launch's wall time.
//   hipcc --offload-arch=gfx950 -O3 -I hclib_amd/csrc scripts/ubench/ub_sha2.hip -o ub_sha2.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "uts_sha1.h"

using namespace hx;

template <int N>
__global__ void k_chain(uint32_t *io, unsigned long long *cyc, int n) {
    uint32_t s[N][5];
    const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < N; ++j)
        for (int k = 0; k < 5; ++k) s[j][k] = io[(gid * 5 + k) & 0xffff] ^ (0x9e3779b9u * (j + 1));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t *pp[N];
        uint32_t ii[N];
        uint32_t o[N][5];
        uint32_t *oo[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            pp[j] = s[j];
            ii[j] = (uint32_t)(it & 3);
            oo[j] = o[j];
        }
        rng_spawn_n<N>(pp, ii, oo);
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int k = 0; k < 5; ++k) s[j][k] = o[j][k];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < N; ++j)
        for (int k = 0; k < 5; ++k) x ^= s[j][k];
    io[0x10000 + gid] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int N>
static void run(int grid, int n, const char *name) {
    uint32_t *io;
    unsigned long long *cyc;
    hipMalloc(&io, (0x10000 + 64 * 8192) * 4);
    hipMalloc(&cyc, 8 * 8192);
    hipMemset(io, 1, (0x10000 + 64 * 8192) * 4);
    hipLaunchKernelGGL(k_chain<N>, dim3(grid), dim3(64), 0, 0, io, cyc, n);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_chain<N>, dim3(grid), dim3(64), 0, 0, io, cyc, n);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double sha = (double)grid * 64 * n * N;
    printf("%-28s grid=%5d  cycles per step (wave 0) %7.1f = %6.1f per SHA-1 | chip %.1f G SHA-1/s\n", name, grid,
           (double)c / n, (double)c / n / N, sha / (ms * 1e-3) / 1e9);
    hipFree(io);
    hipFree(cyc);
}

int main() {
    for (int grid : {1, 1024, 2048, 3072}) {
        run<1>(grid, grid == 1 ? 2000 : 4000, "one chain");
        run<2>(grid, grid == 1 ? 1000 : 2000, "two interleaved chains");
        run<3>(grid, grid == 1 ? 700 : 1400, "three interleaved chains");
    }
    return 0;
}
