// HBM ceiling microbenchmark for the forasync triad (12 B/elem, 2 reads : 1 write):
// read-only, write-only, triad (register loads), triad (LDS-DMA loads), each at
// 2^28 fp32 elements, hipEvent-timed over 20 launches (+3 warm-up).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int64_t N = 1ll << 28, N4 = N / 4;

template <int U>
__global__ __launch_bounds__(256) void k_read2(const v4f *__restrict__ b, const v4f *__restrict__ c, float *out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    v4f acc = {0, 0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N4; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) acc += __builtin_nontemporal_load(&b[j]) + __builtin_nontemporal_load(&c[j]);
        }
    }
    if (acc.x == 12345.f) out[0] = acc.y;  // never true for rand inputs in [0,1)
}

template <int U>
__global__ __launch_bounds__(256) void k_write1(v4f *__restrict__ a, float s) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const v4f v = {s, s, s, s};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N4; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) __builtin_nontemporal_store(v, &a[j]);
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_triad(v4f *__restrict__ a, const v4f *__restrict__ b,
                                               const v4f *__restrict__ c, float s) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N4; i += U * stride) {
        v4f vb[U], vc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) {
                vb[u] = __builtin_nontemporal_load(&b[j]);
                vc[u] = __builtin_nontemporal_load(&c[j]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) __builtin_nontemporal_store(vb[u] + s * vc[u], &a[j]);
        }
    }
}

// LDS-DMA: each wave loads its b and c pieces (1 KiB each per wave instruction)
// into an LDS ring of D stages, consumes the oldest stage, stores a (nt).
template <int D>
__global__ __launch_bounds__(256) void k_triad_lds(v4f *__restrict__ a, const v4f *__restrict__ b,
                                                   const v4f *__restrict__ c, float s) {
    __shared__ v4f ring[4][D][2][64];  // [wave][stage][b|c][lane]
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t wstride = (int64_t)gridDim.x * 4 * 64;  // elements (v4f) per grid step
    const int64_t base = ((int64_t)blockIdx.x * 4 + w) * 64;
    const int64_t steps = (N4 - base + wstride - 1) / wstride;
    auto issue = [&](int64_t t) {
        const int st = (int)(t % D);
        const int64_t j = base + t * wstride + lane;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(b + j),
                                         (void __attribute__((address_space(3))) *)&ring[w][st][0][0], 16, 0, 2);
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(c + j),
                                         (void __attribute__((address_space(3))) *)&ring[w][st][1][0], 16, 0, 2);
    };
    int64_t t = 0;
    for (; t < D - 1 && t < steps; ++t) issue(t);
    for (int64_t k = 0; k < steps; ++k) {
        if (t < steps) { issue(t); ++t; }
        // wait until stage k landed: at most 2*(t-k-1) loads younger than it in flight
        const int64_t ahead = t - k - 1;
        if (ahead >= D - 1) __builtin_amdgcn_s_waitcnt(0x0F70 | ((2 * (D - 1)) & 15) | (((2 * (D - 1)) >> 4) << 14));
        else __builtin_amdgcn_s_waitcnt(0x0F70);
        const int st = (int)(k % D);
        const v4f vb = ring[w][st][0][lane], vc = ring[w][st][1][lane];
        __builtin_nontemporal_store(vb + s * vc, &a[base + k * wstride + lane]);
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) f();
    hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 20;
}

int main() {
    v4f *a, *b, *c;
    float *o;
    (void)hipMalloc(&a, N * 4);
    (void)hipMalloc(&b, N * 4);
    (void)hipMalloc(&c, N * 4);
    (void)hipMalloc(&o, 64);
    (void)hipMemset(b, 0, N * 4);
    (void)hipMemset(c, 0, N * 4);
    int cus = 256;
    for (int bpc : {1, 2, 4}) {
        const int g = cus * bpc;
        float ms;
        ms = timeit([&] { hipLaunchKernelGGL(k_read2<4>, dim3(g), dim3(256), 0, 0, b, c, o); });
        printf("bpc=%d read2  U4   %.4f ms %7.1f GB/s\n", bpc, ms, 8.0 * N / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_read2<8>, dim3(g), dim3(256), 0, 0, b, c, o); });
        printf("bpc=%d read2  U8   %.4f ms %7.1f GB/s\n", bpc, ms, 8.0 * N / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_write1<4>, dim3(g), dim3(256), 0, 0, a, 3.f); });
        printf("bpc=%d write1 U4   %.4f ms %7.1f GB/s\n", bpc, ms, 4.0 * N / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_triad<4>, dim3(g), dim3(256), 0, 0, a, b, c, 3.f); });
        printf("bpc=%d triad  U4   %.4f ms %7.1f GB/s\n", bpc, ms, 12.0 * N / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_triad<8>, dim3(g), dim3(256), 0, 0, a, b, c, 3.f); });
        printf("bpc=%d triad  U8   %.4f ms %7.1f GB/s\n", bpc, ms, 12.0 * N / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_triad_lds<4>, dim3(g), dim3(256), 0, 0, a, b, c, 3.f); });
        printf("bpc=%d triadL D4   %.4f ms %7.1f GB/s\n", bpc, ms, 12.0 * N / ms / 1e6);
        ms = timeit([&] { hipLaunchKernelGGL(k_triad_lds<8>, dim3(g), dim3(256), 0, 0, a, b, c, 3.f); });
        printf("bpc=%d triadL D8   %.4f ms %7.1f GB/s\n", bpc, ms, 12.0 * N / ms / 1e6);
    }
    return 0;
}
