// Triad launch-shape sweep: threads x unroll x blocks/CU x load policy (2^28 fp32).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int64_t N = 1ll << 28, N4 = N / 4;

template <int T, int U, bool NTL>
__global__ __launch_bounds__(T) void k_triad(v4f *__restrict__ a, const v4f *__restrict__ b,
                                             const v4f *__restrict__ c, float s) {
    const int64_t stride = (int64_t)gridDim.x * T;
    for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < N4; i += U * stride) {
        v4f vb[U], vc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) {
                vb[u] = NTL ? __builtin_nontemporal_load(&b[j]) : b[j];
                vc[u] = NTL ? __builtin_nontemporal_load(&c[j]) : c[j];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) __builtin_nontemporal_store(vb[u] + s * vc[u], &a[j]);
        }
    }
}

template <int T, int U, bool NTL>
void run(v4f *a, v4f *b, v4f *c, int bpc) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int g = 256 * bpc;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_triad<T, U, NTL>), dim3(g), dim3(T), 0, 0, a, b, c, 3.f);
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_triad<T, U, NTL>), dim3(g), dim3(T), 0, 0, a, b, c, 3.f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    printf("T=%4d U=%d bpc=%d ntl=%d  best %.4f ms %7.1f GB/s\n", T, U, bpc, (int)NTL, best, 12.0 * N / best / 1e6);
}

int main() {
    v4f *a, *b, *c;
    (void)hipMalloc(&a, N * 4);
    (void)hipMalloc(&b, N * 4);
    (void)hipMalloc(&c, N * 4);
    (void)hipMemset(b, 0, N * 4);
    (void)hipMemset(c, 0, N * 4);
    for (int bpc : {1, 2}) {
        run<128, 4, true>(a, b, c, bpc);
        run<128, 8, true>(a, b, c, bpc);
        run<256, 1, true>(a, b, c, bpc);
        run<256, 2, true>(a, b, c, bpc);
        run<256, 4, true>(a, b, c, bpc);
        run<256, 4, false>(a, b, c, bpc);
        run<512, 1, true>(a, b, c, bpc);
        run<512, 2, true>(a, b, c, bpc);
        run<512, 4, true>(a, b, c, bpc);
        run<1024, 1, true>(a, b, c, bpc);
        run<1024, 2, true>(a, b, c, bpc);
    }
    return 0;
}
