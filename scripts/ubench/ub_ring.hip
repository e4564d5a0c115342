// Ring round-trip microbenchmark: one wave, the megakernel's push/pop LDS
// pattern per iteration, cycles/iteration via s_memtime.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int CAP = 1024;
struct Ring {
    uint2 d[CAP];
    uint4 t0[CAP];
    uint2 t1[CAP];
};

template <int MODE>
__global__ __launch_bounds__(64) void k_ring(unsigned long long *cyc, uint32_t *out, int iters) {
    __shared__ Ring st;
    const uint32_t lane = threadIdx.x;
    for (int i = lane; i < CAP; i += 64) {
        st.d[i] = make_uint2(i, i);
        st.t0[i] = make_uint4(i, 1, 2, 3);
        st.t1[i] = make_uint2(i, 5);
    }
    __syncthreads();
    uint32_t acc = lane, top = 64;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        // pop: desc then template (2 dependent round trips) or template only
        const uint32_t p = (top - 1 - lane) & (CAP - 1);
        uint2 dd = make_uint2(0, 0);
        uint32_t slot = p;
        if (MODE & 1) {
            dd = st.d[p];
            slot = (p - (dd.y >> 24)) & (CAP - 1);
        }
        const uint4 a = st.t0[slot];
        const uint2 b = st.t1[slot];
        acc += a.x + a.w + b.y + dd.x;
        // pretend work: a short dependent VALU chain (no LDS)
#pragma unroll
        for (int r = 0; r < 8; ++r) acc = __builtin_amdgcn_alignbit(acc, acc, 27) + r;
        // push: group template at every 5th lane + lane-contiguous descriptors
        if (MODE & 2) {
            const bool spawn = (acc & 3) != 0 || lane % 5 == 0;
            const uint32_t base = top + 40;
            if (lane % 5 == 0) {
                st.t0[(base + lane) & (CAP - 1)] = make_uint4(acc, a.y, a.z, a.w);
                st.t1[(base + lane) & (CAP - 1)] = make_uint2(b.x, acc);
            }
            const uint32_t kk = lane % 5;
            st.d[(base + lane) & (CAP - 1)] = make_uint2(kk, (kk + 1) | (kk << 24));
            (void)spawn;
        }
        top += 40;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int MODE>
double run(unsigned long long *cyc, uint32_t *out) {
    const int iters = 4000;
    hipLaunchKernelGGL(k_ring<MODE>, dim3(1), dim3(64), 0, 0, cyc, out, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k_ring<MODE>, dim3(1), dim3(64), 0, 0, cyc, out, iters);
    unsigned long long h;
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    return (double)h / iters;
}

int main() {
    unsigned long long *cyc;
    uint32_t *out;
    hipMalloc(&cyc, 8);
    hipMalloc(&out, 256);
    printf("template read only                     %.1f cycles/iter\n", run<0>(cyc, out));
    printf("desc -> template reads                 %.1f cycles/iter\n", run<1>(cyc, out));
    printf("template read + push writes            %.1f cycles/iter\n", run<2>(cyc, out));
    printf("desc -> template reads + push writes   %.1f cycles/iter\n", run<3>(cyc, out));
    return 0;
}
