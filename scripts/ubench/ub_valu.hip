// ub_valu.hip — VALU issue rate of the ops the UTS SHA-1 is made of, on
// gfx950: 8 independent chains per lane (no dependency stalls), 1, 2 and 4
// waves per SIMD on every CU. Reports cycles per wave-instruction for one
// wave and for the SIMD (the roofline of an integer-VALU-bound kernel).
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench/ub_valu.hip -o ub_valu.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define OPS8(OP)                                                                                        \
    asm volatile(OP " %0, %0, %8, %9\n" OP " %1, %1, %8, %9\n" OP " %2, %2, %8, %9\n" OP " %3, %3, %8, %9\n" \
                 OP " %4, %4, %8, %9\n" OP " %5, %5, %8, %9\n" OP " %6, %6, %8, %9\n" OP " %7, %7, %8, %9"   \
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)       \
                 : "v"(y), "v"(z))
#define OPS8_B3                                                                                           \
    asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n"           \
                 "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n"           \
                 "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n"           \
                 "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"              \
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)       \
                 : "v"(y), "v"(z))
#define OPS8_2(OP)                                                                                      \
    asm volatile(OP " %0, %0, %8\n" OP " %1, %1, %8\n" OP " %2, %2, %8\n" OP " %3, %3, %8\n" OP         \
                    " %4, %4, %8\n" OP " %5, %5, %8\n" OP " %6, %6, %8\n" OP " %7, %7, %8"                 \
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)       \
                 : "v"(y))

template <int OP>
__global__ void k_ops(uint32_t *io, unsigned long long *cyc, int n) {
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    uint32_t x0 = io[g & 1023], x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
             x7 = x0 + 7, y = x0 ^ 0x55u, z = x0 ^ 0x77u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (OP == 0) OPS8("v_alignbit_b32");
            if (OP == 1) OPS8_B3;
            if (OP == 2) OPS8("v_add3_u32");
            if (OP == 3) OPS8_2("v_add_u32");
            if (OP == 4) OPS8_2("v_xor_b32");
            if (OP == 5) OPS8("v_fma_f32");
            if (OP == 6) OPS8("v_lshl_add_u32");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    io[4096 + g] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(const char *name, int cus) {
    uint32_t *io;
    unsigned long long *cyc;
    hipMalloc(&io, (4096 + 64 * 16384) * 4);
    hipMalloc(&cyc, 8 * 16384);
    hipMemset(io, 1, (4096 + 64 * 16384) * 4);
    const int n = 400;
    for (int wps : {1, 2, 4}) {
        const int grid = cus * 4 * wps;
        hipLaunchKernelGGL(k_ops<OP>, dim3(grid), dim3(64), 0, 0, io, cyc, n);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_ops<OP>, dim3(grid), dim3(64), 0, 0, io, cyc, n);
        hipEventRecord(e1, 0);
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        const double per_wave = (double)c / (n * 64.0);
        const double winst = (double)grid * n * 64.0;
        printf("%-18s waves/SIMD %d: %5.2f cycles per wave-instr per wave, %5.2f per SIMD; chip %.0f G wave-instr/s\n",
               name, wps, per_wave, per_wave / wps, winst / (ms * 1e-3) / 1e9);
    }
    hipFree(io);
    hipFree(cyc);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
    run<0>("v_alignbit_b32", p.multiProcessorCount);
    run<1>("v_bitop3_b32", p.multiProcessorCount);
    run<2>("v_add3_u32", p.multiProcessorCount);
    run<3>("v_add_u32", p.multiProcessorCount);
    run<4>("v_xor_b32", p.multiProcessorCount);
    run<5>("v_fma_f32", p.multiProcessorCount);
    run<6>("v_lshl_add_u32", p.multiProcessorCount);
    return 0;
}
