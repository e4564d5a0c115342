// ub_valu2.hip — chip-wide VALU issue rate of the SHA-1's instruction forms
// on gfx950, measured soundly: every block's own
// s_memtime span is read back (min / mean / max over all blocks, not block
// 0's), kernels run >= 10 ms so launch ramp is noise, and the chip rate comes
// from the event time. Forms: the operand kinds the compiled SHA-1 uses —
// three VGPR sources, two VGPRs + an SGPR, a rotate (alignbit x, x, const)
// whose sources are one VGPR and an inline constant — 8 independent chains
// per lane, 1 / 2 / 4 waves per SIMD on every CU.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench/ub_valu2.hip -o scripts/ubench/ub_valu2.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

// 8 independent chains x_i = OP(x_i, ...) per asm block
#define CH8(FMT)                                                                                             \
    asm volatile(FMT(0) FMT(1) FMT(2) FMT(3) FMT(4) FMT(5) FMT(6) FMT(7)                                     \
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)            \
                 : "v"(y), "v"(z), "s"(sk))

#define F_ALIGN_VVV(i) "v_alignbit_b32 %" #i ", %" #i ", %8, %9\n"
#define F_ALIGN_ROT(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 27\n"      // rotl(x, 5)
#define F_ALIGN_VVS(i) "v_alignbit_b32 %" #i ", %" #i ", %8, %10\n"
#define F_ADD3_VVV(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n"
#define F_ADD3_VVS(i) "v_add3_u32 %" #i ", %" #i ", %8, %10\n"
#define F_ADD3_VSV(i) "v_add3_u32 %" #i ", %10, %" #i ", %8\n"
#define F_BITOP3_VVV(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n"
#define F_XOR_VV(i) "v_xor_b32 %" #i ", %" #i ", %8\n"
#define F_ADD_VV(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define F_LSHLADD_VCV(i) "v_lshl_add_u32 %" #i ", %" #i ", 3, %8\n"

template <int OP>
__global__ __launch_bounds__(64) void k_ops(uint32_t *io, unsigned long long *cyc, int n, uint32_t sk) {
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    uint32_t x0 = io[g & 1023], x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
             x7 = x0 + 7, y = x0 ^ 0x55u, z = x0 ^ 0x77u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (OP == 0) CH8(F_ALIGN_VVV);
            if (OP == 1) CH8(F_ALIGN_ROT);
            if (OP == 2) CH8(F_ALIGN_VVS);
            if (OP == 3) CH8(F_ADD3_VVV);
            if (OP == 4) CH8(F_ADD3_VVS);
            if (OP == 5) CH8(F_ADD3_VSV);
            if (OP == 6) CH8(F_BITOP3_VVV);
            if (OP == 7) CH8(F_XOR_VV);
            if (OP == 8) CH8(F_ADD_VV);
            if (OP == 9) CH8(F_LSHLADD_VCV);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    io[4096 + g] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static const char *kNames[] = {"alignbit v,v,v,v", "alignbit x,x,x,27 (rotate)", "alignbit v,v,v,s",
                               "add3 v,v,v,v",     "add3 v,v,v,s",               "add3 v,s,v,v",
                               "bitop3 v,v,v,v",   "xor v,v,v",                  "add v,v,v",
                               "lshl_add v,v,3,v"};

template <int OP>
static void run(int cus, int clock_khz) {
    const int max_grid = cus * 4 * 4;
    uint32_t *io;
    unsigned long long *cyc;
    hipMalloc(&io, (4096 + 64 * max_grid) * 4);
    hipMalloc(&cyc, 8 * max_grid);
    hipMemset(io, 1, (4096 + 64 * max_grid) * 4);
    for (int wps : {1, 2, 4}) {
        const int grid = cus * 4 * wps;
        // 12-25 ms per launch: n blocks of 64 instructions per wave, at
        // 2.5 SIMD-cycles per instruction 12 ms (5 cycles: 24 ms)
        const int n = (int)(12e-3 * clock_khz * 1e3 / (64.0 * 2.5 * wps) + 1);
        hipLaunchKernelGGL(k_ops<OP>, dim3(grid), dim3(64), 0, 0, io, cyc, n / 8 + 1, 0x5a827999u);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_ops<OP>, dim3(grid), dim3(64), 0, 0, io, cyc, n, 0x5a827999u);
        hipEventRecord(e1, 0);
        hipDeviceSynchronize();
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> c(grid);
        hipMemcpy(c.data(), cyc, 8 * grid, hipMemcpyDeviceToHost);
        std::sort(c.begin(), c.end());
        double mean = 0;
        for (auto v : c) mean += (double)v;
        mean /= grid;
        const double instr = n * 64.0;  // per wave
        const double winst = (double)grid * instr;
        printf("%-28s waves/SIMD %d: cycles per wave-instr per wave min %.2f mean %.2f max %.2f; per SIMD %.2f; "
               "kernel %.2f ms; chip %.0f G wave-instr/s = %.2f SIMD-cycles each at %d MHz\n",
               kNames[OP], wps, c[0] / instr, mean / instr, c[grid - 1] / instr, mean / instr / wps, ms,
               winst / (ms * 1e-3) / 1e9, (cus * 4.0) * (clock_khz * 1e3) * (ms * 1e-3) / winst, clock_khz / 1000);
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
    hipFree(io);
    hipFree(cyc);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
    run<0>(p.multiProcessorCount, p.clockRate);
    run<1>(p.multiProcessorCount, p.clockRate);
    run<2>(p.multiProcessorCount, p.clockRate);
    run<3>(p.multiProcessorCount, p.clockRate);
    run<4>(p.multiProcessorCount, p.clockRate);
    run<5>(p.multiProcessorCount, p.clockRate);
    run<6>(p.multiProcessorCount, p.clockRate);
    run<7>(p.multiProcessorCount, p.clockRate);
    run<8>(p.multiProcessorCount, p.clockRate);
    run<9>(p.multiProcessorCount, p.clockRate);
    return 0;
}
