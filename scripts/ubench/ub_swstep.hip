// ub_swstep.hip — latency of the Smith-Waterman band step's dependent chain
// on gfx950 (one wave, nothing else on the CU): cycles per step for
//   max3      a chain of v_max3_i32 (one dependent op per step)
//   dpp1      v_mov_b32_dpp wave_shr:1 -> v_max3_i32 (R = 1 step)
//   dpp2      v_mov_b32_dpp wave_shr:1 -> v_max3_i32 -> v_max3_i32 (R = 2)
//   dpp4      ... four max3 (R = 4)
//   row_shr   the same R = 2 step with DPP row_shr:1 (16-lane rows; the
//             row boundary handed over separately) for comparison
//   dppfar    R = 2 step whose DPP reads a value one step old (skew 2)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/ub_swstep.hip -o scripts/ubench/ub_swstep.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define STEP_MAX3 asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(h0) : "v"(u), "v"(d))
#define STEP_DPP1                                                           \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %1, %1, %0, %2"                                 \
                 : "+v"(u), "+v"(h0)                                         \
                 : "v"(d))
#define STEP_DPP2                                                           \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %1, %1, %0, %3\n"                               \
                 "v_max3_i32 %2, %2, %1, %3"                                 \
                 : "+v"(u), "+v"(h0), "+v"(h1)                               \
                 : "v"(d))
#define STEP_DPP4                                                           \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %1, %1, %0, %5\n"                               \
                 "v_max3_i32 %2, %2, %1, %5\n"                               \
                 "v_max3_i32 %3, %3, %2, %5\n"                               \
                 "v_max3_i32 %4, %4, %3, %5"                                 \
                 : "+v"(u), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3)           \
                 : "v"(d))
#define STEP_ROW2                                                           \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %1, %1, %0, %3\n"                               \
                 "v_max3_i32 %2, %2, %1, %3"                                 \
                 : "+v"(u), "+v"(h0), "+v"(h1)                               \
                 : "v"(d))
// skew 2: the DPP moves last step's h1 (o) while this step's h1 is computed
#define STEP_FAR2                                                           \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_mov_b32 %4, %2\n"                                        \
                 "v_max3_i32 %1, %1, %0, %3\n"                               \
                 "v_max3_i32 %2, %2, %1, %3"                                 \
                 : "+v"(u), "+v"(h0), "+v"(h1), "+v"(d), "+v"(o))

// R = 1 step with the band loop's side work: + an independent
// v_add_u32_sdwa (the diagonal + score), + a ds_write_b32 of h (the ring
// write every lane issues), + both
#define STEP_DPP1A                                                          \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_add_u32_sdwa %2, %0, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n" \
                 "v_max3_i32 %1, %1, %0, %2"                                 \
                 : "+v"(u), "+v"(h0), "+v"(d)                                \
                 : "v"(o))
#define STEP_DPP1W                                                          \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_max3_i32 %1, %1, %0, %2\n"                               \
                 "ds_write_b32 %3, %1"                                        \
                 : "+v"(u), "+v"(h0)                                         \
                 : "v"(d), "v"(la)                                           \
                 : "memory")
#define STEP_DPP1AW                                                         \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "v_add_u32_sdwa %2, %0, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n" \
                 "v_max3_i32 %1, %1, %0, %2\n"                               \
                 "ds_write_b32 %4, %1"                                        \
                 : "+v"(u), "+v"(h0), "+v"(d)                                \
                 : "v"(o), "v"(la)                                           \
                 : "memory")

// the ring write one step late: h of the previous step, written right after
// the DPP that already waited for it (two registers alternate)
#define STEP_DPP1WL                                                         \
    asm volatile("s_nop 1\n v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "ds_write_b32 %4, %1\n"                                     \
                 "v_max3_i32 %2, %1, %0, %3\n"                               \
                 "s_nop 1\n v_mov_b32_dpp %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n" \
                 "ds_write_b32 %4, %2 offset:256\n"                          \
                 "v_max3_i32 %1, %2, %0, %3"                                 \
                 : "+v"(u), "+v"(h0), "+v"(h1)                               \
                 : "v"(d), "v"(la)                                           \
                 : "memory")

template <int MODE>
__global__ void k_step(int *io, unsigned long long *cyc, int n) {
    __shared__ int lds[512];
    const uint32_t la = (uint32_t)(uintptr_t)&lds[threadIdx.x];
    const int g = threadIdx.x;
    int u = io[g], h0 = io[g + 64], h1 = io[g + 128], h2 = io[g + 192], h3 = io[g + 256], d = io[g + 320],
        o = io[g + 384];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (MODE == 0) STEP_MAX3;
            if (MODE == 1) STEP_DPP1;
            if (MODE == 2) STEP_DPP2;
            if (MODE == 3) STEP_DPP4;
            if (MODE == 4) STEP_ROW2;
            if (MODE == 5) STEP_FAR2;
            if (MODE == 6) STEP_DPP1A;
            if (MODE == 7) STEP_DPP1W;
            if (MODE == 8) STEP_DPP1AW;
            if (MODE == 9 && (r & 1) == 0) STEP_DPP1WL;  // two steps per macro
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    io[512 + g] = u ^ h0 ^ h1 ^ h2 ^ h3 ^ o ^ lds[(g + 1) & 63];
    if (g == 0) cyc[0] = t1 - t0;
}

template <int MODE>
static void run(const char *name) {
    int *io;
    unsigned long long *cyc;
    (void)hipMalloc(&io, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    (void)hipMemset(io, 0, 1024 * 4);
    const int n = 2000;
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_step<MODE>, dim3(1), dim3(64), 0, 0, io, cyc, n);
        (void)hipDeviceSynchronize();
        unsigned long long c = 0;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        const double per = (double)c / (n * 16.0);
        best = per < best ? per : best;
    }
    printf("%-8s %6.1f cycles per step (s_memtime, one wave)\n", name, best);
    (void)hipFree(io);
    (void)hipFree(cyc);
}

int main() {
    run<0>("max3");
    run<1>("dpp1");
    run<2>("dpp2");
    run<3>("dpp4");
    run<4>("row_shr");
    run<5>("dppfar");
    run<6>("dpp1+add");
    run<7>("dpp1+ds");
    run<8>("dpp1+add+ds");
    run<9>("dpp1+ds late");
    return 0;
}
