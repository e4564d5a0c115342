// ub_pkstep.hip — cycles per step of the packed-half SW sweep (sw.hip
// sw_pk_tile) on gfx950, one wave alone on its CU, operands in registers:
//   full     rot (DPP wave_ror) + up (v_perm) + 2 v_pk_add_f16 + 2 v_pk_maximum3_f16 + pair gather
//   nogather the same without the bottom-row gather (perm + DPP every 2 steps)
//   nodpp    rot = lr1 (no DPP)
//   noperm   up = rot (no per-lane fixup permute)
//   chain    rot + up + 2 max3 only (the dependent chain, no adds, no gather)
//   full+lds full with its operands loaded from LDS as the kernel does
// each on 1, 256 and 512 one-wave workgroups (clock under load)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/ub_pkstep.hip -o scripts/ubench/ub_pkstep.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 ash(uint32_t v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ uint32_t asu(h2 v) { return __builtin_bit_cast(uint32_t, v); }

template <int V>
__global__ __launch_bounds__(64) void k_step(uint32_t *out, unsigned long long *cyc, int nsteps, uint32_t seed) {
    const int lane = threadIdx.x;
    // V == 5: the full step with its operands from LDS as sw_pk_tile reads
    // them (a broadcast int4 of the top row + two uint4 of scores per 4 steps)
    __shared__ uint4 ring[2 * 32 * 64];
    __shared__ int topr[512];
    for (int i = lane; i < 2 * 32 * 64; i += 64) ring[i] = make_uint4(seed * i, seed + i, seed ^ i, i) & make_uint4(0x44004400u, 0x44004400u, 0x44004400u, 0x44004400u);
    for (int i = lane; i < 512; i += 64) topr[i] = (seed + i) & 0x3c00;
    __syncthreads();
    const uint32_t selU = lane == 0 ? 0x05040100u : 0x07060504u;
    h2 lr0 = ash(seed * (lane + 1)), lr1 = ash(seed ^ lane), upp = ash(seed + lane);
    uint32_t acc = 0;
    uint32_t sc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] = (seed * (i + 3)) & 0x44004400u;
    uint32_t tvv = seed & 0x3c00u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s0 = 0; s0 < nsteps; s0 += 16) {
        uint4 q[8];
        int4 tq[4];
        if (V == 5) {
            const uint4 *src = ring + ((s0 >> 4) & 63) * 8 * 64 + lane;
#pragma unroll
            for (int i = 0; i < 8; ++i) q[i] = src[i * 64];
#pragma unroll
            for (int i = 0; i < 4; ++i) tq[i] = *(const int4 *)(topr + ((s0 + 4 * i) & 511));
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            if (V == 5) {
                const uint4 r = q[jj >> 1];
                sc[jj & 7] = (jj & 1) ? r.z : r.x;
                sc[(jj + 1) & 7] = (jj & 1) ? r.w : r.y;
                const int4 t4 = tq[jj >> 2];
                tvv = (jj & 3) == 0 ? t4.x : (jj & 3) == 1 ? t4.y : (jj & 3) == 2 ? t4.z : t4.w;
            }
            const uint32_t rot = V == 2 ? asu(lr1) : (uint32_t)__builtin_amdgcn_mov_dpp((int)asu(lr1), 0x13C, 0xf, 0xf, false);
            const h2 up = V == 3 ? ash(rot) : ash(__builtin_amdgcn_perm(rot, V == 5 ? tvv : tvv + jj, selU));
            h2 h0, h1;
            if (V == 4) {
                h0 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(lr0, up), upp);
                h1 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(lr1, h0), lr0);
            } else {
                h0 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(lr0, up), upp + ash(sc[jj & 7]));
                h1 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(lr1, h0), lr0 + ash(sc[(jj + 1) & 7]));
            }
            if (V != 1 && V != 4 && (jj & 1)) {
                const uint32_t pair = __builtin_amdgcn_perm(asu(h1), asu(lr1), 0x07060302u);
                acc = (uint32_t)__builtin_amdgcn_update_dpp((int)pair, (int)acc, 0x130, 0xf, 0xf, false);
            }
            upp = up;
            lr0 = h0;
            lr1 = h1;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = asu(lr0) ^ asu(lr1) ^ acc;
    if (lane == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int V>
void launch(int grid, uint32_t *out, unsigned long long *cyc, int n) {
    hipLaunchKernelGGL(k_step<V>, dim3(grid), dim3(64), 0, 0, out, cyc, n, 0x3c003c00u);
}

int main() {
    uint32_t *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, 512 * 256);
    hipMalloc(&cyc, 8);
    const int n = 1 << 16;
    const char *names[] = {"full", "nogather", "nodpp", "noperm", "chain", "full+lds"};
    for (int grid : {1, 256, 512})
        for (int rep = 0; rep < 2; ++rep)
            for (int v = 0; v < 6; ++v) {
                switch (v) {
                case 0: launch<0>(grid, out, cyc, n); break;
                case 1: launch<1>(grid, out, cyc, n); break;
                case 2: launch<2>(grid, out, cyc, n); break;
                case 3: launch<3>(grid, out, cyc, n); break;
                case 4: launch<4>(grid, out, cyc, n); break;
                default: launch<5>(grid, out, cyc, n); break;
                }
                hipDeviceSynchronize();
                hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
                if (rep) printf("grid %3d %-9s %6.1f cycles per step (s_memtime, block 0)\n", grid, names[v], (double)h / n);
            }
    return 0;
}
