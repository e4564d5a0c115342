// ub_sha_partner.hip — one dependent rng_spawn SHA-1 per step (the T3L
// narrow loop's critical chain), on one wave alone against a "round wave" that
// gets the tail of its message schedule from a partner wave through LDS.
//
// Round 2's split (ub_sha_split.hip) put the partner on wave 1 of a 2-wave
// workgroup and had it compute all of W16..W79 after the round wave posted its
// inputs: 3,100-3,800 cycles per step against 2,652. Two things change here:
//  * placement: the workgroup has 4 waves; HW_ID tells each wave its SIMD,
//    and the partner is chosen on a SIMD other than the round wave's (a lone
//    wave issues one VALU per ~5 cycles, ub_valu2.log, so a second SIMD is the
//    only place extra issue comes from; the same SIMD shares alignbit/add3's
//    4.27-cycle pipe);
//  * lead: the round wave computes W16..W(15+M) itself and the partner
//    publishes K+W for t >= 16+M in 4-word groups, each behind a sequence word
//    (one LDS queue per wave is in order, so a round-wave read of the sequence
//    word issued before the group's data read and seeing this step's value
//    means the data read sees this step's words). The partner recomputes
//    W16..W(15+M) (it needs them) but does not publish them.
// Output: cycles per step on the round wave (s_memtime), every chain checked
// against the one-wave chain.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I hclib_amd/csrc scripts/ubench/ub_sha_partner.hip -o scripts/ubench/ub_sha_partner.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "uts_sha1.h"

using hx::fch;
using hx::fmaj;
using hx::rl;
using hx::x3;

constexpr uint32_t C6 = 0x80000000u, C15 = 192u;
constexpr uint32_t K0 = 0x5a827999u, K1 = 0x6ed9eba1u, K2 = 0x8f1bbcdcu, K3 = 0xca62c1d6u;

__host__ __device__ constexpr uint32_t kof(int t) { return t < 20 ? K0 : t < 40 ? K1 : t < 60 ? K2 : K3; }

__device__ __forceinline__ void sched(const uint32_t p[5], uint32_t i, uint32_t w[80]) {
    w[0] = p[0]; w[1] = p[1]; w[2] = p[2]; w[3] = p[3]; w[4] = p[4]; w[5] = i;
    w[16] = rl(w[2] ^ w[0], 1);
    w[17] = rl(w[3] ^ w[1], 1);
    w[18] = rl(x3(C15, w[4], w[2]), 1);
    w[19] = rl(x3(w[16], w[5], w[3]), 1);
    w[20] = rl(x3(w[17], C6, w[4]), 1);
    w[21] = rl(w[18] ^ w[5], 1);
    w[22] = rl(w[19] ^ C6, 1);
    w[23] = rl(w[20] ^ C15, 1);
#pragma unroll
    for (int t = 24; t < 29; ++t) w[t] = rl(w[t - 3] ^ w[t - 8], 1);
    w[29] = rl(x3(w[26], w[21], C15), 1);
    w[30] = rl(x3(w[27], w[22], w[16]), 1);
    w[31] = rl(x3(w[28], w[23], w[17]) ^ C15, 1);
#pragma unroll
    for (int t = 32; t < 80; ++t) w[t] = rl(x3(w[t - 3], w[t - 8], w[t - 14]) ^ w[t - 16], 1);
}

// reassociated round: X = F + e + KW does not depend on a; a' = rl5(a) + X
#define R2(F, KW)                                           \
    {                                                       \
        const uint32_t x_ = F(b, c, d) + e + (KW);          \
        const uint32_t t_ = rl(a, 5) + x_;                  \
        e = d; d = c; c = rl(b, 30); b = a; a = t_;         \
    }
#define RT(t, KW)                                   \
    {                                               \
        if ((t) < 20) R2(fch, KW)                   \
        else if ((t) < 40) R2(x3, KW)               \
        else if ((t) < 60) R2(fmaj, KW)             \
        else R2(x3, KW)                             \
    }

// one wave alone (the product's rng_spawn)
__global__ void k_one(uint32_t *io, unsigned long long *cyc, int n) {
    const int lane = threadIdx.x;
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        uint32_t o[5];
        hx::rng_spawn_dev(s, (uint32_t)(it & 3), o);
        for (int k = 0; k < 5; ++k) s[k] = o[k];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[0x1000 + lane * 5 + k] = s[k];
    if (lane == 0) cyc[0] = t1 - t0;
}

struct Shared {
    uint4 kw[16][64];         // group g: K+W[16+4g .. 19+4g]
    uint32_t gseq[16][64];    // group g's sequence word (per lane: one ds_read_b32, no bank conflict)
    uint4 in0[64];            // posted parent state p0..p3
    uint2 in1[64];            // p4, child index
    uint32_t in_seq;
    uint32_t simd[4];
};

// LDS sequence words: relaxed atomics through address-space-3 pointers. A
// volatile access through a generic pointer compiles to a FLAT operation that
// waits for the wave's global traffic too (vmcnt(0)) — which is what round 2's
// split benchmark did on every flag.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t ldv(const uint32_t *p) {
    return __hip_atomic_load((const lds_u32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void stv(uint32_t *p, uint32_t v) {
    __hip_atomic_store((lds_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int M, int PD>
__global__ void k_part(uint32_t *io, unsigned long long *cyc, uint32_t *hw, int n, int pw,
                       unsigned long long *waits) {
    __shared__ Shared sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t hwid = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    if (lane == 0) sh.simd[wave] = (hwid >> 4) & 3;
    for (int g = 0; g < 16; ++g) sh.gseq[g][lane] = 0;
    if (threadIdx.x == 0) sh.in_seq = 0;
    __syncthreads();
    if (threadIdx.x < 4) hw[threadIdx.x] = sh.simd[threadIdx.x];
    if (wave == pw) {
        for (int it = 0; it < n; ++it) {
            const uint32_t seq = (uint32_t)(it + 1);
            for (uint32_t sp = 0; ldv(&sh.in_seq) != seq && sp < (1u << 24); ++sp) {
            }
            asm volatile("" ::: "memory");
            const uint4 a = sh.in0[lane];
            const uint2 b = sh.in1[lane];
            const uint32_t p[5] = {a.x, a.y, a.z, a.w, b.x};
            uint32_t w[80];
            sched(p, b.y, w);
#pragma unroll
            for (int g = M / 4; g < 16; ++g) {
                const int t = 16 + 4 * g;
                sh.kw[g][lane] = make_uint4(w[t] + kof(t), w[t + 1] + kof(t + 1), w[t + 2] + kof(t + 2),
                                            w[t + 3] + kof(t + 3));
                asm volatile("" ::: "memory");
                stv(&sh.gseq[g][lane], seq);
                asm volatile("" ::: "memory");
            }
        }
        return;
    }
    if (wave != 0) return;
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    unsigned long long wsum = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t seq = (uint32_t)(it + 1);
        const uint32_t i = (uint32_t)(it & 3);
        sh.in0[lane] = make_uint4(s[0], s[1], s[2], s[3]);
        sh.in1[lane] = make_uint2(s[4], i);
        asm volatile("" ::: "memory");
        stv(&sh.in_seq, seq);
        asm volatile("" ::: "memory");
        uint32_t w[80];
        w[0] = s[0]; w[1] = s[1]; w[2] = s[2]; w[3] = s[3]; w[4] = s[4]; w[5] = i;
        // the round wave's own lead of the schedule
        if (M > 0) w[16] = rl(w[2] ^ w[0], 1);
        if (M > 1) w[17] = rl(w[3] ^ w[1], 1);
        if (M > 2) w[18] = rl(x3(C15, w[4], w[2]), 1);
        if (M > 3) w[19] = rl(x3(w[16], w[5], w[3]), 1);
        if (M > 4) w[20] = rl(x3(w[17], C6, w[4]), 1);
        if (M > 5) w[21] = rl(w[18] ^ w[5], 1);
        if (M > 6) w[22] = rl(w[19] ^ C6, 1);
        if (M > 7) w[23] = rl(w[20] ^ C15, 1);
#pragma unroll
        for (int t = 24; t < 16 + M && t < 29; ++t) w[t] = rl(w[t - 3] ^ w[t - 8], 1);
        if (M > 13) w[29] = rl(x3(w[26], w[21], C15), 1);
        if (M > 14) w[30] = rl(x3(w[27], w[22], w[16]), 1);
        if (M > 15) w[31] = rl(x3(w[28], w[23], w[17]) ^ C15, 1);
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        R2(fch, K0 + s[0]); R2(fch, K0 + s[1]); R2(fch, K0 + s[2]); R2(fch, K0 + s[3]); R2(fch, K0 + s[4]);
        R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
        for (int t = 7; t < 15; ++t) R2(fch, K0);
        R2(fch, K0 + C15);
#pragma unroll
        for (int t = 16; t < 16 + M; ++t) RT(t, kof(t) + w[t]);
        asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
        // published groups: PD groups in flight ahead of use
        constexpr int G0 = M / 4;
        uint32_t q[16], kv[16][4];
#pragma unroll
        for (int g = G0; g < 16; ++g) {
            if (g == G0) {
#pragma unroll
                for (int h = G0; h < G0 + PD && h < 16; ++h) {
                    q[h] = ldv(&sh.gseq[h][lane]);
                    asm volatile("" ::: "memory");
                    const uint4 v = sh.kw[h][lane];
                    kv[h][0] = v.x; kv[h][1] = v.y; kv[h][2] = v.z; kv[h][3] = v.w;
                    asm volatile("" ::: "memory");
                }
            }
            if (g + PD < 16) {
                q[g + PD] = ldv(&sh.gseq[g + PD][lane]);
                asm volatile("" ::: "memory");
                const uint4 v = sh.kw[g + PD][lane];
                kv[g + PD][0] = v.x; kv[g + PD][1] = v.y; kv[g + PD][2] = v.z; kv[g + PD][3] = v.w;
                asm volatile("" ::: "memory");
            }
            // group g due: re-read until its sequence word is this step's
            if (q[g] != seq) {
                const unsigned long long w0 = __builtin_amdgcn_s_memtime();
                for (uint32_t sp = 0; sp < (1u << 24); ++sp) {
                    q[g] = ldv(&sh.gseq[g][lane]);
                    asm volatile("" ::: "memory");
                    const uint4 v = sh.kw[g][lane];
                    kv[g][0] = v.x; kv[g][1] = v.y; kv[g][2] = v.z; kv[g][3] = v.w;
                    asm volatile("" ::: "memory");
                    if (q[g] == seq) break;
                }
                wsum += __builtin_amdgcn_s_memtime() - w0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) RT(16 + 4 * g + j, kv[g][j]);
            // the group's rounds are issued here, not sunk below the next group's check
            asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
        }
        s[0] = 0x67452301u + a; s[1] = 0xefcdab89u + b; s[2] = 0x98badcfeu + c; s[3] = 0x10325476u + d;
        s[4] = 0xc3d2e1f0u + e;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[0x2000 + lane * 5 + k] = s[k];
    if (lane == 0) {
        cyc[1] = t1 - t0;
        waits[0] = wsum;
    }
}

template <int M, int PD>
__global__ void k_partu(uint32_t *io, unsigned long long *cyc, uint32_t *hw, int n, int pw,
                       unsigned long long *waits) {
    __shared__ Shared sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t hwid = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    if (lane == 0) sh.simd[wave] = (hwid >> 4) & 3;
    for (int g = 0; g < 16; ++g) sh.gseq[g][lane] = 0;
    if (threadIdx.x == 0) sh.in_seq = 0;
    __syncthreads();
    if (threadIdx.x < 4) hw[threadIdx.x] = sh.simd[threadIdx.x];
    if (wave == pw) {
        for (int it = 0; it < n; ++it) {
            const uint32_t seq = (uint32_t)(it + 1);
            for (uint32_t sp = 0; ldv(&sh.in_seq) != seq && sp < (1u << 24); ++sp) {
            }
            asm volatile("" ::: "memory");
            const uint4 a = sh.in0[lane];
            const uint2 b = sh.in1[lane];
            const uint32_t p[5] = {a.x, a.y, a.z, a.w, b.x};
            uint32_t w[80];
            sched(p, b.y, w);
#pragma unroll
            for (int g = M / 4; g < 16; ++g) {
                const int t = 16 + 4 * g;
                sh.kw[g][lane] = make_uint4(w[t] + kof(t), w[t + 1] + kof(t + 1), w[t + 2] + kof(t + 2),
                                            w[t + 3] + kof(t + 3));
                asm volatile("" ::: "memory");
                if ((g & 1) || g == 15) stv(&sh.gseq[g >> 1][0], seq);
                asm volatile("" ::: "memory");
            }
        }
        return;
    }
    if (wave != 0) return;
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    unsigned long long wsum = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t seq = (uint32_t)(it + 1);
        const uint32_t i = (uint32_t)(it & 3);
        sh.in0[lane] = make_uint4(s[0], s[1], s[2], s[3]);
        sh.in1[lane] = make_uint2(s[4], i);
        asm volatile("" ::: "memory");
        stv(&sh.in_seq, seq);
        asm volatile("" ::: "memory");
        uint32_t w[80];
        w[0] = s[0]; w[1] = s[1]; w[2] = s[2]; w[3] = s[3]; w[4] = s[4]; w[5] = i;
        // the round wave's own lead of the schedule
        if (M > 0) w[16] = rl(w[2] ^ w[0], 1);
        if (M > 1) w[17] = rl(w[3] ^ w[1], 1);
        if (M > 2) w[18] = rl(x3(C15, w[4], w[2]), 1);
        if (M > 3) w[19] = rl(x3(w[16], w[5], w[3]), 1);
        if (M > 4) w[20] = rl(x3(w[17], C6, w[4]), 1);
        if (M > 5) w[21] = rl(w[18] ^ w[5], 1);
        if (M > 6) w[22] = rl(w[19] ^ C6, 1);
        if (M > 7) w[23] = rl(w[20] ^ C15, 1);
#pragma unroll
        for (int t = 24; t < 16 + M && t < 29; ++t) w[t] = rl(w[t - 3] ^ w[t - 8], 1);
        if (M > 13) w[29] = rl(x3(w[26], w[21], C15), 1);
        if (M > 14) w[30] = rl(x3(w[27], w[22], w[16]), 1);
        if (M > 15) w[31] = rl(x3(w[28], w[23], w[17]) ^ C15, 1);
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        R2(fch, K0 + s[0]); R2(fch, K0 + s[1]); R2(fch, K0 + s[2]); R2(fch, K0 + s[3]); R2(fch, K0 + s[4]);
        R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
        for (int t = 7; t < 15; ++t) R2(fch, K0);
        R2(fch, K0 + C15);
#pragma unroll
        for (int t = 16; t < 16 + M; ++t) RT(t, kof(t) + w[t]);
        asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
        // published groups: PD groups in flight ahead of use
        constexpr int G0 = M / 4;
        uint32_t q[16], kv[16][4];
#pragma unroll
        for (int g = G0; g < 16; ++g) {
            if (g == G0) {
#pragma unroll
                for (int h = G0; h < G0 + PD && h < 16; ++h) {
                    q[h] = __builtin_amdgcn_readfirstlane(ldv(&sh.gseq[h >> 1][0]));
                    asm volatile("" ::: "memory");
                    const uint4 v = sh.kw[h][lane];
                    kv[h][0] = v.x; kv[h][1] = v.y; kv[h][2] = v.z; kv[h][3] = v.w;
                    asm volatile("" ::: "memory");
                }
            }
            if (g + PD < 16) {
                q[g + PD] = __builtin_amdgcn_readfirstlane(ldv(&sh.gseq[(g + PD) >> 1][0]));
                asm volatile("" ::: "memory");
                const uint4 v = sh.kw[g + PD][lane];
                kv[g + PD][0] = v.x; kv[g + PD][1] = v.y; kv[g + PD][2] = v.z; kv[g + PD][3] = v.w;
                asm volatile("" ::: "memory");
            }
            // group g due: re-read until its sequence word is this step's
            if (q[g] != seq) {
                const unsigned long long w0 = __builtin_amdgcn_s_memtime();
                for (uint32_t sp = 0; sp < (1u << 24); ++sp) {
                    q[g] = __builtin_amdgcn_readfirstlane(ldv(&sh.gseq[g >> 1][0]));
                    asm volatile("" ::: "memory");
                    const uint4 v = sh.kw[g][lane];
                    kv[g][0] = v.x; kv[g][1] = v.y; kv[g][2] = v.z; kv[g][3] = v.w;
                    asm volatile("" ::: "memory");
                    if (q[g] == seq) break;
                }
                wsum += __builtin_amdgcn_s_memtime() - w0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) RT(16 + 4 * g + j, kv[g][j]);
            // the group's rounds are issued here, not sunk below the next group's check
            asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
        }
        s[0] = 0x67452301u + a; s[1] = 0xefcdab89u + b; s[2] = 0x98badcfeu + c; s[3] = 0x10325476u + d;
        s[4] = 0xc3d2e1f0u + e;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[0x2000 + lane * 5 + k] = s[k];
    if (lane == 0) {
        cyc[1] = t1 - t0;
        waits[0] = wsum;
    }
}

template <int M, int PD>
static void run_part(uint32_t *io, unsigned long long *cyc, uint32_t *hw, unsigned long long *waits, int n, int pw,
                     const uint32_t *ref, bool uni = false) {
    hipMemset(io + 0x2000, 0, 320 * 4);
    if (uni)
        hipLaunchKernelGGL((k_partu<M, PD>), dim3(1), dim3(256), 0, 0, io, cyc, hw, n, pw, waits);
    else
        hipLaunchKernelGGL((k_part<M, PD>), dim3(1), dim3(256), 0, 0, io, cyc, hw, n, pw, waits);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed\n");
        return;
    }
    unsigned long long c[2], wt;
    uint32_t h[4], o[320];
    hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
    hipMemcpy(&wt, waits, 8, hipMemcpyDeviceToHost);
    hipMemcpy(h, hw, 16, hipMemcpyDeviceToHost);
    hipMemcpy(o, io + 0x2000, sizeof(o), hipMemcpyDeviceToHost);
    const int match = memcmp(o, ref, sizeof(o)) == 0;
    // s_memtime counts at the 100 MHz constant clock? no: SHADER_CYCLES-style 64-bit core clock on gfx9
    printf("%s M=%2d PD=%d partner wave %d (SIMD %u, round wave SIMD %u): %7.1f cycles/step, waiting %6.1f/step, match %d\n",
           uni ? "scalar check/8 words" : "per-lane check/4 words", M, PD, pw, h[pw], h[0], (double)c[1] / n, (double)wt / n, match);
}

int main() {
    uint32_t *io;
    unsigned long long *cyc, *waits;
    uint32_t *hw;
    hipMalloc(&io, 0x4000 * 4);
    hipMalloc(&cyc, 64);
    hipMalloc(&waits, 64);
    hipMalloc(&hw, 64);
    uint32_t init[320];
    for (int k = 0; k < 320; ++k) init[k] = 0x9e3779b9u * (k + 1) ^ (k << 7);
    hipMemcpy(io, init, sizeof(init), hipMemcpyHostToDevice);
    const int n = 4000;
    hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, io, cyc, n);
    hipDeviceSynchronize();
    unsigned long long c1;
    uint32_t ref[320];
    hipMemcpy(&c1, cyc, 8, hipMemcpyDeviceToHost);
    hipMemcpy(ref, io + 0x1000, sizeof(ref), hipMemcpyDeviceToHost);
    printf("one wave: %.1f cycles/step\n", (double)c1 / n);
    for (int pw = 1; pw < 4; ++pw) {
        run_part<8, 2>(io, cyc, hw, waits, n, pw, ref);
        run_part<12, 2>(io, cyc, hw, waits, n, pw, ref);
        run_part<16, 2>(io, cyc, hw, waits, n, pw, ref);
        run_part<8, 2>(io, cyc, hw, waits, n, pw, ref, true);
        run_part<8, 3>(io, cyc, hw, waits, n, pw, ref, true);
        run_part<12, 2>(io, cyc, hw, waits, n, pw, ref, true);
        run_part<12, 3>(io, cyc, hw, waits, n, pw, ref, true);
        run_part<16, 2>(io, cyc, hw, waits, n, pw, ref, true);
        run_part<16, 3>(io, cyc, hw, waits, n, pw, ref, true);
    }
    return 0;
}
