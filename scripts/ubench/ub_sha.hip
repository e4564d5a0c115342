#include <hip/hip_runtime.h>
#include <stdint.h>
#define HX_ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
#define HX_RND(f, k, wi)                                \
    {                                                   \
        uint32_t t_ = HX_ROTL(a, 5) + (f) + e + (k) + (wi); \
        e = d;                                          \
        d = c;                                          \
        c = HX_ROTL(b, 30);                             \
        b = a;                                          \
        a = t_;                                         \
    }
#define HX_F1 (d ^ (b & (c ^ d)))
#define HX_F2 (b ^ c ^ d)
#define HX_F3 ((b & c) | (d & (b ^ c)))
#define HX_W(i) \
    (w[(i) & 15] = HX_ROTL(w[((i) + 13) & 15] ^ w[((i) + 8) & 15] ^ w[((i) + 2) & 15] ^ w[(i) & 15], 1))
__device__ __forceinline__ void sha1_block(uint32_t w[16], uint32_t h[5]) {
    uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) HX_RND(HX_F1, 0x5a827999u, w[i]);
#pragma unroll
    for (int i = 16; i < 20; ++i) HX_RND(HX_F1, 0x5a827999u, HX_W(i));
#pragma unroll
    for (int i = 20; i < 40; ++i) HX_RND(HX_F2, 0x6ed9eba1u, HX_W(i));
#pragma unroll
    for (int i = 40; i < 60; ++i) HX_RND(HX_F3, 0x8f1bbcdcu, HX_W(i));
#pragma unroll
    for (int i = 60; i < 80; ++i) HX_RND(HX_F2, 0xca62c1d6u, HX_W(i));
    h[0] = 0x67452301u + a; h[1] = 0xefcdab89u + b; h[2] = 0x98badcfeu + c; h[3] = 0x10325476u + d; h[4] = 0xc3d2e1f0u + e;
}
__device__ __forceinline__ void spawn_old(const uint32_t p[5], uint32_t i, uint32_t out[5]) {
    uint32_t w[16];
    w[0] = p[0]; w[1] = p[1]; w[2] = p[2]; w[3] = p[3]; w[4] = p[4]; w[5] = i; w[6] = 0x80000000u;
#pragma unroll
    for (int k = 7; k < 15; ++k) w[k] = 0;
    w[15] = 192;
    sha1_block(w, out);
}
// ---------------- new
__device__ __forceinline__ uint32_t rl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t fch(uint32_t b, uint32_t c, uint32_t d) { return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA); }
__device__ __forceinline__ uint32_t fmaj(uint32_t b, uint32_t c, uint32_t d) { return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); }
#define R(F, K, W) { uint32_t t_ = rl(a, 5) + F(b, c, d) + e + ((K) + (W)); e = d; d = c; c = rl(b, 30); b = a; a = t_; }
__device__ __forceinline__ void spawn_new(const uint32_t p[5], uint32_t i, uint32_t out[5]) {
    uint32_t w[80];
    w[0] = p[0]; w[1] = p[1]; w[2] = p[2]; w[3] = p[3]; w[4] = p[4]; w[5] = i;
    const uint32_t C6 = 0x80000000u, C15 = 192u;
    w[16] = rl(w[2] ^ w[0], 1);
    w[17] = rl(w[3] ^ w[1], 1);
    w[18] = rl(x3(C15, w[4], w[2]), 1);
    w[19] = rl(x3(w[16], w[5], w[3]), 1);
    w[20] = rl(x3(w[17], C6, w[4]), 1);
    w[21] = rl(w[18] ^ w[5], 1);
    w[22] = rl(w[19] ^ C6, 1);
    w[23] = rl(w[20] ^ C15, 1);
    w[24] = rl(w[21] ^ w[16], 1);
    w[25] = rl(w[22] ^ w[17], 1);
    w[26] = rl(w[23] ^ w[18], 1);
    w[27] = rl(w[24] ^ w[19], 1);
    w[28] = rl(w[25] ^ w[20], 1);
    w[29] = rl(x3(w[26], w[21], C15), 1);
    w[30] = rl(x3(w[27], w[22], w[16]), 1);
    w[31] = rl(x3(w[28], w[23], w[17]) ^ C15, 1);
#pragma unroll
    for (int t = 32; t < 80; ++t) w[t] = rl(x3(w[t - 3], w[t - 8], w[t - 14]) ^ w[t - 16], 1);
    const uint32_t K0 = 0x5a827999u, K1 = 0x6ed9eba1u, K2 = 0x8f1bbcdcu, K3 = 0xca62c1d6u;
    uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
    { uint32_t t_ = rl(a, 5) + (d ^ (b & (c ^ d))) + e + K0 + w[0]; e = d; d = c; c = rl(b, 30); b = a; a = t_; }
#pragma unroll
    for (int t = 1; t < 6; ++t) R(fch, K0, w[t]);
    R(fch, K0, C6);
#pragma unroll
    for (int t = 7; t < 15; ++t) R(fch, K0, 0u);
    R(fch, K0, C15);
#pragma unroll
    for (int t = 16; t < 20; ++t) R(fch, K0, w[t]);
#pragma unroll
    for (int t = 20; t < 40; ++t) R(x3, K1, w[t]);
#pragma unroll
    for (int t = 40; t < 60; ++t) R(fmaj, K2, w[t]);
#pragma unroll
    for (int t = 60; t < 80; ++t) R(x3, K3, w[t]);
    out[0] = 0x67452301u + a; out[1] = 0xefcdab89u + b; out[2] = 0x98badcfeu + c; out[3] = 0x10325476u + d; out[4] = 0xc3d2e1f0u + e;
}

extern "C" __global__ void k_chain(uint32_t *io, unsigned long long *cyc, int n, int mode) {
    uint32_t s[5]; for (int k = 0; k < 5; ++k) s[k] = io[threadIdx.x * 5 + k];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {
        for (int it = 0; it < n; ++it) { uint32_t o[5]; spawn_old(s, it & 3, o); for (int k = 0; k < 5; ++k) s[k] = o[k]; }
    } else if (mode == 1) {
        for (int it = 0; it < n; ++it) { uint32_t o[5]; spawn_new(s, it & 3, o); for (int k = 0; k < 5; ++k) s[k] = o[k]; }
    } else if (mode == 2) {  // two independent chains interleaved
        uint32_t s2[5]; for (int k = 0; k < 5; ++k) s2[k] = s[k] ^ 0x1234u;
        for (int it = 0; it < n; it += 2) { uint32_t o[5], o2[5]; spawn_new(s, it & 3, o); spawn_new(s2, it & 3, o2);
            for (int k = 0; k < 5; ++k) { s[k] = o[k]; s2[k] = o2[k]; } }
        for (int k = 0; k < 5; ++k) s[k] ^= s2[k];
    } else if (mode == 3) {  // dependent add3 chain: 100 per iter
        uint32_t x = s[0], y = s[1], z = s[2];
        for (int it = 0; it < n; ++it) {
#pragma unroll
            for (int j = 0; j < 100; ++j) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z)); }
        }
        s[0] = x;
    } else if (mode == 4) {  // 4 independent add3 chains
        uint32_t x = s[0], x2 = s[3], x3_ = s[4], x4 = s[1] ^ 7, y = s[1], z = s[2];
        for (int it = 0; it < n; ++it) {
#pragma unroll
            for (int j = 0; j < 25; ++j) { asm volatile("v_add3_u32 %0, %0, %4, %5\n v_add3_u32 %1, %1, %4, %5\n v_add3_u32 %2, %2, %4, %5\n v_add3_u32 %3, %3, %4, %5" : "+v"(x), "+v"(x2), "+v"(x3_), "+v"(x4) : "v"(y), "v"(z)); }
        }
        s[0] = x ^ x2 ^ x3_ ^ x4;
    } else if (mode == 5) {  // dependent alignbit chain
        uint32_t x = s[0];
        for (int it = 0; it < n; ++it) {
#pragma unroll
            for (int j = 0; j < 100; ++j) { asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x)); }
        }
        s[0] = x;
    } else if (mode == 6) {  // dependent bitop3 chain
        uint32_t x = s[0], y = s[1], z = s[2];
        for (int it = 0; it < n; ++it) {
#pragma unroll
            for (int j = 0; j < 100; ++j) { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z)); }
        }
        s[0] = x;
    } else if (mode == 7) {  // LDS round trip chain
        __shared__ uint32_t lds[64];
        lds[threadIdx.x] = threadIdx.x;
        __syncthreads();
        uint32_t x = threadIdx.x;
        for (int it = 0; it < n; ++it) {
#pragma unroll
            for (int j = 0; j < 100; ++j) { x = lds[x & 63]; }
        }
        s[0] = x;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[threadIdx.x * 5 + k] = s[k];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
#include <stdio.h>
#include <vector>
int main() {
    uint32_t *io; unsigned long long *cyc;
    hipMalloc(&io, 64 * 5 * 4 * 1024); hipMalloc(&cyc, 8 * 1024);
    hipMemset(io, 1, 64 * 5 * 4 * 1024);
    const char *names[] = {"sha1 generic", "sha1 bitop3", "sha1 bitop3 x2 interleaved (per sha)", "dep add3", "4 indep add3 (per op)", "dep alignbit", "dep bitop3", "lds dep load"};
    for (int mode = 0; mode < 8; ++mode) {
        for (int grid : {1, 256 * 4}) {
            int n = mode <= 2 ? 2000 : 200;
            hipLaunchKernelGGL(k_chain, dim3(grid), dim3(64), 0, 0, io, cyc, n, mode);
            hipDeviceSynchronize();
            hipLaunchKernelGGL(k_chain, dim3(grid), dim3(64), 0, 0, io, cyc, n, mode);
            hipDeviceSynchronize();
            unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            double per = (double)c / n;
            if (mode >= 3) per /= 100.0;
            printf("%-40s grid=%5d cycles/unit=%.2f\n", names[mode], grid, per);
        }
    }
    return 0;
}
