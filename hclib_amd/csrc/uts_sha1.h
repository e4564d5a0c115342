// uts_sha1.h — the UTS rng_spawn SHA-1 (test/uts/rng/brg_sha1.c:68-83,
// 195-327) specialised for its one-block message, on gfx950 VALU idioms.
//
// rng_spawn: SHA1(parent || i) with the 24-byte message padding, specialised
// for the one-block message W = {p0..p4, i, 0x80000000, 0 x8, 192}: the
// schedule drops every known-zero term, the round functions are single
// v_bitop3_b32 ops (gfx950: ch 0xCA, parity 0x96, maj 0xE8), rotates are
// v_alignbit_b32 — ~550 VALU ops instead of ~740 for the generic block.
//
// rng_spawn_n<N> computes N independent spawns with their instructions
// interleaved step by step (round t of chain 0, round t of chain 1, ...): one
// wave's dependent SHA-1 chain issues a VALU op only every ~4-5 cycles, so a
// second independent chain in the same lane fills the issue slots the first
// leaves empty (instruction-level parallelism inside the wave, where more
// waves per SIMD are limited by LDS).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

namespace hx {

__device__ __forceinline__ uint32_t rl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t fch(uint32_t b, uint32_t c, uint32_t d) {
    return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);
}
__device__ __forceinline__ uint32_t fmaj(uint32_t b, uint32_t c, uint32_t d) {
    return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);
}

// one SHA-1 round of chain j
#define HX_RJ(F, K, W, j)                                               \
    {                                                                   \
        uint32_t t_ = rl(a[j], 5) + F(b[j], c[j], d[j]) + e[j] + ((K) + (W)); \
        e[j] = d[j];                                                    \
        d[j] = c[j];                                                    \
        c[j] = rl(b[j], 30);                                            \
        b[j] = a[j];                                                    \
        a[j] = t_;                                                      \
    }

template <int N>
__device__ __forceinline__ void rng_spawn_n(const uint32_t *const p[N], const uint32_t i[N], uint32_t *const out[N]) {
    constexpr uint32_t C6 = 0x80000000u, C15 = 192u;  // padding word, bit length
    constexpr uint32_t K0 = 0x5a827999u, K1 = 0x6ed9eba1u, K2 = 0x8f1bbcdcu, K3 = 0xca62c1d6u;
    uint32_t w[N][80];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        w[j][0] = p[j][0];
        w[j][1] = p[j][1];
        w[j][2] = p[j][2];
        w[j][3] = p[j][3];
        w[j][4] = p[j][4];
        w[j][5] = i[j];
    }
    // W[t] = rotl1(W[t-3]^W[t-8]^W[t-14]^W[t-16]) with W6 = C6, W7..W14 = 0, W15 = C15
#pragma unroll
    for (int j = 0; j < N; ++j) {
        w[j][16] = rl(w[j][2] ^ w[j][0], 1);
        w[j][17] = rl(w[j][3] ^ w[j][1], 1);
        w[j][18] = rl(x3(C15, w[j][4], w[j][2]), 1);
        w[j][19] = rl(x3(w[j][16], w[j][5], w[j][3]), 1);
        w[j][20] = rl(x3(w[j][17], C6, w[j][4]), 1);
        w[j][21] = rl(w[j][18] ^ w[j][5], 1);
        w[j][22] = rl(w[j][19] ^ C6, 1);
        w[j][23] = rl(w[j][20] ^ C15, 1);
    }
#pragma unroll
    for (int t = 24; t < 29; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) w[j][t] = rl(w[j][t - 3] ^ w[j][t - 8], 1);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        w[j][29] = rl(x3(w[j][26], w[j][21], C15), 1);
        w[j][30] = rl(x3(w[j][27], w[j][22], w[j][16]), 1);
        w[j][31] = rl(x3(w[j][28], w[j][23], w[j][17]) ^ C15, 1);
    }
#pragma unroll
    for (int t = 32; t < 80; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) w[j][t] = rl(x3(w[j][t - 3], w[j][t - 8], w[j][t - 14]) ^ w[j][t - 16], 1);
    uint32_t a[N], b[N], c[N], d[N], e[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        a[j] = 0x67452301u;
        b[j] = 0xefcdab89u;
        c[j] = 0x98badcfeu;
        d[j] = 0x10325476u;
        e[j] = 0xc3d2e1f0u;
    }
    // round 0: every input but W0 is a constant (folded by the compiler)
#pragma unroll
    for (int j = 0; j < N; ++j) HX_RJ(fch, K0, w[j][0], j);
#pragma unroll
    for (int t = 1; t < 6; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) HX_RJ(fch, K0, w[j][t], j);
#pragma unroll
    for (int j = 0; j < N; ++j) HX_RJ(fch, K0, C6, j);
#pragma unroll
    for (int t = 7; t < 15; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) HX_RJ(fch, K0, 0u, j);
#pragma unroll
    for (int j = 0; j < N; ++j) HX_RJ(fch, K0, C15, j);
#pragma unroll
    for (int t = 16; t < 20; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) HX_RJ(fch, K0, w[j][t], j);
#pragma unroll
    for (int t = 20; t < 40; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) HX_RJ(x3, K1, w[j][t], j);
#pragma unroll
    for (int t = 40; t < 60; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) HX_RJ(fmaj, K2, w[j][t], j);
#pragma unroll
    for (int t = 60; t < 80; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) HX_RJ(x3, K3, w[j][t], j);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        out[j][0] = 0x67452301u + a[j];
        out[j][1] = 0xefcdab89u + b[j];
        out[j][2] = 0x98badcfeu + c[j];
        out[j][3] = 0x10325476u + d[j];
        out[j][4] = 0xc3d2e1f0u + e[j];
    }
}
#undef HX_RJ

__device__ __forceinline__ void rng_spawn_dev(const uint32_t p[5], uint32_t i, uint32_t out[5]) {
    const uint32_t *pp[1] = {p};
    const uint32_t ii[1] = {i};
    uint32_t *oo[1] = {out};
    rng_spawn_n<1>(pp, ii, oo);
}

}  // namespace hx
