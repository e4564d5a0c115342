// Microbenchmark: latency of one dependent rng_spawn SHA-1 per step, computed
// by one wave alone vs split over two waves of a workgroup (the helper wave
// computes the message schedule W[16..79] into LDS while the round wave runs
// rounds 0..15 on W[0..15], then consumes W in 16-word chunks behind LDS
// flags). Checks both give the same chain. Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/ubench/ub_sha_split.hip -o /tmp/ub_sha_split
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t rl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t fch(uint32_t b, uint32_t c, uint32_t d) { return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA); }
__device__ __forceinline__ uint32_t fmaj(uint32_t b, uint32_t c, uint32_t d) { return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); }
#define R(F, K, W) { uint32_t t_ = rl(a, 5) + F(b, c, d) + e + ((K) + (W)); e = d; d = c; c = rl(b, 30); b = a; a = t_; }
constexpr uint32_t C6 = 0x80000000u, C15 = 192u;
constexpr uint32_t K0 = 0x5a827999u, K1 = 0x6ed9eba1u, K2 = 0x8f1bbcdcu, K3 = 0xca62c1d6u;

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

// rounds 0..15 (W0..W5 live, W6..W15 constants)
#define ROUNDS_0_15()                                                          \
    {                                                                          \
        uint32_t t_ = rl(a, 5) + (d ^ (b & (c ^ d))) + e + K0 + p[0];          \
        e = d; d = c; c = rl(b, 30); b = a; a = t_;                            \
        R(fch, K0, p[1]); R(fch, K0, p[2]); R(fch, K0, p[3]); R(fch, K0, p[4]); \
        R(fch, K0, i); R(fch, K0, C6);                                         \
        _Pragma("unroll") for (int t = 7; t < 15; ++t) R(fch, K0, 0u);         \
        R(fch, K0, C15);                                                       \
    }

__device__ __forceinline__ void spawn_one(const uint32_t p[5], uint32_t i, uint32_t out[5]) {
    uint32_t w[80];
    sched(p, i, w);
    uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
    ROUNDS_0_15();
#pragma unroll
    for (int t = 16; t < 20; ++t) R(fch, K0, w[t]);
#pragma unroll
    for (int t = 20; t < 40; ++t) R(x3, K1, w[t]);
#pragma unroll
    for (int t = 40; t < 60; ++t) R(fmaj, K2, w[t]);
#pragma unroll
    for (int t = 60; t < 80; ++t) R(x3, K3, w[t]);
    out[0] = 0x67452301u + a; out[1] = 0xefcdab89u + b; out[2] = 0x98badcfeu + c; out[3] = 0x10325476u + d;
    out[4] = 0xc3d2e1f0u + e;
}

// one wave alone
extern "C" __global__ void k_one(uint32_t *io, unsigned long long *cyc, int n) {
    const int lane = threadIdx.x;
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        uint32_t o[5];
        spawn_one(s, (uint32_t)(it & 3), o);
        for (int k = 0; k < 5; ++k) s[k] = o[k];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = s[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// rounds-only floor: the schedule of the first step reused every step (wrong
// values, right instruction stream of the round wave)
extern "C" __global__ void k_rounds(uint32_t *io, unsigned long long *cyc, int n) {
    const int lane = threadIdx.x;
    uint32_t p[5];
    for (int k = 0; k < 5; ++k) p[k] = io[lane * 5 + k];
    uint32_t w[80];
    sched(p, 1, w);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t i = (uint32_t)(it & 3);
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        ROUNDS_0_15();
#pragma unroll
        for (int t = 16; t < 20; ++t) R(fch, K0, w[t]);
#pragma unroll
        for (int t = 20; t < 40; ++t) R(x3, K1, w[t]);
#pragma unroll
        for (int t = 40; t < 60; ++t) R(fmaj, K2, w[t]);
#pragma unroll
        for (int t = 60; t < 80; ++t) R(x3, K3, w[t]);
        p[0] = 0x67452301u + a; p[1] = 0xefcdab89u + b; p[2] = 0x98badcfeu + c; p[3] = 0x10325476u + d;
        p[4] = 0xc3d2e1f0u + e;
        asm volatile("" : "+v"(w[16]), "+v"(w[40]), "+v"(w[79]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = p[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// two waves: wave 0 = rounds, wave 1 = schedule
struct Split {
    uint4 w[16][64];        // W[16..79] as 16 groups of 4 words, lane-contiguous
    uint32_t p[6][64];      // parent state + child index of the step
    uint32_t flag_in;       // step number whose inputs are posted (+1)
    uint32_t flag_w[4];     // chunk c of step it ready: it + 1
};

__device__ __forceinline__ uint32_t lds_ld(volatile uint32_t *p) { return *p; }

extern "C" __global__ void k_split(uint32_t *io, unsigned long long *cyc, int n, int prio_mode) {
    __shared__ Split sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        sh.flag_in = 0;
        for (int c = 0; c < 4; ++c) sh.flag_w[c] = 0;
    }
    __syncthreads();
    if (wave == 1) {
        for (int it = 0; it < n; ++it) {
            for (uint32_t sp = 0; lds_ld(&sh.flag_in) != (uint32_t)(it + 1) && sp < (1u << 22); ++sp) __builtin_amdgcn_s_sleep(0);
            asm volatile("" ::: "memory");
            uint32_t p[5];
            for (int k = 0; k < 5; ++k) p[k] = sh.p[k][lane];
            const uint32_t i = sh.p[5][lane];
            uint32_t w[80];
            sched(p, i, w);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int t = 16 + c * 16 + g * 4;
                    sh.w[c * 4 + g][lane] = make_uint4(w[t], w[t + 1], w[t + 2], w[t + 3]);
                }
                // LDS ops of one wave complete in order: the flag lands after the chunk
                asm volatile("" ::: "memory");
                if (lane == 0) *(volatile uint32_t *)&sh.flag_w[c] = (uint32_t)(it + 1);
            }
        }
        return;
    }
    if (prio_mode) __builtin_amdgcn_s_setprio(3);
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t i = (uint32_t)(it & 3);
        for (int k = 0; k < 5; ++k) sh.p[k][lane] = s[k];
        sh.p[5][lane] = i;
        asm volatile("" ::: "memory");
        if (lane == 0) *(volatile uint32_t *)&sh.flag_in = (uint32_t)(it + 1);
        const uint32_t *p = s;
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        ROUNDS_0_15();
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
            for (uint32_t sp = 0; lds_ld(&sh.flag_w[ch]) != (uint32_t)(it + 1) && sp < (1u << 22); ++sp) {}
            asm volatile("" ::: "memory");
            uint32_t w[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint4 v = sh.w[ch * 4 + g][lane];
                w[g * 4] = v.x; w[g * 4 + 1] = v.y; w[g * 4 + 2] = v.z; w[g * 4 + 3] = v.w;
            }
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int tt = 16 + ch * 16 + t;
                if (tt < 20) R(fch, K0, w[t])
                else if (tt < 40) R(x3, K1, w[t])
                else if (tt < 60) R(fmaj, K2, w[t])
                else R(x3, K3, w[t])
            }
        }
        s[0] = 0x67452301u + a; s[1] = 0xefcdab89u + b; s[2] = 0x98badcfeu + c; s[3] = 0x10325476u + d;
        s[4] = 0xc3d2e1f0u + e;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = s[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// reassociated round: X = F + e + KW (independent of a), a' = rl5(a) + X (2 dependent ops per round)
__device__ __forceinline__ uint32_t add_pin(uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
#define R2(F, KW) { const uint32_t x_ = F(b, c, d) + e + (KW); const uint32_t t_ = add_pin(rl(a, 5), x_); e = d; d = c; c = rl(b, 30); b = a; a = t_; }

__device__ __forceinline__ void spawn_one2(const uint32_t p[5], uint32_t i, uint32_t out[5]) {
    uint32_t w[80];
    sched(p, i, w);
    uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
    R2(fch, K0 + p[0]); R2(fch, K0 + p[1]); R2(fch, K0 + p[2]); R2(fch, K0 + p[3]); R2(fch, K0 + p[4]);
    R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
    for (int t = 7; t < 15; ++t) R2(fch, K0);
    R2(fch, K0 + C15);
#pragma unroll
    for (int t = 16; t < 20; ++t) R2(fch, K0 + w[t]);
#pragma unroll
    for (int t = 20; t < 40; ++t) R2(x3, K1 + w[t]);
#pragma unroll
    for (int t = 40; t < 60; ++t) R2(fmaj, K2 + w[t]);
#pragma unroll
    for (int t = 60; t < 80; ++t) R2(x3, K3 + w[t]);
    out[0] = 0x67452301u + a; out[1] = 0xefcdab89u + b; out[2] = 0x98badcfeu + c; out[3] = 0x10325476u + d;
    out[4] = 0xc3d2e1f0u + e;
}

extern "C" __global__ void k_one2(uint32_t *io, unsigned long long *cyc, int n) {
    const int lane = threadIdx.x;
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        uint32_t o[5];
        spawn_one2(s, (uint32_t)(it & 3), o);
        for (int k = 0; k < 5; ++k) s[k] = o[k];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = s[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" __global__ void k_rounds2(uint32_t *io, unsigned long long *cyc, int n) {
    const int lane = threadIdx.x;
    uint32_t p[5];
    for (int k = 0; k < 5; ++k) p[k] = io[lane * 5 + k];
    uint32_t w[80];
    sched(p, 1, w);
    uint32_t kw[80];
#pragma unroll
    for (int t = 16; t < 80; ++t) kw[t] = w[t] + (t < 20 ? K0 : t < 40 ? K1 : t < 60 ? K2 : K3);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t i = (uint32_t)(it & 3);
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        R2(fch, K0 + p[0]); R2(fch, K0 + p[1]); R2(fch, K0 + p[2]); R2(fch, K0 + p[3]); R2(fch, K0 + p[4]);
        R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
        for (int t = 7; t < 15; ++t) R2(fch, K0);
        R2(fch, K0 + C15);
#pragma unroll
        for (int t = 16; t < 20; ++t) R2(fch, kw[t]);
#pragma unroll
        for (int t = 20; t < 40; ++t) R2(x3, kw[t]);
#pragma unroll
        for (int t = 40; t < 60; ++t) R2(fmaj, kw[t]);
#pragma unroll
        for (int t = 60; t < 80; ++t) R2(x3, kw[t]);
        p[0] = 0x67452301u + a; p[1] = 0xefcdab89u + b; p[2] = 0x98badcfeu + c; p[3] = 0x10325476u + d;
        p[4] = 0xc3d2e1f0u + e;
        asm volatile("" : "+v"(kw[16]), "+v"(kw[40]), "+v"(kw[79]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = p[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// split v2: the helper writes KW = K + W per chunk followed by a per-lane tag
// (the batch number); the worker reads chunk c+1 (tag first, then data: LDS
// serves one wave's reads in order, so a fresh tag vouches for the data read
// after it) while it runs chunk c's rounds, and re-reads only on a stale tag
struct Split2 {
    uint4 kw[4][5][64];     // chunk c: 4 groups of 4 KW words + {tag, -, -, -}
    uint4 p0[64];
    uint2 p1[64];
    uint32_t flag_in;
};

__device__ __forceinline__ void ld_chunk(Split2 &sh, int ch, int lane, uint32_t &tag, uint32_t w[16]) {
    tag = *(volatile uint32_t *)&sh.kw[ch][4][lane].x;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const uint4 v = sh.kw[ch][g][lane];
        w[g * 4] = v.x; w[g * 4 + 1] = v.y; w[g * 4 + 2] = v.z; w[g * 4 + 3] = v.w;
    }
}

extern "C" __global__ void k_split2(uint32_t *io, unsigned long long *cyc, int n, int prio_mode) {
    __shared__ Split2 sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < 64) {
        sh.flag_in = 0;
        for (int c = 0; c < 4; ++c) sh.kw[c][4][lane] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    if (wave == 1) {
        for (int it = 0; it < n; ++it) {
            for (uint32_t sp = 0; *(volatile uint32_t *)&sh.flag_in != (uint32_t)(it + 1) && sp < (1u << 22); ++sp) {}
            asm volatile("" ::: "memory");
            const uint4 a = sh.p0[lane];
            const uint2 b = sh.p1[lane];
            const uint32_t p[5] = {a.x, a.y, a.z, a.w, b.x};
            uint32_t w[80];
            sched(p, b.y, w);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int t = 16 + c * 16 + g * 4;
                    const uint32_t K = t < 20 ? K0 : t < 40 ? K1 : t < 60 ? K2 : K3;
                    const uint32_t K_ = t + 4 <= 20 ? K0 : t + 4 <= 40 ? K1 : t + 4 <= 60 ? K2 : K3;
                    (void)K_;
                    uint32_t q[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int tt = t + j;
                        q[j] = w[tt] + (tt < 20 ? K0 : tt < 40 ? K1 : tt < 60 ? K2 : K3);
                    }
                    (void)K;
                    sh.kw[c][g][lane] = make_uint4(q[0], q[1], q[2], q[3]);
                }
                asm volatile("" ::: "memory");
                *(volatile uint32_t *)&sh.kw[c][4][lane].x = (uint32_t)(it + 1);
                // keep the next chunk's arithmetic below this chunk's stores
                asm volatile("" ::: "memory");
            }
        }
        return;
    }
    if (prio_mode) __builtin_amdgcn_s_setprio(3);
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t seq = (uint32_t)(it + 1);
        const uint32_t i = (uint32_t)(it & 3);
        sh.p0[lane] = make_uint4(s[0], s[1], s[2], s[3]);
        sh.p1[lane] = make_uint2(s[4], i);
        asm volatile("" ::: "memory");
        if (lane == 0) *(volatile uint32_t *)&sh.flag_in = seq;
        const uint32_t *p = s;
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        R2(fch, K0 + p[0]); R2(fch, K0 + p[1]); R2(fch, K0 + p[2]); R2(fch, K0 + p[3]); R2(fch, K0 + p[4]);
        R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
        for (int t = 7; t < 13; ++t) R2(fch, K0);
        uint32_t tag, wn[16];
        ld_chunk(sh, 0, lane, tag, wn);
        R2(fch, K0); R2(fch, K0);
        R2(fch, K0 + C15);
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
            uint32_t w[16];
            // stale tag (the helper was late): re-read until fresh
            for (uint32_t sp = 0; __builtin_amdgcn_readfirstlane(__ballot(tag != seq) != 0) && sp < (1u << 22); ++sp)
                ld_chunk(sh, ch, lane, tag, wn);
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = wn[k];
            if (ch < 3) ld_chunk(sh, ch + 1, lane, tag, wn);
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int tt = 16 + ch * 16 + t;
                if (tt < 20) R2(fch, w[t])
                else if (tt < 40) R2(x3, w[t])
                else if (tt < 60) R2(fmaj, w[t])
                else R2(x3, w[t])
            }
        }
        s[0] = 0x67452301u + a; s[1] = 0xefcdab89u + b; s[2] = 0x98badcfeu + c; s[3] = 0x10325476u + d;
        s[4] = 0xc3d2e1f0u + e;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = s[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// split v3: the helper's poll reads the flag and the inputs in one round trip
// (flag first); the schedule is computed chunk by chunk (pinned with asm so
// the compiler cannot hoist later chunks above earlier stores); the worker
// reads chunk c+1 half way through chunk c
__device__ __forceinline__ uint32_t kof(int t) { return t < 20 ? K0 : t < 40 ? K1 : t < 60 ? K2 : K3; }

extern "C" __global__ void k_split3(uint32_t *io, unsigned long long *cyc, int n, int prio_mode) {
    __shared__ Split2 sh;
    unsigned long long wait_cyc[4] = {0, 0, 0, 0}, wait_sp[4] = {0, 0, 0, 0};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < 64) {
        sh.flag_in = 0;
        for (int c = 0; c < 4; ++c) sh.kw[c][4][lane] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    if (wave == 1) {
        for (int it = 0; it < n; ++it) {
            uint4 a;
            uint2 b;
            for (uint32_t sp = 0; sp < (1u << 22); ++sp) {
                const uint32_t f = *(volatile uint32_t *)&sh.flag_in;
                asm volatile("" ::: "memory");
                a = sh.p0[lane];
                b = sh.p1[lane];
                if (f == (uint32_t)(it + 1)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            uint32_t w[80];
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (c == 0) {
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
                } else {
#pragma unroll
                    for (int t = 16 + 16 * c; t < 32 + 16 * c; ++t) w[t] = rl(x3(w[t - 3], w[t - 8], w[t - 14]) ^ w[t - 16], 1);
                }
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int t = 16 + c * 16 + g * 4;
                    sh.kw[c][g][lane] = make_uint4(w[t] + kof(t), w[t + 1] + kof(t + 1), w[t + 2] + kof(t + 2), w[t + 3] + kof(t + 3));
                }
                asm volatile("" ::: "memory");
                *(volatile uint32_t *)&sh.kw[c][4][lane].x = (uint32_t)(it + 1);
                // pin the window the next chunk reads: its arithmetic stays below these stores
                const int b0 = 16 + 16 * c;
                asm volatile("" : "+v"(w[b0 + 0]), "+v"(w[b0 + 1]), "+v"(w[b0 + 2]), "+v"(w[b0 + 3]),
                                  "+v"(w[b0 + 4]), "+v"(w[b0 + 5]), "+v"(w[b0 + 6]), "+v"(w[b0 + 7]),
                                  "+v"(w[b0 + 8]), "+v"(w[b0 + 9]), "+v"(w[b0 + 10]), "+v"(w[b0 + 11]),
                                  "+v"(w[b0 + 12]), "+v"(w[b0 + 13]), "+v"(w[b0 + 14]), "+v"(w[b0 + 15]) :: "memory");
            }
        }
        return;
    }
    if (prio_mode) __builtin_amdgcn_s_setprio(3);
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t seq = (uint32_t)(it + 1);
        const uint32_t i = (uint32_t)(it & 3);
        sh.p0[lane] = make_uint4(s[0], s[1], s[2], s[3]);
        sh.p1[lane] = make_uint2(s[4], i);
        asm volatile("" ::: "memory");
        if (lane == 0) *(volatile uint32_t *)&sh.flag_in = seq;
        const uint32_t *p = s;
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        R2(fch, K0 + p[0]); R2(fch, K0 + p[1]); R2(fch, K0 + p[2]); R2(fch, K0 + p[3]); R2(fch, K0 + p[4]);
        R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
        for (int t = 7; t < 15; ++t) R2(fch, K0);
        R2(fch, K0 + C15);
        uint32_t tag, wn[16];
        ld_chunk(sh, 0, lane, tag, wn);
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
            uint32_t w[16];
            const unsigned long long tw0 = __builtin_amdgcn_s_memtime();
            uint32_t sp = 0;
            for (; __builtin_amdgcn_readfirstlane(__ballot(tag != seq) != 0) && sp < (1u << 22); ++sp)
                ld_chunk(sh, ch, lane, tag, wn);
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = wn[k];
            asm volatile("" : "+v"(w[0]));
            wait_cyc[ch] += __builtin_amdgcn_s_memtime() - tw0;
            wait_sp[ch] += sp;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                if (t == 10 && ch < 3) ld_chunk(sh, ch + 1, lane, tag, wn);
                const int tt = 16 + ch * 16 + t;
                if (tt < 20) R2(fch, w[t])
                else if (tt < 40) R2(x3, w[t])
                else if (tt < 60) R2(fmaj, w[t])
                else R2(x3, w[t])
            }
        }
        s[0] = 0x67452301u + a; s[1] = 0xefcdab89u + b; s[2] = 0x98badcfeu + c; s[3] = 0x10325476u + d;
        s[4] = 0xc3d2e1f0u + e;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = s[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    if (lane == 0 && blockIdx.x == 0)
        for (int c = 0; c < 4; ++c) { cyc[1024 + c] = wait_cyc[c]; cyc[1028 + c] = wait_sp[c]; }
}

// split v4: the worker computes W16..W31 itself (cheap: many constant terms)
// and the helper W32..W79 in three chunks, which gives the helper the 32
// rounds 0..31 of slack before its first chunk is due
extern "C" __global__ void k_split4(uint32_t *io, unsigned long long *cyc, int n, int prio_mode) {
    __shared__ Split2 sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < 64) {
        sh.flag_in = 0;
        for (int c = 0; c < 4; ++c) sh.kw[c][4][lane] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    if (wave == 1) {
        for (int it = 0; it < n; ++it) {
            uint4 a;
            uint2 b;
            for (uint32_t sp = 0; sp < (1u << 22); ++sp) {
                const uint32_t f = *(volatile uint32_t *)&sh.flag_in;
                asm volatile("" ::: "memory");
                a = sh.p0[lane];
                b = sh.p1[lane];
                if (f == (uint32_t)(it + 1)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            uint32_t w[80];
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y;
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
            for (int c = 1; c < 4; ++c) {
#pragma unroll
                for (int t = 16 + 16 * c; t < 32 + 16 * c; ++t) w[t] = rl(x3(w[t - 3], w[t - 8], w[t - 14]) ^ w[t - 16], 1);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int t = 16 + c * 16 + g * 4;
                    sh.kw[c][g][lane] = make_uint4(w[t] + kof(t), w[t + 1] + kof(t + 1), w[t + 2] + kof(t + 2), w[t + 3] + kof(t + 3));
                }
                asm volatile("" ::: "memory");
                *(volatile uint32_t *)&sh.kw[c][4][lane].x = (uint32_t)(it + 1);
                const int b0 = 16 + 16 * c;
                asm volatile("" : "+v"(w[b0 + 0]), "+v"(w[b0 + 1]), "+v"(w[b0 + 2]), "+v"(w[b0 + 3]),
                                  "+v"(w[b0 + 4]), "+v"(w[b0 + 5]), "+v"(w[b0 + 6]), "+v"(w[b0 + 7]),
                                  "+v"(w[b0 + 8]), "+v"(w[b0 + 9]), "+v"(w[b0 + 10]), "+v"(w[b0 + 11]),
                                  "+v"(w[b0 + 12]), "+v"(w[b0 + 13]), "+v"(w[b0 + 14]), "+v"(w[b0 + 15]) :: "memory");
            }
        }
        return;
    }
    if (prio_mode) __builtin_amdgcn_s_setprio(3);
    uint32_t s[5];
    for (int k = 0; k < 5; ++k) s[k] = io[lane * 5 + k];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < n; ++it) {
        const uint32_t seq = (uint32_t)(it + 1);
        const uint32_t i = (uint32_t)(it & 3);
        sh.p0[lane] = make_uint4(s[0], s[1], s[2], s[3]);
        sh.p1[lane] = make_uint2(s[4], i);
        asm volatile("" ::: "memory");
        if (lane == 0) *(volatile uint32_t *)&sh.flag_in = seq;
        const uint32_t *p = s;
        uint32_t w[32];
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
        uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
        R2(fch, K0 + p[0]); R2(fch, K0 + p[1]); R2(fch, K0 + p[2]); R2(fch, K0 + p[3]); R2(fch, K0 + p[4]);
        R2(fch, K0 + i); R2(fch, K0 + C6);
#pragma unroll
        for (int t = 7; t < 15; ++t) R2(fch, K0);
        R2(fch, K0 + C15);
        uint32_t tag, wn[16];
#pragma unroll
        for (int t = 16; t < 32; ++t) {
            if (t == 22) ld_chunk(sh, 1, lane, tag, wn);
            if (t < 20) R2(fch, K0 + w[t])
            else R2(x3, K1 + w[t])
        }
#pragma unroll
        for (int ch = 1; ch < 4; ++ch) {
            uint32_t wc[16];
            for (uint32_t sp = 0; __builtin_amdgcn_readfirstlane(__ballot(tag != seq) != 0) && sp < (1u << 22); ++sp)
                ld_chunk(sh, ch, lane, tag, wn);
#pragma unroll
            for (int k = 0; k < 16; ++k) wc[k] = wn[k];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                if (t == 6 && ch < 3) ld_chunk(sh, ch + 1, lane, tag, wn);
                const int tt = 16 + ch * 16 + t;
                if (tt < 40) R2(x3, wc[t])
                else if (tt < 60) R2(fmaj, wc[t])
                else R2(x3, wc[t])
            }
        }
        s[0] = 0x67452301u + a; s[1] = 0xefcdab89u + b; s[2] = 0x98badcfeu + c; s[3] = 0x10325476u + d;
        s[4] = 0xc3d2e1f0u + e;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 5; ++k) io[lane * 5 + k] = s[k];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const int n = 4000;
    uint32_t *io1, *io2, *io3;
    unsigned long long *cyc;
    hipMalloc(&io1, 64 * 5 * 4 * 2048);
    hipMalloc(&io2, 64 * 5 * 4 * 2048);
    hipMalloc(&io3, 64 * 5 * 4 * 2048);
    hipMalloc(&cyc, 8 * 2048);
    for (int grid : {1, 512}) {
        hipMemset(io1, 7, 64 * 5 * 4 * 2048);
        hipMemset(io2, 7, 64 * 5 * 4 * 2048);
        unsigned long long c1 = 0, c2 = 0, c3 = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipMemset(io1, 7, 64 * 5 * 4 * 2048);
            hipMemset(io2, 7, 64 * 5 * 4 * 2048);
            hipMemset(io3, 7, 64 * 5 * 4 * 2048);
            hipLaunchKernelGGL(k_one, dim3(grid), dim3(64), 0, 0, io1, cyc, n);
            hipDeviceSynchronize();
            hipMemcpy(&c1, cyc, 8, hipMemcpyDeviceToHost);
            hipLaunchKernelGGL(k_split, dim3(grid), dim3(128), 0, 0, io2, cyc, n, 0);
            hipDeviceSynchronize();
            hipMemcpy(&c2, cyc, 8, hipMemcpyDeviceToHost);
            hipLaunchKernelGGL(k_rounds, dim3(grid), dim3(64), 0, 0, io3, cyc, n);
            hipDeviceSynchronize();
            hipMemcpy(&c3, cyc, 8, hipMemcpyDeviceToHost);
        }
        unsigned long long c4 = 0, c5 = 0, c6 = 0;
        uint32_t *io4 = io3;
        hipMemset(io3, 7, 64 * 5 * 4 * 2048);
        hipLaunchKernelGGL(k_one2, dim3(grid), dim3(64), 0, 0, io3, cyc, n);
        hipDeviceSynchronize();
        hipMemcpy(&c4, cyc, 8, hipMemcpyDeviceToHost);
        uint32_t h4[320];
        hipMemcpy(h4, io3, sizeof(h4), hipMemcpyDeviceToHost);
        hipMemset(io4, 7, 64 * 5 * 4 * 2048);
        hipLaunchKernelGGL(k_split2, dim3(grid), dim3(128), 0, 0, io4, cyc, n, 0);
        hipDeviceSynchronize();
        hipMemcpy(&c5, cyc, 8, hipMemcpyDeviceToHost);
        uint32_t h5[320];
        hipMemcpy(h5, io4, sizeof(h5), hipMemcpyDeviceToHost);
        unsigned long long c7 = 0;
        hipMemset(io4, 7, 64 * 5 * 4 * 2048);
        hipLaunchKernelGGL(k_split3, dim3(grid), dim3(128), 0, 0, io4, cyc, n, 0);
        hipDeviceSynchronize();
        hipMemcpy(&c7, cyc, 8, hipMemcpyDeviceToHost);
        {
            unsigned long long c8 = 0;
            hipMemset(io4, 7, 64 * 5 * 4 * 2048);
            hipLaunchKernelGGL(k_split4, dim3(grid), dim3(128), 0, 0, io4, cyc, n, 0);
            hipDeviceSynchronize();
            hipMemcpy(&c8, cyc, 8, hipMemcpyDeviceToHost);
            uint32_t h8[320], h0[320];
            hipMemcpy(h8, io4, sizeof(h8), hipMemcpyDeviceToHost);
            hipMemcpy(h0, io1, sizeof(h0), hipMemcpyDeviceToHost);
            int s8 = 1;
            for (int k = 0; k < 320; ++k) s8 &= h0[k] == h8[k];
            printf("grid=%4d split4 %.1f (match %d)\n", grid, (double)c8 / n, s8);
            hipMemset(io4, 7, 64 * 5 * 4 * 2048);
            hipLaunchKernelGGL(k_split4, dim3(grid), dim3(128), 0, 0, io4, cyc, n, 1);
            hipDeviceSynchronize();
            hipMemcpy(&c8, cyc, 8, hipMemcpyDeviceToHost);
            hipMemcpy(h8, io4, sizeof(h8), hipMemcpyDeviceToHost);
            s8 = 1;
            for (int k = 0; k < 320; ++k) s8 &= h0[k] == h8[k];
            printf("grid=%4d split4+prio %.1f (match %d)\n", grid, (double)c8 / n, s8);
            hipMemset(io4, 7, 64 * 5 * 4 * 2048);
            hipLaunchKernelGGL(k_split3, dim3(grid), dim3(128), 0, 0, io4, cyc, n, 1);
            hipDeviceSynchronize();
            hipMemcpy(&c8, cyc, 8, hipMemcpyDeviceToHost);
            printf("grid=%4d split3+prio %.1f\n", grid, (double)c8 / n);
        }
        unsigned long long wc[8];
        hipMemcpy(wc, cyc + 1024, sizeof(wc), hipMemcpyDeviceToHost);
        printf("split3 wait cycles/step per chunk: %.0f %.0f %.0f %.0f; re-reads/step: %.2f %.2f %.2f %.2f\n",
               (double)wc[0] / n, (double)wc[1] / n, (double)wc[2] / n, (double)wc[3] / n,
               (double)wc[4] / n, (double)wc[5] / n, (double)wc[6] / n, (double)wc[7] / n);
        uint32_t h7[320];
        hipMemcpy(h7, io4, sizeof(h7), hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(k_rounds2, dim3(grid), dim3(64), 0, 0, io3, cyc, n);
        hipDeviceSynchronize();
        hipMemcpy(&c6, cyc, 8, hipMemcpyDeviceToHost);
        uint32_t h1[320], h2[320];
        hipMemcpy(h1, io1, sizeof(h1), hipMemcpyDeviceToHost);
        hipMemcpy(h2, io2, sizeof(h2), hipMemcpyDeviceToHost);
        int same = 1;
        for (int k = 0; k < 320; ++k) same &= h1[k] == h2[k];
        int s4 = 1, s5 = 1, s7 = 1;
        for (int k = 0; k < 320; ++k) { s4 &= h1[k] == h4[k]; s5 &= h1[k] == h5[k]; s7 &= h1[k] == h7[k]; }
        printf("grid=%4d split3 %.1f (match %d)\n", grid, (double)c7 / n, s7);
        printf("grid=%4d one-wave reassoc %.1f (match %d) | split2 %.1f (match %d) | rounds2 floor %.1f\n", grid,
               (double)c4 / n, s4, (double)c5 / n, s5, (double)c6 / n);
        printf("grid=%4d one-wave %.1f cyc/step | split %.1f cyc/step (match %d) | rounds-only floor %.1f cyc/step\n",
               grid, (double)c1 / n, (double)c2 / n, same, (double)c3 / n);
    }
    return 0;
}
