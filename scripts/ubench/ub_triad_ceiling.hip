// ub_triad_ceiling.hip — the HBM ceiling of the forasync triad's access mix
// (VERDICT r05 item 8): 2 read streams + 1 write stream, 12 B per element,
// 2^28 fp32 per array, the three arrays in one allocation staggered by
// 2 MiB + 4 KiB exactly as bench.py lays them out. Every form is timed with
// hipEvents over 20 launches after 3 warm-ups (average and best single
// launch). Forms:
//   read2   : the two read streams alone (float4 nt loads)      -> 8 B/elem
//   write1  : the write stream alone (float4 nt stores)         -> 4 B/elem
//   copy    : one read + one write stream                       -> 8 B/elem
//   triad   : float4 nt loads to VGPRs + nt stores (the product's form),
//             U (b, c) pairs in flight per lane, grid-stride or one
//             contiguous slice per workgroup
//   triadL  : LDS-DMA reads (global_load_lds, 16 B per lane, nt or default
//             policy) through a D-deep per-wave LDS ring + nt stores — the
//             guide's ldsdma-fill row (6.5-6.8 TB/s read-only, nt)
// at 1, 2, 3, 4 and 8 workgroups of 256 threads per CU; `triad U1 pf` is the
// product's form software-pipelined (next loads before this store).
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench/ub_triad_ceiling.hip -o scripts/ubench/ub_triad_ceiling.bin
#include <hip/hip_runtime.h>
#include <string>
#include <stdint.h>
#include <stdio.h>

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int64_t N = 1ll << 28, N4 = N / 4;

template <int U>
__global__ __launch_bounds__(256) void k_read2(const v4f *__restrict__ b, const v4f *__restrict__ c, float *out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    v4f acc = {0, 0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N4; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) acc += __builtin_nontemporal_load(&b[j]) + __builtin_nontemporal_load(&c[j]);
        }
    }
    if (acc.x == -1.f) out[0] = acc.y;  // never true for inputs >= 0
}

template <int U>
__global__ __launch_bounds__(256) void k_write1(v4f *__restrict__ a, float s) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    const v4f v = {s, s, s, s};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N4; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) __builtin_nontemporal_store(v, &a[j]);
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_copy(v4f *__restrict__ a, const v4f *__restrict__ b) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N4; i += U * stride) {
        v4f vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) vb[u] = __builtin_nontemporal_load(&b[j]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < N4) __builtin_nontemporal_store(vb[u], &a[j]);
        }
    }
}

template <int U, bool CONTIG>
__global__ __launch_bounds__(256) void k_triad(v4f *__restrict__ a, const v4f *__restrict__ b,
                                               const v4f *__restrict__ c, float s) {
    int64_t i, end, stride;
    if (CONTIG) {
        const int64_t q = 256 * U;
        const int64_t span = ((N4 + gridDim.x - 1) / gridDim.x + q - 1) / q * q;
        i = (int64_t)blockIdx.x * span + threadIdx.x;
        end = (int64_t)blockIdx.x * span + span;
        if (end > N4) end = N4;
        stride = 256;
    } else {
        i = (int64_t)blockIdx.x * 256 + threadIdx.x;
        end = N4;
        stride = (int64_t)gridDim.x * 256;
    }
    for (; i < end; i += U * stride) {
        v4f vb[U], vc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < end) {
                vb[u] = __builtin_nontemporal_load(&b[j]);
                vc[u] = __builtin_nontemporal_load(&c[j]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * stride;
            if (j < end) __builtin_nontemporal_store(vb[u] + s * vc[u], &a[j]);
        }
    }
}

// the product's form (U = 1, grid-stride) software-pipelined: the next
// element's two loads are issued before this element's store
__global__ __launch_bounds__(256) void k_triad_pf(v4f *__restrict__ a, const v4f *__restrict__ b,
                                                  const v4f *__restrict__ c, float s) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N4) return;
    v4f vb = __builtin_nontemporal_load(&b[i]), vc = __builtin_nontemporal_load(&c[i]);
    for (; i < N4; i += stride) {
        const int64_t j = i + stride < N4 ? i + stride : i;
        const v4f nb = __builtin_nontemporal_load(&b[j]), nc = __builtin_nontemporal_load(&c[j]);
        __builtin_nontemporal_store(vb + s * vc, &a[i]);
        vb = nb;
        vc = nc;
    }
}

// LDS-DMA: each wave streams its own 64-float4 chunks of b and c into a
// D-deep LDS ring, consumes the oldest chunk once its two DMAs landed, and
// stores a non-temporally. AUX: the DMA's cache policy (2 = nt, 0 = default).
template <int D, int AUX>
__global__ __launch_bounds__(256) void k_triad_lds(v4f *__restrict__ a, const v4f *__restrict__ b,
                                                   const v4f *__restrict__ c, float s) {
    __shared__ v4f ring[4][D][2][64];  // [wave][stage][b|c][lane]
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t wstride = (int64_t)gridDim.x * 4 * 64;
    const int64_t base = ((int64_t)blockIdx.x * 4 + w) * 64;
    const int64_t steps = base < N4 ? (N4 - base + wstride - 1) / wstride : 0;
    auto issue = [&](int64_t t) {
        const int st = (int)(t % D);
        const int64_t j = base + t * wstride + lane;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(b + j),
                                         (void __attribute__((address_space(3))) *)&ring[w][st][0][0], 16, 0, AUX);
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(c + j),
                                         (void __attribute__((address_space(3))) *)&ring[w][st][1][0], 16, 0, AUX);
    };
    int64_t t = 0;
    for (; t < D && t < steps; ++t) issue(t);
    for (int64_t k = 0; k < steps; ++k) {
        // stage k's two DMAs landed once at most 2D - 2 younger ops are
        // outstanding (younger: 2 DMAs per later stage in flight, D - 1 or
        // more, and the stores issued since; vmcnt retires in order)
        if (steps - k < D) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D - 2) : "memory");
        const int st = (int)(k % D);
        const v4f vb = ring[w][st][0][lane], vc = ring[w][st][1][lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (t < steps) {
            issue(t);
            ++t;
        }
        __builtin_nontemporal_store(vb + s * vc, &a[base + k * wstride + lane]);
    }
}

static hipEvent_t e0, e1;
template <typename F>
void timeit(const char *name, int bpc, double bytes, F f) {
    for (int i = 0; i < 3; ++i) f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) f();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    float best = 1e9f;
    for (int i = 0; i < 10; ++i) {
        (void)hipEventRecord(e0);
        f();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float one;
        (void)hipEventElapsedTime(&one, e0, e1);
        if (one < best) best = one;
    }
    printf("{\"form\": \"%s\", \"wg_per_cu\": %d, \"avg_ms\": %.4f, \"gbs_avg\": %.1f, \"gbs_best\": %.1f}\n", name, bpc,
           ms, bytes / ms / 1e6, bytes / best / 1e6);
    fflush(stdout);
}

// `quick` (bench.py's live ceiling): the read-only, write-only and best
// triad forms of the full sweep at 1 and 2 workgroups per CU only
int main(int argc, char **argv) {
    const bool quick = argc > 1 && std::string(argv[1]) == "quick";
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int64_t pad = 0x201000 / 4;
    float *buf, *o;
    if (hipMalloc(&buf, (3 * N + 2 * pad) * 4) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, (3 * N + 2 * pad) * 4);
    v4f *b = (v4f *)buf, *c = (v4f *)(buf + N + pad), *a = (v4f *)(buf + 2 * N + 2 * pad);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int bpc : {1, 2, 3, 4, 8}) {
        const dim3 g(cus * bpc), t(256);
        if (quick) {
            if (bpc > 2) break;
            timeit("read2 U2", bpc, 8.0 * N, [&] { hipLaunchKernelGGL(k_read2<2>, g, t, 0, 0, b, c, o); });
            timeit("write1 U4", bpc, 4.0 * N, [&] { hipLaunchKernelGGL(k_write1<4>, g, t, 0, 0, a, 3.f); });
            timeit("triad U1", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad<1, false>), g, t, 0, 0, a, b, c, 3.f); });
            timeit("triad U1 pf", bpc, 12.0 * N, [&] { hipLaunchKernelGGL(k_triad_pf, g, t, 0, 0, a, b, c, 3.f); });
            timeit("triadL D2 nt", bpc, 12.0 * N,
                   [&] { hipLaunchKernelGGL((k_triad_lds<2, 2>), g, t, 0, 0, a, b, c, 3.f); });
            timeit("triadL D4 nt", bpc, 12.0 * N,
                   [&] { hipLaunchKernelGGL((k_triad_lds<4, 2>), g, t, 0, 0, a, b, c, 3.f); });
            continue;
        }
        timeit("read2 U2", bpc, 8.0 * N, [&] { hipLaunchKernelGGL(k_read2<2>, g, t, 0, 0, b, c, o); });
        timeit("read2 U4", bpc, 8.0 * N, [&] { hipLaunchKernelGGL(k_read2<4>, g, t, 0, 0, b, c, o); });
        timeit("write1 U4", bpc, 4.0 * N, [&] { hipLaunchKernelGGL(k_write1<4>, g, t, 0, 0, a, 3.f); });
        timeit("copy U2", bpc, 8.0 * N, [&] { hipLaunchKernelGGL(k_copy<2>, g, t, 0, 0, a, b); });
        timeit("triad U1", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad<1, false>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triad U2", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad<2, false>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triad U4", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad<4, false>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triad U1 pf", bpc, 12.0 * N, [&] { hipLaunchKernelGGL(k_triad_pf, g, t, 0, 0, a, b, c, 3.f); });
        timeit("triad U1 contig", bpc, 12.0 * N,
               [&] { hipLaunchKernelGGL((k_triad<1, true>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triad U2 contig", bpc, 12.0 * N,
               [&] { hipLaunchKernelGGL((k_triad<2, true>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triadL D2 nt", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad_lds<2, 2>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triadL D4 nt", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad_lds<4, 2>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triadL D8 nt", bpc, 12.0 * N, [&] { hipLaunchKernelGGL((k_triad_lds<8, 2>), g, t, 0, 0, a, b, c, 3.f); });
        timeit("triadL D4 default", bpc, 12.0 * N,
               [&] { hipLaunchKernelGGL((k_triad_lds<4, 0>), g, t, 0, 0, a, b, c, 3.f); });
    }
    return 0;
}
