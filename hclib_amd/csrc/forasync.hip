// forasync.hip — hclib_forasync lowered to coalesced grid-stride tiles.
//
// The reference spawns one task per tile and calls the user function once
// per index through a pointer (forasync1D_runner, src/hclib.c:110-120;
// FLAT 316-351, RECURSIVE 158-190; 2-D/3-D 122-156, 192-314, 353-416). On the
// GPU the tiles are not tasks: the exact iteration set of the requested mode
// is described per dimension as a list of runs {first, count, stride} (one
// run per reference tile, merged when contiguous), and a single launch
// sweeps the cartesian product with consecutive lanes on consecutive
// indices. The common case — stride 1, contiguous coverage, 1-D — is the
// fast path: float4 grid-stride tiles with non-temporal stores (the HBM
// roofline kernel of BASELINE config 1).
#include <string.h>

#include <vector>

#include "../../include/hclib_forasync_sets.h"
#include "hx_module.h"

namespace hx {

// ------------------------------------------------------- triad fast path
// a[i] = b[i] + s*c[i], no contraction: __fmul_rn / __fadd_rn keep the
// product rounded before the add, bit-identical to the CPU reference loop.
__device__ __forceinline__ float triad1(float b, float c, float s) {
    return __fadd_rn(b, __fmul_rn(s, c));
}

constexpr int kTriadThreads = 256;
typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4f ld4(const v4f *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(v4f v, v4f *p) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// 16 B per lane; UNROLL independent (b, c) pairs per lane in flight;
// NTL / NTS select non-temporal loads / stores. CONTIG: each workgroup
// streams one contiguous slice (else grid-stride interleave).
template <bool NTL, bool NTS, int UNROLL, int THREADS, bool CONTIG>
__global__ __launch_bounds__(THREADS) void k_triad_f32(float *__restrict__ a,
                                                       const float *__restrict__ b,
                                                       const float *__restrict__ c, float s,
                                                       int64_t n4) {
    int64_t i, end, stride;
    if constexpr (CONTIG) {
        const int64_t q = (int64_t)THREADS * UNROLL;
        const int64_t span = ((n4 + gridDim.x - 1) / gridDim.x + q - 1) / q * q;
        i = (int64_t)blockIdx.x * span + threadIdx.x;
        end = (int64_t)blockIdx.x * span + span;
        if (end > n4) end = n4;
        stride = THREADS;
    } else {
        i = (int64_t)blockIdx.x * THREADS + threadIdx.x;
        end = n4;
        stride = (int64_t)gridDim.x * THREADS;
    }
    const v4f *b4 = reinterpret_cast<const v4f *>(b);
    const v4f *c4 = reinterpret_cast<const v4f *>(c);
    v4f *a4 = reinterpret_cast<v4f *>(a);
    for (; i + (UNROLL - 1) * stride < end; i += UNROLL * stride) {
        v4f vb[UNROLL], vc[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            vb[u] = ld4<NTL>(&b4[i + u * stride]);
            vc[u] = ld4<NTL>(&c4[i + u * stride]);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            v4f r;
            r.x = triad1(vb[u].x, vc[u].x, s);
            r.y = triad1(vb[u].y, vc[u].y, s);
            r.z = triad1(vb[u].z, vc[u].z, s);
            r.w = triad1(vb[u].w, vc[u].w, s);
            st4<NTS>(r, &a4[i + u * stride]);
        }
    }
    for (; i < end; i += stride) {
        v4f vb = ld4<NTL>(&b4[i]), vc = ld4<NTL>(&c4[i]), r;
        r.x = triad1(vb.x, vc.x, s);
        r.y = triad1(vb.y, vc.y, s);
        r.z = triad1(vb.z, vc.z, s);
        r.w = triad1(vb.w, vc.w, s);
        st4<NTS>(r, &a4[i]);
    }
}

// LDS-DMA form (MI355X_MICROARCH.md "ldsdma-fill": global_load_lds streams
// reach a higher chip rate than loads to VGPRs): every wave streams its own
// chunks of 64 float4 (1 KiB per array), DEPTH chunks of b and c in flight
// in a per-wave LDS ring; a chunk is computed from LDS once its two DMAs
// have landed (counted vmcnt) and a is stored non-temporally. AUX: the DMA's
// cache-policy bits (2 = nt).
template <int DEPTH, int AUX>
__global__ __launch_bounds__(256) void k_triad_lds(float *__restrict__ a, const float *__restrict__ b,
                                                   const float *__restrict__ c, float s, int64_t n4) {
    __shared__ v4f ring[4][DEPTH][2][64];  // [wave][slot][b|c][lane]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + wave, nw = (int64_t)gridDim.x * 4;
    const int64_t nchunks = n4 >> 6;  // whole 64-float4 chunks; the rest below
    const v4f *b4 = reinterpret_cast<const v4f *>(b);
    const v4f *c4 = reinterpret_cast<const v4f *>(c);
    v4f *a4 = reinterpret_cast<v4f *>(a);
    auto issue = [&](int64_t k, int slot) {
        const int64_t i = (k * nw + gw) * 64 + lane;
        __builtin_amdgcn_global_load_lds((const void *)&b4[i],
                                         (__attribute__((address_space(3))) void *)&ring[wave][slot][0][0], 16, 0, AUX);
        __builtin_amdgcn_global_load_lds((const void *)&c4[i],
                                         (__attribute__((address_space(3))) void *)&ring[wave][slot][1][0], 16, 0, AUX);
    };
    // chunks of this wave: k = 0, 1, ... with (k * nw + gw) < nchunks
    const int64_t mine = gw < nchunks ? (nchunks - gw + nw - 1) / nw : 0;
    int64_t k = 0;
    for (; k < DEPTH && k < mine; ++k) issue(k, (int)k);
    for (int64_t j = 0; j < mine; ++j) {
        const int slot = (int)(j % DEPTH);
        // chunk j's two DMAs are the oldest outstanding ops: younger are the
        // DMAs of up to DEPTH-1 later chunks and the stores of up to DEPTH-1
        // earlier ones (stores count in vmcnt on gfx9)
        // (in the first DEPTH iterations fewer stores are younger: at least
        // 2 (DEPTH - 1) ops are; near the end fewer refills: wait for all)
        if (mine - j < DEPTH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (j < DEPTH) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DEPTH - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (DEPTH - 1)) : "memory");
        const v4f vb = ring[wave][slot][0][lane], vc = ring[wave][slot][1][lane];
        v4f r;
        r.x = triad1(vb.x, vc.x, s);
        r.y = triad1(vb.y, vc.y, s);
        r.z = triad1(vb.z, vc.z, s);
        r.w = triad1(vb.w, vc.w, s);
        __builtin_nontemporal_store(r, &a4[(j * nw + gw) * 64 + lane]);
        // the slot is refilled only after this wave's reads of it returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (k < mine) {
            issue(k, slot);
            ++k;
        }
    }
    // the float4s past the last whole chunk
    for (int64_t i = nchunks * 64 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const v4f vb = b4[i], vc = c4[i];
        v4f r;
        r.x = triad1(vb.x, vc.x, s);
        r.y = triad1(vb.y, vc.y, s);
        r.z = triad1(vb.z, vc.z, s);
        r.w = triad1(vb.w, vc.w, s);
        a4[i] = r;
    }
}

typedef void (*triad_kernel_t)(float *, const float *, const float *, float, int64_t);

template <int THREADS, bool CONTIG>
static triad_kernel_t triad_pick(int v) {
    if (v & 64) return (v & 3) == 3 ? k_triad_f32<true, true, 2, THREADS, CONTIG>
                                    : k_triad_f32<false, true, 2, THREADS, CONTIG>;
    if (v & 128) return (v & 3) == 3 ? k_triad_f32<true, true, 1, THREADS, CONTIG>
                                     : k_triad_f32<false, true, 1, THREADS, CONTIG>;
    switch (v & 7) {
    case 0: return k_triad_f32<false, false, 4, THREADS, CONTIG>;
    case 1: return k_triad_f32<true, false, 4, THREADS, CONTIG>;
    case 2: return k_triad_f32<false, true, 4, THREADS, CONTIG>;
    case 3: return k_triad_f32<true, true, 4, THREADS, CONTIG>;
    case 4: return k_triad_f32<false, false, 8, THREADS, CONTIG>;
    case 5: return k_triad_f32<true, false, 8, THREADS, CONTIG>;
    case 6: return k_triad_f32<false, true, 8, THREADS, CONTIG>;
    default: return k_triad_f32<true, true, 8, THREADS, CONTIG>;
    }
}

// variant bits: 1 = nt loads, 2 = nt stores, 4 = unroll 8 (else 4),
// 8 = contiguous slice per workgroup, 16/32 = 512/1024 threads (else 256),
// 64 / 128 = unroll 2 / 1 (nt stores; nt loads when bits 0-1 are 3)
static triad_kernel_t triad_variant(int v, int *threads) {
    if (v & 256) {  // LDS-DMA: bits 0-1 = depth 2/4/8/16, bit 2 = nt DMA
        *threads = 256;
        const bool nt = (v & 4) != 0;
        switch (v & 3) {
        case 0: return nt ? k_triad_lds<2, 2> : k_triad_lds<2, 0>;
        case 1: return nt ? k_triad_lds<4, 2> : k_triad_lds<4, 0>;
        case 2: return nt ? k_triad_lds<8, 2> : k_triad_lds<8, 0>;
        default: return nt ? k_triad_lds<16, 2> : k_triad_lds<16, 0>;
        }
    }
    const bool contig = (v & 8) != 0;
    const int t = (v >> 4) & 3;
    *threads = t == 1 ? 512 : (t == 2 ? 1024 : 256);
    if (t == 1) return contig ? triad_pick<512, true>(v) : triad_pick<512, false>(v);
    if (t == 2) return contig ? triad_pick<1024, true>(v) : triad_pick<1024, false>(v);
    return contig ? triad_pick<256, true>(v) : triad_pick<256, false>(v);
}

__global__ void k_triad_tail(float *a, const float *b, const float *c, float s, int64_t from,
                             int64_t n) {
    int64_t i = from + threadIdx.x;
    if (i < n) a[i] = triad1(b[i], c[i], s);
}

// -------------------------------------------------------- generic sweep
using hclib_sets::Run;

struct DimRuns {
    const Run *runs;
    const int64_t *prefix;  // prefix[r] = iterations before run r; prefix[nruns] = total
    int nruns;
};

struct SweepArgs {
    DimRuns dim[3];
    int ndim;
    int64_t total;
    int body;
    hclib_hip_triad_args_t triad;
    hclib_hip_iota_args_t iota;
    hclib_hip_visit_args_t visit;
};

__device__ __forceinline__ int run_index(const DimRuns &d, int64_t t, int64_t &off) {
    int lo = 0, hi = d.nruns - 1;
    while (lo < hi) {  // last run with prefix <= t
        int mid = (lo + hi + 1) >> 1;
        if (d.prefix[mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    off = t - d.prefix[lo];
    return lo;
}

__device__ __forceinline__ int idx_of(const DimRuns &d, int64_t t) {
    int64_t off;
    const Run r = d.runs[run_index(d, t, off)];
    return r.first + (int)off * r.stride;
}

__global__ __launch_bounds__(256) void k_forasync_sweep(SweepArgs A) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int64_t n1 = A.ndim > 1 ? A.dim[1].prefix[A.dim[1].nruns] : 1;
    const int64_t n2 = A.ndim > 2 ? A.dim[2].prefix[A.dim[2].nruns] : 1;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < A.total; t += step) {
        // innermost dimension varies fastest -> consecutive lanes, consecutive indices
        int64_t t2 = t % n2, r = t / n2;
        int64_t t1 = r % n1, t0 = r / n1;
        const int i = idx_of(A.dim[0], t0);
        const int j = A.ndim > 1 ? idx_of(A.dim[1], t1) : 0;
        const int k = A.ndim > 2 ? idx_of(A.dim[2], t2) : 0;
        switch (A.body) {
        case HCLIB_HIP_BODY_TRIAD_F32:
            A.triad.a[i] = triad1(A.triad.b[i], A.triad.c[i], A.triad.s);
            break;
        case HCLIB_HIP_BODY_IOTA_CHECK:
            if (A.iota.ran[i] != -1) atomicAdd(A.iota.errors, 1);
            A.iota.ran[i] = i;
            break;
        case HCLIB_HIP_BODY_VISIT_COUNT: {
            const hclib_hip_visit_args_t &v = A.visit;
            const long li = (long)(i - v.base[0]), lj = (long)(j - v.base[1]),
                       lk = (long)(k - v.base[2]);
            if (li >= 0 && li < v.extent[0] && lj >= 0 && lj < v.extent[1] && lk >= 0 &&
                lk < v.extent[2])
                atomicAdd(&v.counts[(li * v.extent[1] + lj) * v.extent[2] + lk], 1);
            break;
        }
        default:
            break;
        }
    }
}

// -------------------------------------------------- host: iteration sets

// include/hclib_forasync_sets.h (shared with the C++ layers)
static std::vector<Run> dim_runs(const hclib_hip_loop_domain_t &d, int ndim, int mode) {
    const hclib_sets::Domain dd{d.low, d.high, d.stride, d.tile};
    return hclib_sets::runs(dd, ndim, mode == HCLIB_HIP_FORASYNC_RECURSIVE ? 1 : 0);
}

}  // namespace hx

using namespace hx;

extern "C" int hclib_hip_forasync_triad_f32(float *a, const float *b, const float *c, float s,
                                            int64_t n, void *stream) {
    if (!a || !b || !c || n < 0) {
        set_error("hclib_hip_forasync_triad_f32: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    hipStream_t st = (hipStream_t)stream;
    const bool aligned = (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) == 0;
    if (!aligned) {
        set_error("hclib_hip_forasync_triad_f32: arrays must be 16-byte aligned");
        return HCLIB_HIP_EINVAL;
    }
    const int64_t n4 = n / 4;
    if (n4 > 0) {
        // measured best on MI355X (scripts/probe_triad2.py, profiles/r02/triad_variants.log):
        // two 256-thread workgroups per CU, one (b, c) pair of non-temporal
        // 16-B loads per lane in flight (16 KiB of loads per CU) and
        // non-temporal stores: 6.22-6.26 TB/s, against 6.15-6.22 for one
        // workgroup with two pairs; the LDS-DMA form (variants 256-263) and
        // deeper pipelines measured no faster
        const int bpc = env_int("HCLIB_HIP_TRIAD_BLOCKS_PER_CU", 2);
        int threads = kTriadThreads;
        triad_kernel_t k = triad_variant(env_int("HCLIB_HIP_TRIAD_VARIANT", 131), &threads);
        int64_t grid = (int64_t)mod().num_cus * bpc;
        const int64_t need = (n4 + threads - 1) / threads;
        if (grid > need) grid = need;
        hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(threads), 0, st, a, b, c, s, n4);
        HX_HIP(hipGetLastError());
    }
    if (n4 * 4 < n) {
        hipLaunchKernelGGL(k_triad_tail, dim3(1), dim3(64), 0, st, a, b, c, s, n4 * 4, n);
        HX_HIP(hipGetLastError());
    }
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_forasync_plan(int dim, hclib_hip_loop_domain_t *domain, int mode, void *stream,
                                       hclib_hip_sweep_plan_t *plan) {
    static_assert(sizeof(hclib_hip_run_t) == sizeof(Run), "hclib_hip_run_t is hclib_sets::Run");
    if (!domain || !plan || dim < 1 || dim > 3 || (mode != 0 && mode != 1)) {
        set_error("hclib_hip_forasync_plan: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    memset(plan, 0, sizeof(*plan));
    HX_TRY(ensure_device());
    const int nworkers = hclib_hip_num_workers();
    for (int d = 0; d < dim; ++d) {
        if (domain[d].stride < 1) {
            set_error("hclib_hip_forasync_plan: stride must be >= 1");
            return HCLIB_HIP_EINVAL;
        }
        if (domain[d].tile == -1)  // src/hclib.c:455-461, written back
            domain[d].tile = ((domain[d].high - domain[d].low) + nworkers - 1) / nworkers;
        if (domain[d].tile < 1) domain[d].tile = 1;
    }
    std::vector<Run> runs[3];
    std::vector<int64_t> pre[3];
    size_t bytes = 0;
    plan->ndim = dim;
    plan->total = 1;
    for (int d = 0; d < dim; ++d) {
        runs[d] = dim_runs(domain[d], dim, mode);
        pre[d].resize(runs[d].size() + 1);
        pre[d][0] = 0;
        for (size_t r = 0; r < runs[d].size(); ++r) pre[d][r + 1] = pre[d][r] + runs[d][r].count;
        if (runs[d].empty()) runs[d].push_back(Run{0, 0, 1, 0});
        bytes += ((runs[d].size() * sizeof(Run) + 15) & ~(size_t)15) + ((pre[d].size() * 8 + 15) & ~(size_t)15);
        plan->total *= pre[d].back();
    }
    if (plan->total == 0) return HCLIB_HIP_OK;
    hipStream_t st = (hipStream_t)stream;
    char *dbuf = nullptr;
    HX_HIP(hipMallocAsync((void **)&dbuf, bytes, st));
    std::vector<char> hbuf(bytes);
    size_t off = 0;
    for (int d = 0; d < dim; ++d) {
        memcpy(&hbuf[off], runs[d].data(), runs[d].size() * sizeof(Run));
        plan->runs[d] = (const hclib_hip_run_t *)(dbuf + off);
        off += (runs[d].size() * sizeof(Run) + 15) & ~(size_t)15;
        memcpy(&hbuf[off], pre[d].data(), pre[d].size() * 8);
        plan->prefix[d] = (const int64_t *)(dbuf + off);
        off += (pre[d].size() * 8 + 15) & ~(size_t)15;
        plan->nruns[d] = (int)runs[d].size();
    }
    HX_TRY(upload_async(dbuf, hbuf.data(), bytes, st));
    plan->mem = dbuf;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_forasync_plan_release(hclib_hip_sweep_plan_t *plan, void *stream) {
    if (!plan) return HCLIB_HIP_EINVAL;
    if (plan->mem) HX_HIP(hipFreeAsync(plan->mem, (hipStream_t)stream));
    plan->mem = nullptr;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_forasync(int body, const void *args, int dim,
                                  hclib_hip_loop_domain_t *domain, int mode, void *stream) {
    if (!args || !domain || dim < 1 || dim > 3 || (mode != 0 && mode != 1) ||
        (body == HCLIB_HIP_BODY_TRIAD_F32 && dim != 1) ||
        (body == HCLIB_HIP_BODY_IOTA_CHECK && dim != 1) || body < 1 || body > 3) {
        set_error("hclib_hip_forasync: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    const int nworkers = hclib_hip_num_workers();
    for (int d = 0; d < dim; ++d) {
        if (domain[d].stride < 1) {
            set_error("hclib_hip_forasync: stride must be >= 1");
            return HCLIB_HIP_EINVAL;
        }
        if (domain[d].tile == -1)  // src/hclib.c:455-461, written back
            domain[d].tile = ((domain[d].high - domain[d].low) + nworkers - 1) / nworkers;
        if (domain[d].tile < 1) domain[d].tile = 1;
    }
    std::vector<Run> runs[3];
    for (int d = 0; d < dim; ++d) runs[d] = dim_runs(domain[d], dim, mode);
    // fast path: triad over one contiguous unit-stride run starting at 0
    if (body == HCLIB_HIP_BODY_TRIAD_F32 && runs[0].size() == 1 && runs[0][0].stride == 1 &&
        runs[0][0].first == 0) {
        const hclib_hip_triad_args_t *t = (const hclib_hip_triad_args_t *)args;
        return hclib_hip_forasync_triad_f32(t->a, t->b, t->c, t->s, runs[0][0].count, stream);
    }
    SweepArgs A;
    memset(&A, 0, sizeof(A));
    A.ndim = dim;
    A.body = body;
    if (body == HCLIB_HIP_BODY_TRIAD_F32) A.triad = *(const hclib_hip_triad_args_t *)args;
    if (body == HCLIB_HIP_BODY_IOTA_CHECK) A.iota = *(const hclib_hip_iota_args_t *)args;
    if (body == HCLIB_HIP_BODY_VISIT_COUNT) A.visit = *(const hclib_hip_visit_args_t *)args;
    // upload runs + prefixes in one buffer
    size_t bytes = 0;
    std::vector<int64_t> pre[3];
    A.total = 1;
    for (int d = 0; d < dim; ++d) {
        pre[d].resize(runs[d].size() + 1);
        pre[d][0] = 0;
        for (size_t r = 0; r < runs[d].size(); ++r) pre[d][r + 1] = pre[d][r] + runs[d][r].count;
        if (runs[d].empty()) runs[d].push_back(Run{0, 0, 1, 0});
        bytes += runs[d].size() * sizeof(Run) + pre[d].size() * 8 + 64;
        A.total *= pre[d].back();
    }
    if (A.total == 0) return HCLIB_HIP_OK;
    hipStream_t st = (hipStream_t)stream;
    // the run table is stream-ordered memory: allocated, uploaded, used and
    // freed in the launch's stream order, so the call never waits for the
    // sweep (a forasync inside a finish completes when the finish ends)
    char *dbuf = nullptr;
    HX_HIP(hipMallocAsync((void **)&dbuf, bytes, st));
    std::vector<char> hbuf(bytes);
    size_t off = 0;
    for (int d = 0; d < dim; ++d) {
        memcpy(&hbuf[off], runs[d].data(), runs[d].size() * sizeof(Run));
        A.dim[d].runs = (const Run *)(dbuf + off);
        off += (runs[d].size() * sizeof(Run) + 15) & ~(size_t)15;
        memcpy(&hbuf[off], pre[d].data(), pre[d].size() * 8);
        A.dim[d].prefix = (const int64_t *)(dbuf + off);
        off += (pre[d].size() * 8 + 15) & ~(size_t)15;
        A.dim[d].nruns = (int)runs[d].size();
    }
    HX_TRY(upload_async(dbuf, hbuf.data(), bytes, st));
    int64_t grid = (A.total + 255) / 256;
    const int64_t maxg = (int64_t)mod().num_cus * 16;
    if (grid > maxg) grid = maxg;
    hipLaunchKernelGGL(k_forasync_sweep, dim3((unsigned)grid), dim3(256), 0, st, A);
    HX_HIP(hipGetLastError());
    HX_HIP(hipFreeAsync(dbuf, st));
    return HCLIB_HIP_OK;
}
