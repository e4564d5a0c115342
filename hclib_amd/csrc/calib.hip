// calib.hip — L2 atomic-throughput calibration (the "peak" the scheduler's
// atomics are priced against; BASELINE north_star: "rocprof evidence of the
// fraction of peak L2 atomic throughput").
//
// The megakernel's cross-wave traffic is device-scope (agent) atomics that
// resolve in the per-XCD L2 (or past it, for lines another XCD touched).
// Three shapes, each the saturated form of one pattern the runtime uses:
//
//   SCATTER_RET64  every lane: returning 64-bit fetch-add on its own random
//                  16-B record of a 256 MiB table — fib's join check-out
//                  (fib.hip FibKind::check_out; src/hclib-runtime.c:431-446)
//                  and SW's dependency counters (src/hclib-promise.c:200-245).
//   HOT_WORD       lane 0 of every wave: returning 32-bit fetch-add on ONE
//                  shared word — the deque ticket / `outstanding` counter
//                  pattern (hx_sched.h enqueue_chunk/dequeue_chunk).
//   COALESCED32    every lane: non-returning 32-bit add, 64 consecutive
//                  dwords per wave instruction into a 64 MiB table — the
//                  L2 atomic ALU's streaming peak.
//
// Each mode is a plain kernel over a fixed number of operations; the rate is
// ops / kernel time (HIP events on the module stream).
#include "hx_module.h"
#include "uts_sha1.h"

namespace hx {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// kUnroll independent returning atomics in flight per lane
constexpr int kUnroll = 4;

__global__ __launch_bounds__(256) void k_atomic_scatter_ret64(unsigned long long *tab, uint32_t mask,
                                                              int iters, unsigned long long *sink) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; it += kUnroll) {
        unsigned long long r[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint32_t rec = mix32(tid * 0x9e3779b9u + (uint32_t)(it + u) * 0x85ebca6bu) & mask;
            r[u] = add_agent(&tab[(size_t)rec * 2], 1ull);  // 16-B records
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) acc += r[u];
    }
    if (acc == 0x5eed5eed5eedull) sink[0] = acc;  // keeps the returns live
}

__global__ __launch_bounds__(64) void k_atomic_hot_word(uint32_t *word, int iters, uint32_t *sink) {
    uint32_t acc = 0;
    if (threadIdx.x == 0)
        for (int it = 0; it < iters; ++it) acc += add_agent(word, 1u);
    if (acc == 0x5eed5eedu) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_atomic_coalesced32(uint32_t *tab, uint32_t mask_rows, int iters) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    for (int it = 0; it < iters; ++it) {
        const uint32_t row = mix32(wave * 0x9e3779b9u + (uint32_t)it) & mask_rows;
        __hip_atomic_fetch_add(&tab[(size_t)row * 64 + lane], 1u, __ATOMIC_RELAXED, HX_AGENT);
    }
}

// The UTS rng_spawn SHA-1 (uts_sha1.h, the instruction stream k_uts_search
// runs per node) back to back: every lane chains CH independent spawns
// (state_{k+1} = SHA1(state_k || k)) for `iters` steps, WPC waves per CU.
// The rate is the chip's SHA-1 issue ceiling: the "peak" of a kernel whose
// unavoidable per-node work is one such compression (k_uts_search on a
// throughput-bound tree; SURVEY §8d "Int VALU (SHA-1)").
template <int CH>
__global__ __launch_bounds__(64) void k_sha1_chain(const uint32_t *seed, int iters, uint32_t *sink) {
    const uint32_t gid = blockIdx.x * 64 + threadIdx.x;
    uint32_t s[CH][5], o[CH][5];
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int k = 0; k < 5; ++k) s[j][k] = seed[(gid * 5 + k) & 1023] ^ (0x9e3779b9u * (uint32_t)(j + 1));
    for (int it = 0; it < iters; ++it) {
        const uint32_t *pp[CH];
        uint32_t ii[CH];
        uint32_t *oo[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            pp[j] = s[j];
            ii[j] = (uint32_t)it;
            oo[j] = o[j];
        }
        rng_spawn_n<CH>(pp, ii, oo);
#pragma unroll
        for (int j = 0; j < CH; ++j)
#pragma unroll
            for (int k = 0; k < 5; ++k) s[j][k] = o[j][k];
    }
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int k = 0; k < 5; ++k) x ^= s[j][k];
    if (x == 0x5eed5eedu) sink[0] = x;  // keeps the chains live
}

}  // namespace hx

using namespace hx;

extern "C" int hclib_hip_sha1_calibrate(int chains, int waves_per_cu, int iters, double *sha1_per_s,
                                        double *kernel_ms) {
    if (chains < 1 || chains > 2 || waves_per_cu < 1 || waves_per_cu > 16 || iters < 1 || iters > (1 << 16) ||
        !sha1_per_s) {
        set_error("hclib_hip_sha1_calibrate: chains 1..2, waves_per_cu 1..16, iters in [1, 2^16]");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = mod();
    void *d = nullptr;
    HX_HIP(hipMalloc(&d, 4096 + 256));
    uint32_t *seed = (uint32_t *)d, *sink = (uint32_t *)((char *)d + 4096);
    int rc = hip_check(hipMemsetAsync(d, 0x5a, 4096 + 256, m.stream), "memset");
    const int blocks = m.num_cus * waves_per_cu;
    for (int rep = 0; rep < 2 && rc == HCLIB_HIP_OK; ++rep) {  // warm-up, then the timed launch
        if (rep == 1) rc = hip_check(hipEventRecord(m.ev0, m.stream), "event");
        if (chains == 1) hipLaunchKernelGGL(k_sha1_chain<1>, dim3(blocks), dim3(64), 0, m.stream, seed, iters, sink);
        else hipLaunchKernelGGL(k_sha1_chain<2>, dim3(blocks), dim3(64), 0, m.stream, seed, iters, sink);
        if (rc == HCLIB_HIP_OK) rc = hip_check(hipGetLastError(), "sha1 calibration launch");
    }
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipEventRecord(m.ev1, m.stream), "event");
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipStreamSynchronize(m.stream), "sync");
    float ms = 0;
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipEventElapsedTime(&ms, m.ev0, m.ev1), "elapsed");
    (void)hipFree(d);
    if (rc != HCLIB_HIP_OK) return rc;
    *sha1_per_s = ms > 0 ? (double)blocks * 64.0 * chains * iters / (ms * 1e-3) : 0.0;
    if (kernel_ms) *kernel_ms = ms;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_atomic_calibrate(int mode, int iters, double *mops_per_s, double *kernel_ms) {
    if (mode < 0 || mode > 2 || iters < kUnroll || iters > (1 << 20) || !mops_per_s) {
        set_error("hclib_hip_atomic_calibrate: mode 0..2, iters in [%d, 2^20]", kUnroll);
        return HCLIB_HIP_EINVAL;
    }
    iters = iters / kUnroll * kUnroll;
    HX_TRY(ensure_device());
    Module &m = mod();
    const size_t table = 256ull << 20;  // 16-B records spread past the Infinity Cache's reach
    void *d = nullptr;
    HX_HIP(hipMalloc(&d, table + 256));
    unsigned long long *sink = (unsigned long long *)((char *)d + table);
    int rc = hip_check(hipMemsetAsync(d, 0, table + 256, m.stream), "memset");
    double ops = 0;
    // warm-up launch (page tables, clocks), then the timed one
    for (int rep = 0; rep < 2 && rc == HCLIB_HIP_OK; ++rep) {
        if (rep == 1) rc = hip_check(hipEventRecord(m.ev0, m.stream), "event");
        const int blocks = m.num_cus * 8;
        if (mode == 0) {  // 32 waves per CU, every lane its own record
            hipLaunchKernelGGL(k_atomic_scatter_ret64, dim3(blocks), dim3(256), 0, m.stream,
                               (unsigned long long *)d, (uint32_t)(table / 16 - 1), iters, sink);
            ops = (double)blocks * 256 * iters;
        } else if (mode == 1) {  // 8 waves per CU on one word
            hipLaunchKernelGGL(k_atomic_hot_word, dim3(blocks), dim3(64), 0, m.stream, (uint32_t *)d, iters,
                               (uint32_t *)sink);
            ops = (double)blocks * iters;
        } else {  // 32 waves per CU, 256-B rows of a 64 MiB table
            hipLaunchKernelGGL(k_atomic_coalesced32, dim3(blocks), dim3(256), 0, m.stream, (uint32_t *)d,
                               (uint32_t)((64ull << 20) / 256 - 1), iters);
            ops = (double)blocks * 256 * iters;
        }
        if (rc == HCLIB_HIP_OK) rc = hip_check(hipGetLastError(), "atomic calibration launch");
    }
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipEventRecord(m.ev1, m.stream), "event");
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipStreamSynchronize(m.stream), "sync");
    float ms = 0;
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipEventElapsedTime(&ms, m.ev0, m.ev1), "elapsed");
    (void)hipFree(d);
    if (rc != HCLIB_HIP_OK) return rc;
    *mops_per_s = ms > 0 ? ops / (ms * 1e3) : 0.0;
    if (kernel_ms) *kernel_ms = ms;
    return HCLIB_HIP_OK;
}
