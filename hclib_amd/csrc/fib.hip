// fib.hip — the fib workload (test/fib/fib.c) as a device task kind.
//
// Each fib(n) call is one task (one lane-item), exactly as each
// hclib_async(fib, ...) is one task in the reference (fib.c:57-71). A task
// with n >= 2 opens a finish scope for its two child asyncs (the reference's
// finish counter is the owner's 1 + the two check-ins, src/hclib-runtime.c:
// 1219-1247, 431-446) with the generic device finish of hx_finish.h: the
// children add their result and check out with ONE 64-bit atomic, and the
// child that closes the scope runs the continuation (res = lhs + rhs,
// fib.c:70: the scope's sum) inline and checks out of the parent scope —
// the GPU analogue of help_finish's work-shift (no stacks, no fibers). This
// also is the DDT form (fib.c:113-141): the scope word is the promise pair
// subres[0..1] and the last put releases fib_ddt_res.
#include <stdio.h>
#include <string.h>

#include "hx_module.h"
#include "../../include/hclib_hip/hx_finish.h"

namespace hx {

struct FibCtx {
    int n;
    int local;  // scopes in the wave's LDS while they stay inside it (hx_finish.h LocalScopes)
    int blocks; // HBM scope ids taken kScopeBlock at a time per wave
    FinishArena fin;
};

// the wave's LDS finish scopes (file scope: every access is a ds_* op)
constexpr int kFibLocalScopes = 512;
__shared__ LocalScopes<kFibLocalScopes> s_fib_scopes;
// the wave's block of HBM scope ids (hx_finish.h finish_open `blk`)
__shared__ uint32_t s_fib_blk[2];

struct FibKind {
    // template = {n + 1 of the parent call, the parent's scope}; child k is
    // fib(n - 1 - k) of that call
    static constexpr int kTmplWords = 2;
    static constexpr int kWords = 4;
    static constexpr bool kPure = false;           // scopes are opened / checked out in HBM
    static constexpr bool kBoundedChildren = true;  // 0 or 2
    using Ctx = FibCtx;
    struct Acc {
        unsigned long long tasks = 0, joins = 0;
        // the wave's totals go into its exit record (hx_sched.h Kind concept)
        __device__ void totals(unsigned long long (&c)[8], unsigned long long (&)[4]) {
            c[0] = wave_sum(tasks);
            c[1] = wave_sum(joins);
        }
    };

    __device__ static int roots(const Ctx &c, Acc &, uint32_t *tmpl) {
        tmpl[0] = (uint32_t)c.n + 1;  // child 0 of {n+1, root} is fib(n)
        tmpl[1] = kScopeRoot;
        return 1;
    }

    __device__ static int process(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k,
                                  uint32_t *child, uint32_t *err, bool) {
        acc.tasks += 1;
        const int n = (int)t[0] - 1 - (int)k;
        const bool spawn = n >= 2;
        // FINISH { async fib(n-1); async fib(n-2); }  (one bump allocation
        // per wave for every lane that opens a scope)
        const uint32_t j = c.local ? finish_open_local(c.fin, s_fib_scopes, spawn, t[1], 2, 0, err,
                                                       c.blocks ? s_fib_blk : nullptr)
                                   : finish_open(c.fin, spawn, t[1], 2, 0, err, c.blocks ? s_fib_blk : nullptr);
        if (!spawn) {  // a leaf returns n: check out, continuations inline
            acc.joins += c.local ? finish_check_out_local(c.fin, s_fib_scopes, t[1], (unsigned long long)n, PassSum())
                                 : finish_check_out(c.fin, t[1], (unsigned long long)n, PassSum());
            return 0;
        }
        if (j == kScopeRoot) return 0;  // arena error (reported)
        child[0] = (uint32_t)n;  // children fib(n-1), fib(n-2)
        child[1] = j;
        return 2;
    }

    // an item leaving the wave names an HBM scope (its LDS scope promoted)
    __device__ static void export_item(const Ctx &c, uint32_t *w, bool valid, uint32_t *err) {
        if (!c.local) return;
        const uint32_t s = finish_promote(c.fin, s_fib_scopes, valid ? w[1] : kScopeRoot, err);
        if (valid) w[1] = s;
    }
};

constexpr int kFibCap = 1024;  // ring items per wave (16 KiB of LDS)

__global__ __launch_bounds__(64) void k_fib(FibCtx ctx, PoolView pool, SchedGlobals *g,
                                            SchedConfig cfg) {
    __shared__ WaveStack<FibKind, kFibCap> st;
    if (ctx.local) s_fib_scopes.init();
    if (threadIdx.x < 2) s_fib_blk[threadIdx.x] = 0;
    __syncthreads();
    run_worker<FibKind, kFibCap>(ctx, pool, g, cfg, st, blockIdx.x == 0);
}

}  // namespace hx

using namespace hx;

extern "C" int hclib_hip_fib(int n, int64_t *value, hclib_hip_fib_result_t *result) {
    if (n < 0 || n > 80 || !value) {
        set_error("hclib_hip_fib: n must be in [0, 80]");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = mod();
    // scopes = internal nodes of the call tree = fib(n+1) - 1
    unsigned long long a = 0, b = 1;
    for (int i = 0; i <= n; ++i) {
        unsigned long long t = a + b;
        a = b;
        b = t;
    }
    const unsigned long long scopes = a;  // fib(n+1)
    if (scopes > 0xfffffff0ull) {
        set_error("hclib_hip_fib: n too large for the join arena");
        return HCLIB_HIP_EINVAL;
    }
    const int grid = env_int("HCLIB_HIP_GRID", 0) > 0 ? env_int("HCLIB_HIP_GRID", 0)
                                                    : m.num_cus * env_int("HCLIB_HIP_WAVES_PER_CU", 2);
    const int blocks = env_int("HCLIB_HIP_FIB_BLOCKS", 1);
    // the arena: every scope once, plus each wave's last partly used id block
    const unsigned long long ids = scopes + 1 + (blocks ? (unsigned long long)grid * kScopeBlock : 0ull);
    if (ids > 0xfffffff0ull) {
        set_error("hclib_hip_fib: n too large for the join arena");
        return HCLIB_HIP_EINVAL;
    }
    const size_t jb = sizeof(FinishScope) * (size_t)ids;
    void *dmem = nullptr;
    HX_HIP(hipMalloc(&dmem, jb + 512));
    FibCtx ctx;
    ctx.n = n;
    ctx.local = env_int("HCLIB_HIP_FIB_LOCAL", 0);  // LDS scopes: measured slower so far (profiles/r04/fib_stamps.log)
    ctx.fin.scopes = (FinishScope *)dmem;
    ctx.fin.next = (uint32_t *)((char *)dmem + ((jb + 255) & ~(size_t)255));
    ctx.fin.cap = (uint32_t)ids;
    ctx.blocks = blocks;
    ctx.fin.root_value = (unsigned long long *)(ctx.fin.next + 16);
    HX_HIP(hipMemsetAsync(ctx.fin.next, 0, 256, m.stream));
    PoolView pool;
    HX_TRY(make_pool((uint32_t)env_int("HCLIB_HIP_DEQUES", 64),
                     (uint32_t)env_int("HCLIB_HIP_DEQUE_CAP", 4096),
                     // 32-item chunks at 2 waves per CU: fib(30) 1.47 -> 0.92 ms
                     // (profiles/r02/fib_knobs.log; 8-item chunks made the 2,048
                     // idle-polling waves of the old default fight over crumbs)
                     (uint32_t)env_int("HCLIB_HIP_FIB_CHUNK", 32), FibKind::kWords, &pool));
    SchedConfig cfg;
    cfg.spill_hi = (uint32_t)env_int("HCLIB_HIP_FIB_SPILL_HI", 256);
    // scripts/sweep_uts.py fib30 (profiles/r01_s5/knob_sweeps.log): 32 -> 1.50 ms, 2 -> 1.70 ms
    cfg.spill_lo = (uint32_t)env_int("HCLIB_HIP_FIB_SPILL_LO", 32);
    cfg.spin_limit = (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    cfg.nwaves = (uint32_t)grid;
    cfg.stamps = (uint32_t)env_int("HCLIB_HIP_STAMPS", 0);
    cfg.hunger = (uint32_t)env_int("HCLIB_HIP_FIB_HUNGER", 8);
    cfg.carry = (uint32_t)env_int("HCLIB_HIP_CARRY", 1);
    HX_TRY(reset_sched(pool, 1, false, (uint32_t)grid));
    HX_HIP(hipEventRecord(m.ev0, m.stream));
    hipLaunchKernelGGL(k_fib, dim3(grid), dim3(64), 0, m.stream, ctx, pool, m.globals, cfg);
    HX_HIP(hipGetLastError());
    HX_HIP(hipEventRecord(m.ev1, m.stream));
    SchedGlobals gl;
    int rc = finish_sched(&gl, "hclib_hip_fib");
    unsigned long long v = 0;
    if (rc == HCLIB_HIP_OK) rc = hip_check(hipMemcpy(&v, ctx.fin.root_value, 8, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == HCLIB_HIP_OK && env_int("HCLIB_HIP_FIB_DEBUG", 0)) {
        uint32_t used = 0;  // scopes that lived in HBM (opened there or promoted from LDS)
        if (hipMemcpy(&used, ctx.fin.next, 4, hipMemcpyDeviceToHost) == hipSuccess)
            fprintf(stderr, "fib(%d): %u of %llu scopes in HBM (local %d)\n", n, used, scopes - 1, ctx.local);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, m.ev0, m.ev1);
    (void)hipFree(dmem);
    if (rc != HCLIB_HIP_OK) return rc;
    *value = (int64_t)v;
    if (result) {
        result->tasks = gl.counters[0];
        result->joins = gl.counters[1];
        result->chunks_pushed = gl.counters[kCtrPushed];
        result->chunks_stolen = gl.counters[kCtrStolen];
        result->kernel_ms = ms;
        const double busy = (double)gl.counters[kCtrBusyCycles],
                     idle = (double)gl.counters[kCtrIdleCycles];
        result->busy_frac = (busy + idle) > 0 ? busy / (busy + idle) : 0.0;
    }
    return HCLIB_HIP_OK;
}
