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
    int local;  // scopes in the wave's LDS while they stay inside it (hx_finish.h LocalScopes);
                // their HBM check-out steps are issued in one batch and resolved in the next
                // (finish_issue / finish_resolve)
    int blocks; // HBM scope ids taken kScopeBlock at a time per wave
    uint32_t *seed;     // breadth-first seeding (HCLIB_HIP_FIB_SEED): [0] ready flag, [1] items, [64..] items; or null
    int seed_per_wave;  // ... items per worker it aims at
    FinishArena fin;
};

// the wave's LDS finish scopes (file scope: every access is a ds_* op)
// (smaller rings and scope sets at more waves per CU measured slower:
// 0.83-1.1 vs 0.74 ms, profiles/r04/fibsmall_sweep.log)
constexpr int kFibLocalScopes = 512;
__shared__ LocalScopes<kFibLocalScopes> s_fib_scopes;
// the wave's block of HBM scope ids (hx_finish.h finish_open `blk`)
__shared__ uint32_t s_fib_blk[2];
// items a seeding level may hold (worker 0 expands the levels in its own,
// still empty, ring arrays: d[] and t1[], one {n, parent scope} per slot)
constexpr uint32_t kFibSeedCap = 1024;

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
        FinishInFlight q;  // this lane's HBM check-out step in flight (LDS mode)
        // HX_STAMPS builds: cycles in process's phases (resolve, open, check-out), first active lane only
        unsigned long long cyc[3] = {0, 0, 0};
        // the wave's totals go into its exit record (hx_sched.h Kind concept)
        __device__ void totals(unsigned long long (&c)[8], unsigned long long (&)[4]) {
            c[0] = wave_sum(tasks);
            c[1] = wave_sum(joins);
#if defined(HX_STAMPS) && HX_STAMPS
            c[2] = wave_sum(cyc[1]);  // check-out cycles
            c[3] = wave_sum(cyc[2]);  // lock-step climb iterations  (the scheduler keeps c[4..7])
#endif
        }
    };

    __device__ static int roots(const Ctx &c, Acc &, uint32_t *tmpl) {
        tmpl[0] = (uint32_t)c.n + 1;  // child 0 of {n+1, root} is fib(n)
        tmpl[1] = kScopeRoot;
        return 1;
    }

    __device__ static int process(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k,
                                  uint32_t *child, uint32_t *err, bool) {
#if defined(HX_STAMPS) && HX_STAMPS
        const bool lead = lane_id() == __builtin_ctzll(__ballot(1));
        auto stamp = [&](int i, unsigned long long &ts) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            if (lead && i >= 0) acc.cyc[i] += now - ts;
            ts = now;
        };
#else
        auto stamp = [](int, unsigned long long &) {};
#endif
        unsigned long long tst = 0;
        stamp(-1, tst);
        // the HBM check-out this lane issued a batch ago: its result is in
        if (c.local) acc.joins += finish_resolve(c.fin, acc.q, PassSum());
        stamp(0, tst);
        const int n = (int)t[0] - 1 - (int)k;
        const bool spawn = n >= 2;
        acc.tasks += 1;
        // FINISH { async fib(n-1); async fib(n-2); }  (one bump allocation
        // per wave for every lane that opens a scope)
        const uint32_t j = c.local ? finish_open_local(c.fin, s_fib_scopes, spawn, t[1], 2, 0, err,
                                                       c.blocks ? s_fib_blk : nullptr)
                                   : finish_open(c.fin, spawn, t[1], 2, 0, err, c.blocks ? s_fib_blk : nullptr);
        stamp(1, tst);
        if (spawn) {
            if (j == kScopeRoot) return 0;  // arena error (reported)
            child[0] = (uint32_t)n;  // children fib(n-1), fib(n-2)
            child[1] = j;
            return 2;
        }
        // a leaf returns n: it checks out, and the last task out of each scope
        // runs its continuation inline, up the chain (an unbounded climb:
        // round 4 measured bounded climbs and one level per continuation item
        // no faster)
        stamp(-1, tst);
#if defined(HX_STAMPS) && HX_STAMPS
        uint32_t steps = 0;
        uint32_t *stp = lead ? &steps : nullptr;
#else
        uint32_t *stp = nullptr;
#endif
        acc.joins += c.local ? finish_check_out_local(c.fin, s_fib_scopes, t[1], (unsigned long long)n, PassSum(),
                                                      &acc.q, stp)
                             : finish_check_out(c.fin, t[1], (unsigned long long)n, PassSum());
        stamp(1, tst);
#if defined(HX_STAMPS) && HX_STAMPS
        acc.cyc[2] += steps;  // (c[3]: lock-step iterations, first active lane)
#endif
        return 0;
    }

    // Breadth-first seeding: worker 0 runs the call tree's top levels (each
    // internal call opens an HBM scope, the calls below it are the next
    // level) until the next level would pass workers x seed_per_wave items,
    // publishes the last level, and every worker takes an equal share as
    // its first ring items — all waves busy from the start instead of
    // waiting for the work to spread from one root.
    __device__ static bool seeding(const Ctx &c) { return c.seed != nullptr; }
    template <class WS>
    __device__ static uint32_t seed(const Ctx &c, Acc &acc, WS &st, uint32_t gid, uint32_t nwaves, uint32_t spin_ms,
                                    uint32_t *err) {
        const uint32_t lane = (uint32_t)lane_id();
        uint32_t *flag = c.seed, *items = c.seed + 64;
        if (gid == 0) {
            static_assert(sizeof(st.d) / sizeof(st.d[0]) >= kFibSeedCap && sizeof(st.t1) / sizeof(st.t1[0]) >= kFibSeedCap,
                          "the seeding levels live in the ring arrays");
            unsigned long long tgt = (unsigned long long)nwaves * (unsigned long long)c.seed_per_wave;
            const uint32_t target = tgt > kFibSeedCap ? kFibSeedCap : (uint32_t)tgt;
            uint32_t *cur = (uint32_t *)st.d, *nxt = (uint32_t *)st.t1;
            if (lane == 0) {
                cur[0] = (uint32_t)c.n;
                cur[1] = kScopeRoot;
            }
            // every scope the seeding can open (< target: a binary tree of
            // fewer than `target` leaves), taken with one atomic
            uint32_t base = 0, used = 0;
            if (lane == 0) base = add_agent(c.fin.next, target);
            base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
            const bool ids_ok = base + target <= c.fin.cap;
            if (!ids_ok && lane == 0) dev_error(err, kErrArena);
            uint32_t cnt = 1;
            while (cnt > 0 && 2 * cnt <= target) {
                uint32_t ncnt = 0;
                for (uint32_t b = 0; b < cnt; b += 64) {
                    const uint32_t i = b + lane;
                    const bool has = i < cnt;
                    const uint32_t m = has ? cur[2 * i] : 0u, p = has ? cur[2 * i + 1] : kScopeRoot;
                    const bool open = has && m >= 2 && ids_ok;
                    const unsigned long long om = __ballot(open);
                    const uint32_t rk = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(om >> 32),
                                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)om, 0u));
                    const uint32_t S = base + used + rk;
                    used += (uint32_t)__popcll(om);
                    if (open) {  // (as finish_open: count 2, no continuation)
                        FinishScope *f = &c.fin.scopes[S];
                        st_agent(&f->word, 2ull << 56);
                        st_agent(&f->parent, p);
                        st_agent(&f->cont, 0u);
                    }
                    if (open) {
                        const uint32_t o = ncnt + 2 * rk;
                        nxt[2 * o] = m - 1;
                        nxt[2 * o + 1] = S;
                        nxt[2 * o + 2] = m - 2;
                        nxt[2 * o + 3] = S;
                    }
                    if (has) acc.tasks += 1;
                    if (has && !open) acc.joins += finish_check_out(c.fin, p, (unsigned long long)m, PassSum());
                    ncnt += 2u * (uint32_t)__popcll(om);
                }
                uint32_t *t = cur;
                cur = nxt;
                nxt = t;
                cnt = ncnt;
            }
            for (uint32_t i = lane; i < cnt; i += 64) {
                st_agent(&items[2 * i], cur[2 * i]);
                st_agent(&items[2 * i + 1], cur[2 * i + 1]);
            }
            if (lane == 0) st_agent(&flag[1], cnt);
            release_agent();
            if (lane == 0) st_agent(&flag[0], 1u);
        }
        uint32_t ready = 0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (true) {
            if (lane == 0) ready = ld_agent(&flag[0]);
            ready = (uint32_t)__builtin_amdgcn_readfirstlane((int)ready);
            if (ready) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * spin_ms) {
                if (lane == 0) dev_error(err, kErrSpinTimeout);
                return 0;
            }
            __builtin_amdgcn_s_sleep(4);
        }
        acquire_agent();
        const uint32_t cnt = (uint32_t)__builtin_amdgcn_readfirstlane((int)ld_agent(&flag[1]));
        const uint32_t lo = (uint32_t)(((unsigned long long)cnt * gid) / nwaves),
                       hi = (uint32_t)(((unsigned long long)cnt * (gid + 1)) / nwaves);
        for (uint32_t j = lane; j < hi - lo; j += 64) {
            const uint32_t tm[2] = {ld_agent(&items[2 * (lo + j)]) + 1u, ld_agent(&items[2 * (lo + j) + 1])};
            store_tmpl(st, j, tm);  // template {n + 1, scope}: child 0 is the call fib(n)
            st.d[j] = make_uint2(0u, 1u);
        }
        return hi - lo;
    }

    // the ring ran empty: the check-outs still in flight, to their ends
    __device__ static void drain(const Ctx &c, Acc &acc, uint32_t *) {
        if (c.local) acc.joins += finish_drain(c.fin, acc.q, PassSum());
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
    // 3 waves per CU with seeding (fib(30) 0.65 -> 0.48-0.49 ms against 2,
    // profiles/r04/fibseed2_sweep.log)
    const int grid = env_int("HCLIB_HIP_GRID", 0) > 0 ? env_int("HCLIB_HIP_GRID", 0)
                                                    : m.num_cus * env_int("HCLIB_HIP_WAVES_PER_CU", 3);
    const int blocks = env_int("HCLIB_HIP_FIB_BLOCKS", 1);
    // the arena: every scope once, plus each wave's last partly used id block,
    // plus the seeding's reservation (worker 0 takes up to kFibSeedCap ids in
    // one atomic and opens only as many as its levels need)
    const int seed_pw = env_int("HCLIB_HIP_FIB_SEED", 2);
    const unsigned long long ids = scopes + 1 + (blocks ? (unsigned long long)grid * kScopeBlock : 0ull) +
                                   (seed_pw > 0 ? (unsigned long long)kFibSeedCap : 0ull);
    if (ids > 0xfffffff0ull) {
        set_error("hclib_hip_fib: n too large for the join arena");
        return HCLIB_HIP_EINVAL;
    }
    const size_t jb = sizeof(FinishScope) * (size_t)ids;
    // seeding buffer behind the arena's counters: [0] flag, [1] count, [64..] items
    // (2 items per worker, at most kFibSeedCap: fib(30) 0.70-0.74 -> 0.47-0.49 ms,
    // profiles/r04/fibseed_sweep.log, fibseed2_sweep.log; 0: from one root)
    const size_t sb = seed_pw > 0 ? (64 + 2 * (size_t)kFibSeedCap) * 4 : 0;
    void *dmem = nullptr;
    HX_HIP(hipMalloc(&dmem, jb + 512 + sb));
    FibCtx ctx;
    ctx.n = n;
    // LDS scopes (hx_finish.h LocalScopes, batched promotion): fib(30)
    // 0.807 -> 0.688 ms (profiles/r04/fiblds_sweep.log)
    ctx.local = env_int("HCLIB_HIP_FIB_LOCAL", 1);
    ctx.fin.scopes = (FinishScope *)dmem;
    ctx.fin.next = (uint32_t *)((char *)dmem + ((jb + 255) & ~(size_t)255));
    ctx.fin.cap = (uint32_t)ids;
    ctx.blocks = blocks;
    ctx.fin.root_value = (unsigned long long *)(ctx.fin.next + 16);
    HX_HIP(hipMemsetAsync(ctx.fin.next, 0, 256, m.stream));
    ctx.seed = nullptr;
    ctx.seed_per_wave = seed_pw;
    if (seed_pw > 0) {
        ctx.seed = (uint32_t *)((char *)dmem + ((jb + 255) & ~(size_t)255) + 256);
        HX_HIP(hipMemsetAsync(ctx.seed, 0, 256, m.stream));
    }
    PoolView pool;
    HX_TRY(make_pool((uint32_t)env_int("HCLIB_HIP_DEQUES", 64),
                     (uint32_t)env_int("HCLIB_HIP_DEQUE_CAP", 4096),
                     // 32-item chunks at 2 waves per CU: fib(30) 1.47 -> 0.92 ms
                     // (profiles/r02/fib_knobs.log; 8-item chunks made the 2,048
                     // idle-polling waves of the old default fight over crumbs)
                     (uint32_t)env_int("HCLIB_HIP_FIB_CHUNK", 32), FibKind::kWords, &pool));
    SchedConfig cfg;
    // seeded launches: 320 / 64 (fib(30) 0.49 -> 0.45 ms against 256 / 32,
    // profiles/r04/fibknobs_f.log, fibknobs_g.log)
    cfg.spill_hi = (uint32_t)env_int("HCLIB_HIP_FIB_SPILL_HI", seed_pw > 0 ? 320 : 256);
    // scripts/sweep_uts.py fib30 (profiles/r01_s5/knob_sweeps.log): 32 -> 1.50 ms, 2 -> 1.70 ms
    cfg.spill_lo = (uint32_t)env_int("HCLIB_HIP_FIB_SPILL_LO", seed_pw > 0 ? 64 : 32);
    // seeded fib: its first batches see every wave busy, as the host set it
    // (fib(30) 0.40 -> 0.39 ms, profiles/r06/ab_outstpf.log)
    cfg.hunger_init_full = 1;
    cfg.spin_limit = (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    cfg.nwaves = (uint32_t)grid;
    cfg.stamps = (uint32_t)env_int("HCLIB_HIP_STAMPS", 0);
    cfg.hunger = (uint32_t)env_int("HCLIB_HIP_FIB_HUNGER", 8);
    cfg.carry = (uint32_t)env_int("HCLIB_HIP_CARRY", 1);
    // seeded: every wave starts holding its share (outstanding = every wave)
    HX_TRY(reset_sched(pool, ctx.seed ? (uint32_t)grid : 1u, false, (uint32_t)grid));
    HX_HIP(hipEventRecord(m.ev0, m.stream));
    if (int rc0 = check_resident((const void *)k_fib, grid, 64, 0, "hclib_hip_fib")) {
        (void)hipFree(dmem);
        return rc0;
    }
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
