// uts.hip — UTS tree search as a device task kind of the megakernel.
//
// One lane-item = one rng_spawn (test/uts/rng/brg_sha1.c:68-83): the child
// state is a single SHA-1 block compression of parent[20] || i, computed in
// registers. A task entry is a non-leaf node with children left to spawn
// (leaves are counted and never stored). numChildren (test/uts/uts.c:225-274)
// runs on integer threshold tables that the host derives from the
// reference's own libm formula (uts.c:171-222), so the device needs no libm
// and stays bit-exact: n = #{k in 1..100 : thr[depth][k] <= rand}.
// Counting follows UTS.cpp: a node counts when it is generated (each node is
// popped exactly once in the reference), leaves when numChildren <= 0,
// depth = max height.
#include <math.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "hx_module.h"
#include "uts_sha1.h"

namespace hx {

// ------------------------------------------------------------- SHA-1
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

// rng_spawn (the device SHA-1, one and several interleaved chains): uts_sha1.h

// --------------------------------------------------------- depth rules
// rule.x: 0 = constant rule.y children; 1 = BIN: rand < rule.y ? m : 0;
//         2 = GEO: threshold table rule.z (128 words, entries 1..100)
struct UtsCtx {
    uint32_t root[5];
    int root_nc;
    int nrules;
    int stationary;
    int gran;
    int m;
    int shard, nshards, split;
    int hist_levels;
    int lds_tables;  // rules/thr fit the per-wave LDS cache
    uint32_t bin_thr;  // BIN trees: a node has m children iff rand < bin_thr (every depth >= 1)
    int nthr;        // words in thr
    int geo_depth;   // kUtsGeoFixed: depths 1..geo_depth-1 use table 0, deeper nodes are leaves
    // kUtsGeoFixed: table 0's bucket bytes (kUtsBuckets, see uts_nc): per
    // 2^21-wide bucket of rand, the thresholds at or below its start (| 0x80
    // when more than two thresholds fall inside it)
    const uint32_t *nb;
    const int4 *rules;
    const uint32_t *thr;
    unsigned long long *hist;
    const uint32_t *chain;  // FEAT 3 (diagnostic): chain[d] = child index of the traced chain's depth-d node
};

constexpr size_t kUtsLdsRules = 64;     // depth rules cached in LDS per wave
constexpr size_t kUtsLdsThr = 4 * 128;  // up to 4 GEO threshold tables
// kUtsGeoFixed: 1024 buckets of rand (2^21 wide), one byte each, kept in
// s_thr words 128..383 (a fixed-shape tree has one table: the rest is free)
constexpr int kUtsBuckets = 1024, kUtsBucketShift = 21;

// LDS copies of the rule tables (file scope, so every access is a ds_read:
// a generic pointer to them would compile to flat loads whose waits also
// drain the in-flight global loads).
__shared__ int4 s_rules[kUtsLdsRules];
__shared__ uint32_t s_thr[kUtsLdsThr];

// numChildren lookup modes (the kernel is instantiated per mode)
enum UtsMode : int {
    kUtsRulesGlobal = 0,  // depth rules in device memory (large tables)
    kUtsRulesLds = 1,     // depth rules cached in LDS
    kUtsBin = 2,          // BIN tree: one rule for every depth >= 1 (no lookup at all)
    kUtsGeoFixed = 3,     // GEO tree with one table above a depth and leaves below
                          // (shape -a 3: T1, T1L, T1XL): no rule lookup, the first 16
                          // thresholds in registers, the rest (P(n > 16) = 0.8^17 at
                          // b = 4) binary-searched in LDS
};

template <int MODE>
__device__ __forceinline__ int uts_nc(const UtsCtx &c, int d, uint32_t r, uint32_t *err) {
    if (MODE == kUtsBin) return r < c.bin_thr ? c.m : 0;
    if (MODE == kUtsGeoFixed) {
        if (d >= c.geo_depth) return 0;
        // bucket of rand: the thresholds at or below its start (n_lo), and
        // the next two compared — exact whenever at most two thresholds fall
        // inside the bucket (thresholds are sorted): n = #{k : thr[k] <= r}.
        // 6-8 VALU and two LDS reads per node instead of 16 compares (and a
        // binary search in 3 of 4 batches at b = 4, where P(n > 16) is 2.3 %)
        const uint32_t e = ((const uint8_t *)(s_thr + 128))[r >> kUtsBucketShift];
        const uint32_t nlo = e & 0x7fu;
        uint32_t n = nlo + (s_thr[nlo + 1] <= r ? 1u : 0u) + (s_thr[nlo + 2] <= r ? 1u : 0u);
        if (e & 0x80u) {
            // a dense bucket (thresholds past ~23 at b = 4, P ~ 0.6 % per
            // node): binary search of the LDS table above n_lo
            int lo = (int)nlo, hi = 100;
            for (int s = 0; s < 7; ++s) {
                int mid = (lo + hi + 1) >> 1;
                if (lo < hi) {
                    if (s_thr[mid] <= r) lo = mid;
                    else hi = mid - 1;
                }
            }
            n = (uint32_t)lo;
        }
        return (int)n;
    }
    constexpr bool LDS = MODE == kUtsRulesLds;
    int ri = d;
    if (d >= c.nrules) {
        if (!c.stationary) {
            dev_error(err, kErrDepthTable);
            return 0;
        }
        ri = c.nrules - 1;
    }
    const int4 rule = LDS ? s_rules[ri] : c.rules[ri];
    if (rule.x == 0) return rule.y;
    if (rule.x == 1) return r < (uint32_t)rule.y ? c.m : 0;
    const int tb = rule.z * 128;
    int lo = 0, hi = 100;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
        int mid = (lo + hi + 1) >> 1;
        if (lo < hi) {
            const uint32_t t = LDS ? s_thr[tb + mid] : c.thr[tb + mid];
            if (t <= r) lo = mid;
            else hi = mid - 1;
        }
    }
    return lo;
}

// ring items per wave (CAP) and the pieces a task's children are pushed as:
// BIN trees 1024 / 8 (m <= 8 children keep every batch uniform: the register
// carry); GEO trees 512 by default (16 KiB: 8 waves per CU resident), 256 / 1
// (8 KiB) and 1024 / 8 as measured alternatives (HCLIB_HIP_UTS_RING). On 512
// rings a fixed-shape GEO tree pushes a task's children as ONE range item
// (the residual splits in halves as it is popped): fewer ring writes and a
// one-iteration push loop, T1XL 49.7 -> 37.6 ms, T1L 4.48 -> 4.04, against
// 5 pieces (45.0 / 4.17 at 3, 42.3 / 4.43 at 2); rule-table trees keep 5
// (T4 0.88 -> 2.35 ms at 1, T2 1.37 -> 1.65): profiles/r02/pieces_ab.log
template <int MODE, int CAP>
constexpr int uts_pieces() {
    return CAP >= 1024 ? 8 : (CAP >= 512 ? (MODE == kUtsGeoFixed ? 1 : 5) : 1);
}

// FEAT = 0: plain search; 1: sharded (nshards > 1) and/or per-level histogram;
// 2: diagnostic trace (HCLIB_HIP_UTS_TRACE=1): per depth, the earliest
// s_memrealtime (100 MHz) at which any wave reached it, recorded by a wave
// only when its own deepest depth grows (the level_hist array receives
// these times instead of counts); 3: chain stamps (HCLIB_HIP_UTS_TRACE=2,
// BIN trees): one given root-to-leaf chain (HCLIB_HIP_UTS_CHAIN, a file from
// scripts/critpath/uts_chain.c) is followed through the search — its nodes
// carry a flag in the height word's top bit — and level_hist[4d], [4d+1]
// receive when its depth-d node ran and where (worker, narrow loop or not,
// batch fill, dual batch), [4d+2], [4d+3] when it was given away and taken
// if it changed hands (trace_item)
template <int MODE, int FEAT, int CAP = (MODE == kUtsBin ? 1024 : 512)>
struct UtsKind {
    // template = the node {state[5], height}; an item = its children [k, kend)
    static constexpr int kTmplWords = 6;
    static constexpr int kPieces = uts_pieces<MODE, CAP>();
    static constexpr int kWords = 8;
    // every side effect (histogram atomics, trace stamps) is guarded by
    // `counted` / lane 0, so invalid lanes may run the body: branch-free
    // batches for every variant
    static constexpr bool kPure = true;
    static constexpr bool kBoundedChildren = true;  // <= 100 (the root goes through roots())
    using Ctx = UtsCtx;
    // BIN trees: a node has m children or none (the narrow loop's fast path;
    // hx_sched.h KindFixedChildren). Sharded BIN searches drop foreign nodes
    // (0 children) at the split: still none-or-m.
    static constexpr bool kFixedChildren = MODE == kUtsBin;
    __device__ static uint32_t fixed_children(const Ctx &c) { return c.m > 0 ? (uint32_t)c.m : 0u; }
    struct Acc {
        // per lane: at most one node per batch, so 32 bits last 4G batches
        uint32_t nodes = 0, leaves = 0;
        uint32_t maxd = 0;
        uint32_t trace_seen = 0;  // FEAT 2: the deepest depth this wave has stamped
        uint32_t mode = 0;        // FEAT 2: 1 while the scheduler runs the narrow loop (hx_sched.h)
        uint32_t wid = 0;         // FEAT 2: this worker's id (hx_sched.h acc_set_wid)
        // the wave's totals go into its exit record (hx_sched.h Kind concept)
        __device__ void totals(unsigned long long (&c)[8], unsigned long long (&m)[4]) {
            c[0] = wave_sum((unsigned long long)nodes);
            c[1] = wave_sum((unsigned long long)leaves);
            m[0] = (unsigned long long)wave_max(maxd);
        }
    };

    // cross-GPU sharing (GLOBAL launches): a task may move to another rank
    // once its children lie below the shard split (the levels above it are
    // expanded by every rank and counted by shard 0)
    __device__ static bool movable(const Ctx &c, const uint32_t *tmpl) {
        return c.nshards <= 1 || (int)tmpl[5] >= c.split;
    }

    __device__ static int roots(const Ctx &c, Acc &acc, uint32_t *tmpl) {
        // the root node (height 0) is counted once, by shard 0
        if (lane_id() == 0 && c.shard == 0) {
            acc.nodes += 1;
            if (c.root_nc <= 0) acc.leaves += 1;
            if (c.hist && c.hist_levels > 0) atomicAdd(&c.hist[0], 1ull);
        }
        for (int k = 0; k < 5; ++k) tmpl[k] = c.root[k];
        tmpl[5] = FEAT == 3 ? 0x80000000u : 0u;  // FEAT 3: the root heads the traced chain
        return c.root_nc;
    }

    // everything after the spawn: counting, numChildren, the child template
    // (F: the FEAT whose side paths run; the shard filter from F = 1 on)
    template <int F = FEAT>
    __device__ static __forceinline__ int finish(const Ctx &c, Acc &acc, const uint32_t *t, const uint32_t *ch,
                                                 uint32_t *child, uint32_t *err, bool valid) {
        const int h1 = (int)(F == 3 ? t[5] & 0x7fffffffu : t[5]) + 1;
        bool counted = valid;
        // (the worker loop filters only where the seeding cannot reach the
        // split; a wave-uniform branch around this was no faster: the FEAT
        // = 1 body's cost is its code generation, profiles/r06/shard_big_a.log)
        if (F && c.nshards > 1) {
            if (h1 == c.split && (ch[0] % (uint32_t)c.nshards) != (uint32_t)c.shard) return 0;
            if (h1 < c.split && c.shard != 0) counted = false;
        }
        // an invalid lane's template is stale ring bytes: look it up at depth 1
        // so it can neither index past the rule table nor raise kErrDepthTable
        int nc = uts_nc<MODE>(c, valid ? h1 : 1, ch[4] & 0x7fffffffu, err);
        // branch-free counting (invalid lanes of a pure batch count nothing)
        acc.nodes += counted ? 1u : 0u;
        acc.leaves += (counted && nc <= 0) ? 1u : 0u;
        acc.maxd = (counted && (uint32_t)h1 > acc.maxd) ? (uint32_t)h1 : acc.maxd;
        if (F == 1 && counted && c.hist && h1 < c.hist_levels) atomicAdd(&c.hist[h1], 1ull);
        if (F == 2 && c.hist) {
            const uint32_t dm = wave_max(counted ? (uint32_t)h1 : 0u);
            if (dm > acc.trace_seen) {
                acc.trace_seen = dm;
                // stamp = time (low 46 bits: 8 days of 100 MHz ticks, so a box up
                // longer does not push every stamp past the 0xff.. fill) << 17 |
                // worker (16 bits) << 1 | reached in the narrow loop (1) or not
                if (lane_id() == 0 && (int)dm < c.hist_levels)
                    __hip_atomic_fetch_min(&c.hist[dm],
                                           ((__builtin_amdgcn_s_memrealtime() & 0x3fffffffffffull) << 17) |
                                               ((unsigned long long)(acc.wid & 0xffffu) << 1) | acc.mode,
                                           __ATOMIC_RELAXED, HX_AGENT);
            }
        }
        if (!valid) nc = 0;
        child[0] = ch[0];
        child[1] = ch[1];
        child[2] = ch[2];
        child[3] = ch[3];
        child[4] = ch[4];
        child[5] = (uint32_t)h1;
        return nc;
    }

    // FEAT 3: the traced chain's next child index, loaded before the SHA-1
    // by lanes whose node is on the chain (its latency hides behind it)
    __device__ static __forceinline__ uint32_t chain_next(const Ctx &c, const uint32_t *t, bool valid) {
        uint32_t kc = 0xffffffffu;
        if (FEAT == 3 && valid && (t[5] >> 31)) kc = c.chain[(t[5] & 0x7fffffffu) + 1u];
        return kc;
    }
    __device__ static __forceinline__ void chain_stamp(const Ctx &c, const Acc &acc, uint32_t *child, bool on,
                                                       bool valid, uint32_t dual) {
        if constexpr (FEAT == 3) {
            const uint32_t fill = (uint32_t)__builtin_popcountll(__ballot(valid));
            if (on) {
                const uint32_t d = child[5];
                child[5] = d | 0x80000000u;
                c.hist[4 * d] = __builtin_amdgcn_s_memrealtime();
                c.hist[4 * d + 1] = (unsigned long long)((acc.wid & 0xffffu) | (acc.mode << 16) | (dual << 17) |
                                                         (fill << 20));
            }
        }
    }

    // FEAT 3: an item {template, k, kend} holding the traced chain's next
    // node changes hands (hx_sched.h kind_trace_item): level_hist[4d + 2] =
    // when it was given away, [4d + 3] = when it was taken (bit 63: through
    // a sibling's LDS inbox rather than the HBM deques)
    __device__ static void trace_item(const Ctx &c, const uint32_t *w, bool valid, uint32_t ev, bool via_inbox) {
        if constexpr (FEAT == 3) {
            if (valid && (w[5] >> 31)) {
                const uint32_t d = (w[5] & 0x7fffffffu) + 1u;
                const uint32_t kc = c.chain[d];
                if (kc >= w[kWords - 2] && kc < w[kWords - 1])
                    c.hist[4 * d + ev] = __builtin_amdgcn_s_memrealtime() | (via_inbox ? 1ull << 63 : 0ull);
            }
        }
    }

    __device__ static int process(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k,
                                  uint32_t *child, uint32_t *err, bool valid) {
        uint32_t ch[5];
        const uint32_t kc = chain_next(c, t, valid);
        rng_spawn_dev(t, k, ch);
        for (int g = 1; g < c.gran; ++g) rng_spawn_dev(t, k, ch);  // -g: repeated spawns
        const int nc = finish(c, acc, t, ch, child, err, valid);
        chain_stamp(c, acc, child, k == kc, valid, 0u);
        return nc;
    }

    // the fixed-size narrow loop's form (hx_sched.h narrow_loop_fixed; FEAT 0,
    // where a node counts iff its lane is valid): finish<0> without the node
    // and leaf counts, which the loop sums per level as wave-uniform values
    // (nodes = the carry, leaves = the carry less the spawning lanes)
    // Returns whether the node spawns (its m children; the loop runs only
    // with m > 0, so the test is the threshold alone)
    static constexpr bool kBulkCount = FEAT == 0;
    __device__ static __forceinline__ bool process_bulk(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k,
                                                        uint32_t *child, uint32_t *err, bool valid) {
        static_assert(MODE == kUtsBin, "the fixed-size narrow loop runs BIN trees");
        uint32_t ch[5];
        rng_spawn_dev(t, k, ch);
        for (int g = 1; g < c.gran; ++g) rng_spawn_dev(t, k, ch);
        const int h1 = (int)t[5] + 1;
        acc.maxd = (valid && (uint32_t)h1 > acc.maxd) ? (uint32_t)h1 : acc.maxd;
        for (int i = 0; i < 5; ++i) child[i] = ch[i];
        child[5] = (uint32_t)h1;
        return valid && (ch[4] & 0x7fffffffu) < c.bin_thr;
    }
    // (lane 0 holds a wave's bulk counts: at most the tree's nodes, < 2^32
    // for every published tree)
    __device__ static void count_bulk(Acc &acc, uint32_t nodes, uint32_t leaves) {
        if (lane_id() == 0) {
            acc.nodes += nodes;
            acc.leaves += leaves;
        }
    }

    // the breadth-first seeding's slots (hx_sched.h seed_levels) run with the
    // shard filter and the top levels' counting rule whatever FEAT is: a
    // seeded shard's levels reach past its split depth (the host launches
    // FEAT = 0 only then), so its work-stealing loop, the plain kernel of a
    // whole-tree search, never meets a node at or above the split
    __device__ static int seed_process(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k, uint32_t *child,
                                       uint32_t *err, bool valid) {
        uint32_t ch[5];
        rng_spawn_dev(t, k, ch);
        for (int g = 1; g < c.gran; ++g) rng_spawn_dev(t, k, ch);
        return finish<FEAT == 0 ? 1 : FEAT>(c, acc, t, ch, child, err, valid);
    }

    // two nodes per lane (dual batches of the megakernel, hx_sched.h): the two
    // SHA-1 chains interleaved instruction by instruction (uts_sha1.h)
    __device__ static void process2(const Ctx &c, Acc &acc, const uint32_t *tA, uint32_t kA, uint32_t *childA,
                                    int &ncA, const uint32_t *tB, uint32_t kB, uint32_t *childB, int &ncB,
                                    uint32_t *err, bool validB) {
        uint32_t chA[5], chB[5];
        const uint32_t kcA = chain_next(c, tA, true), kcB = chain_next(c, tB, validB);
        const uint32_t *pp[2] = {tA, tB};
        const uint32_t ii[2] = {kA, kB};
        uint32_t *oo[2] = {chA, chB};
        rng_spawn_n<2>(pp, ii, oo);
        for (int g = 1; g < c.gran; ++g) rng_spawn_n<2>(pp, ii, oo);  // -g: repeated spawns
        ncA = finish(c, acc, tA, chA, childA, err, true);
        ncB = finish(c, acc, tB, chB, childB, err, validB);
        chain_stamp(c, acc, childA, kA == kcA, true, 1u);
        chain_stamp(c, acc, childB, kB == kcB, validB, 1u);
    }
};

// GLOBAL: a sharded launch that shares work with the other ranks
// (hclib_hip_global_attach; hx_sched.h GlobalView). WPG: worker waves per
// workgroup, handing work to idle siblings through LDS inboxes (hx_sched.h
// Inbox) before the HBM deques.
template <int MODE, int FEAT, int CAP = (MODE == kUtsBin ? 1024 : 512), bool GLOBAL = false, int WPG = 1>
__global__ __launch_bounds__(64 * WPG) void k_uts_search(UtsCtx ctx, PoolView pool, SchedGlobals *g,
                                                         SchedConfig cfg) {
    constexpr int kUtsCap = CAP;
    using K = UtsKind<MODE, FEAT, CAP>;
    __shared__ WaveStack<K, kUtsCap> st[WPG];
    __shared__ Inbox<K> ib[WPG];
    const uint32_t wave = WPG > 1 ? threadIdx.x / 64 : 0;
    const uint32_t worker = blockIdx.x * WPG + wave;
    if (WPG > 1) {
        if (threadIdx.x < WPG) {
            ib[threadIdx.x].state = 0;
            ib[threadIdx.x].idle = 0;
        }
    }
    if (MODE == kUtsGeoFixed) {
        // table 0 and its bucket bytes in LDS (uts_nc)
        for (int i = threadIdx.x; i < 128; i += 64 * WPG) s_thr[i] = ctx.thr[i];
        for (int i = threadIdx.x; i < kUtsBuckets / 4; i += 64 * WPG) s_thr[128 + i] = ctx.nb[i];
    }
    if (MODE == kUtsRulesLds) {
        // the per-node rule lookup becomes LDS-latency (no dependent HBM/L2 loads)
        for (int i = threadIdx.x; i < ctx.nrules; i += 64 * WPG) s_rules[i] = ctx.rules[i];
        for (int i = threadIdx.x; i < ctx.nthr; i += 64 * WPG) s_thr[i] = ctx.thr[i];
    }
    __syncthreads();
    run_worker<K, kUtsCap, GLOBAL, WPG>(ctx, pool, g, cfg, st[wave], worker == 0, ib, wave, worker);
}

// ------------------------------------------------------ host: rules/tables
// The reference's per-node formula, uts.c:143-222, evaluated with libm.
static int cvt_int_x86(double x) {
    // (int) conversion as x86-64 cvttsd2si: NaN / out of range -> INT_MIN
    if (!(x >= -2147483648.0 && x < 2147483648.0)) return (int)0x80000000u;
    return (int)x;
}

static double geo_bi(const hclib_hip_uts_params_t &p, int depth) {
    double b_i = p.b_0;
    if (depth > 0) {
        switch (p.shape_fn) {
        case 1: b_i = p.b_0 * pow((double)depth, -log(p.b_0) / log((double)p.gen_mx)); break;
        case 2:
            if (depth > 5 * p.gen_mx) { b_i = 0.0; break; }
            b_i = pow(p.b_0, sin(2.0 * 3.141592653589793 * (double)depth / (double)p.gen_mx));
            break;
        case 3: b_i = (depth < p.gen_mx) ? p.b_0 : 0; break;
        default: b_i = p.b_0 * (1.0 - (double)depth / (double)p.gen_mx); break;
        }
    }
    return b_i;
}

static int geo_n(double prob, uint32_t h) {
    double u = (double)(int)h / 2147483648.0;
    return cvt_int_x86(floor(log(1 - u) / log(1 - prob)));
}

// Expected node count of a GEO / HYBRID tree (sum over depths of the product
// of the mean branching factors above it) — a launch-shape heuristic only:
// T1 1.4 M, T2 0.8 M, T4 3.3 M, T5 3.8 M, T1L 89 M, T2L 184 M
static double uts_expected_nodes(const hclib_hip_uts_params_t &p) {
    double tot = 0.0, prod = 1.0;
    for (int d = 0; d < 10 * p.gen_mx + 10 && prod > 1e-9 && tot < 1e13; ++d) {
        tot += prod;
        const bool bin_level = p.type == 0 ? d > 0 : (p.type == 2 && d >= p.shift_depth * p.gen_mx);
        const double mu = bin_level ? p.non_leaf_prob * p.non_leaf_bf : geo_bi(p, d);
        prod *= mu > 0.0 ? mu : 0.0;
    }
    return tot;
}

struct UtsTables {
    std::vector<int4> rules;
    std::vector<uint32_t> thr;  // 128 words per geo table
    int stationary = 1;
    int root_nc = 0;
    uint32_t root[5];
};

static void sha1_host(uint32_t w[16], uint32_t h[5]) {
    uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u, e = 0xc3d2e1f0u;
    for (int i = 0; i < 80; ++i) {
        uint32_t wi = (i < 16) ? w[i] : HX_W(i);
        if (i < 20) HX_RND(HX_F1, 0x5a827999u, wi)
        else if (i < 40) HX_RND(HX_F2, 0x6ed9eba1u, wi)
        else if (i < 60) HX_RND(HX_F3, 0x8f1bbcdcu, wi)
        else HX_RND(HX_F2, 0xca62c1d6u, wi)
    }
    h[0] = 0x67452301u + a;
    h[1] = 0xefcdab89u + b;
    h[2] = 0x98badcfeu + c;
    h[3] = 0x10325476u + d;
    h[4] = 0xc3d2e1f0u + e;
}

// Build the geo table for b_i; returns table index (deduplicated) or -1 for
// "always 0 children"; -2 if the formula is not monotone in rand (unsupported).
static int geo_table(UtsTables &T, double b_i) {
    const double prob = 1.0 / (1.0 + b_i);
    uint32_t thr[128];
    thr[0] = 0;
    bool any = false;
    const int nmax = geo_n(prob, 0x7fffffffu);
    for (int k = 1; k <= 100; ++k) {
        if (nmax < k) {  // never reached (INT_MIN / capped by the range end)
            thr[k] = 0x80000000u;
            continue;
        }
        uint32_t lo = 0, hi = 0x7fffffffu;  // smallest h with n(h) >= k
        while (lo < hi) {
            uint32_t mid = lo + (hi - lo) / 2;
            if (geo_n(prob, mid) >= k) hi = mid;
            else lo = mid + 1;
        }
        thr[k] = lo;
        any = true;
    }
    for (int k = 101; k < 128; ++k) thr[k] = 0x80000000u;
    if (!any) return -1;
    // spot-verify monotonicity / table agreement around every threshold
    for (int k = 1; k <= 100; ++k) {
        if (thr[k] == 0x80000000u) break;
        for (int dlt = -2; dlt <= 2; ++dlt) {
            int64_t hh = (int64_t)thr[k] + dlt;
            if (hh < 0 || hh > 0x7fffffff) continue;
            int n = geo_n(prob, (uint32_t)hh);
            int want = n < 0 ? 0 : (n > 100 ? 100 : n);
            int got = 0;
            for (int q = 1; q <= 100; ++q) got += thr[q] <= (uint32_t)hh;
            if (got != want) return -2;
        }
    }
    const size_t nt = T.thr.size() / 128;
    if (nt && !memcmp(&T.thr[(nt - 1) * 128], thr, sizeof(thr))) return (int)(nt - 1);
    T.thr.insert(T.thr.end(), thr, thr + 128);
    return (int)nt;
}

static int bin_threshold(double q) {
    // smallest h with h/2^31 >= q; rand < thr  <=>  d < q (uts.c:162-168)
    uint32_t lo = 0, hi = 0x80000000u;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (((double)(int)mid) / 2147483648.0 >= q) hi = mid;
        else lo = mid + 1;
    }
    return (int)lo;
}

static int build_tables(const hclib_hip_uts_params_t &p, UtsTables &T) {
    T.rules.clear();
    T.thr.clear();
    auto geo_rule = [&](int d) -> int4 {
        int t = geo_table(T, geo_bi(p, d));
        if (t == -1) return make_int4(0, 0, 0, 0);
        if (t == -2) return make_int4(-1, 0, 0, 0);
        return make_int4(2, 0, t, 0);
    };
    int D = 0;
    switch (p.type) {
    case 0:  // BIN
        T.rules.push_back(make_int4(0, 0, 0, 0));  // root handled by root_nc
        T.rules.push_back(make_int4(1, bin_threshold(p.non_leaf_prob), 0, 0));
        T.stationary = 1;
        break;
    case 1:  // GEO
        if (p.shape_fn == 3 || p.shape_fn == 0) { D = p.gen_mx + 1; T.stationary = 1; }
        else if (p.shape_fn == 2) { D = 5 * p.gen_mx + 2; T.stationary = 1; }
        else { D = 4096; T.stationary = 0; }
        for (int d = 0; d < D; ++d) T.rules.push_back(geo_rule(d));
        if (T.stationary) T.rules.push_back(make_int4(0, 0, 0, 0));
        break;
    case 2: {  // HYBRID: geo below shift_depth*gen_mx, bin after
        int d = 0;
        for (; d < p.shift_depth * p.gen_mx; ++d) T.rules.push_back(geo_rule(d));
        T.rules.push_back(make_int4(1, bin_threshold(p.non_leaf_prob), 0, 0));
        T.stationary = 1;
        break;
    }
    case 3:  // BALANCED
        for (int d = 0; d < p.gen_mx; ++d) T.rules.push_back(make_int4(0, (int)p.b_0, 0, 0));
        T.rules.push_back(make_int4(0, 0, 0, 0));
        T.stationary = 1;
        break;
    default:
        set_error("uts: unknown tree type %d", p.type);
        return HCLIB_HIP_EINVAL;
    }
    for (auto &r : T.rules)
        if (r.x == -1) {
            set_error("uts: numChildren is not monotone in rand for these parameters");
            return HCLIB_HIP_EINVAL;
        }
    if (T.thr.empty()) T.thr.assign(128, 0x80000000u);
    // the root (uts_initRoot uts.c:151-159 + uts_numChildren at height 0)
    uint32_t w[16] = {0};
    w[4] = (uint32_t)p.root_id;
    w[5] = 0x80000000u;
    w[15] = 160;
    sha1_host(w, T.root);
    const uint32_t r = T.root[4] & 0x7fffffffu;
    int nc = 0;
    switch (p.type) {
    case 0: nc = (int)floor(p.b_0); break;
    case 1: nc = geo_n(1.0 / (1.0 + geo_bi(p, 0)), r); break;
    case 2: nc = (0 < p.shift_depth * p.gen_mx) ? geo_n(1.0 / (1.0 + geo_bi(p, 0)), r)
                                               : ((((double)(int)r) / 2147483648.0 < p.non_leaf_prob) ? p.non_leaf_bf : 0);
            break;
    case 3: nc = (0 < p.gen_mx) ? (int)p.b_0 : 0; break;
    }
    if (p.type == 0) {
        int root_bf = (int)ceil(p.b_0);
        if (nc > root_bf) nc = root_bf;
    } else if (p.type != 3 && nc > 100) {
        nc = 100;
    }
    T.root_nc = nc;
    return HCLIB_HIP_OK;
}

// table 0's bucket bytes (kUtsGeoFixed, uts_nc): per bucket
// [b 2^21, (b+1) 2^21) of rand, n_lo = #{k : thr[k] <= b 2^21} and 0x80 when
// more than two thresholds lie strictly inside it
static void build_buckets(const uint32_t *t0, uint8_t nb[kUtsBuckets]) {
    for (int b = 0; b < kUtsBuckets; ++b) {
        const uint64_t lo = (uint64_t)b << kUtsBucketShift, hi = (uint64_t)(b + 1) << kUtsBucketShift;
        int nlo = 0, inside = 0;
        for (int k = 1; k <= 100; ++k) {
            nlo += t0[k] <= lo;
            inside += t0[k] > lo && t0[k] < hi;
        }
        nb[b] = (uint8_t)(nlo | (inside > 2 ? 0x80 : 0));
    }
}

// the device lookup of uts_nc<kUtsGeoFixed> (below the depth cut), on the
// host: bucket byte, two compares, binary search in a dense bucket
static int bucket_nc(const uint32_t *t0, const uint8_t *nb, uint32_t r) {
    const uint32_t e = nb[r >> kUtsBucketShift], nlo = e & 0x7fu;
    uint32_t n = nlo + (t0[nlo + 1] <= r ? 1u : 0u) + (t0[nlo + 2] <= r ? 1u : 0u);
    if (e & 0x80u) {
        int lo = (int)nlo, hi = 100;
        for (int s = 0; s < 7; ++s) {
            const int mid = (lo + hi + 1) >> 1;
            if (lo < hi) {
                if (t0[mid] <= r) lo = mid;
                else hi = mid - 1;
            }
        }
        n = (uint32_t)lo;
    }
    return (int)n;
}

static int host_nc(const hclib_hip_uts_params_t &p, const UtsTables &T, int d, uint32_t r) {
    int ri = d < (int)T.rules.size() ? d : (int)T.rules.size() - 1;
    int4 rule = T.rules[ri];
    if (rule.x == 0) return rule.y;
    if (rule.x == 1) return r < (uint32_t)rule.y ? p.non_leaf_bf : 0;
    int n = 0;
    for (int k = 1; k <= 100; ++k) n += T.thr[(size_t)rule.z * 128 + k] <= r;
    return n;
}

}  // namespace hx

using namespace hx;

extern "C" int hclib_hip_uts_num_children_host(const hclib_hip_uts_params_t *params, int height,
                                               const uint32_t st[5]) {
    // tables are pure functions of the parameters: cache the last set
    static hclib_hip_uts_params_t last_p;
    static UtsTables T;
    static bool have = false;
    if (!have || memcmp(&last_p, params, sizeof(last_p)) != 0) {
        have = false;
        if (build_tables(*params, T) != HCLIB_HIP_OK) return -1;
        last_p = *params;
        have = true;
    }
    if (height == 0) return T.root_nc;
    return host_nc(*params, T, height, st[4] & 0x7fffffffu);
}

// Host check of the bucketed numChildren lookup (no GPU needed): for the
// tree's first threshold table, the bucket method against the exact count
// #{k : thr[k] <= r} at every threshold +-3, every bucket edge +-1 and
// `nrandom` splitmix values of rand. Returns the mismatches (0) or a negative
// error; *checked receives the values compared.
extern "C" int hclib_hip_uts_bucket_check(const hclib_hip_uts_params_t *params, uint64_t nrandom,
                                          uint64_t *checked) {
    if (!params) {
        set_error("hclib_hip_uts_bucket_check: NULL params");
        return HCLIB_HIP_EINVAL;
    }
    UtsTables T;
    if (build_tables(*params, T) != HCLIB_HIP_OK) return HCLIB_HIP_EINVAL;
    if (T.thr.size() < 128) {  // no threshold table (BIN or constant rules)
        if (checked) *checked = 0;
        return 0;
    }
    const uint32_t *t0 = T.thr.data();
    uint8_t nb[kUtsBuckets];
    build_buckets(t0, nb);
    uint64_t n = 0;
    int bad = 0;
    auto one = [&](int64_t v) {
        if (v < 0 || v > 0x7fffffffll) return;
        const uint32_t r = (uint32_t)v;
        int exact = 0;
        for (int k = 1; k <= 100; ++k) exact += t0[k] <= r;
        bad += bucket_nc(t0, nb, r) != exact;
        ++n;
    };
    for (int k = 1; k <= 100; ++k)
        if (t0[k] != 0x80000000u)
            for (int d = -3; d <= 3; ++d) one((int64_t)t0[k] + d);
    for (int b = 0; b <= kUtsBuckets; ++b)
        for (int d = -1; d <= 1; ++d) one(((int64_t)b << kUtsBucketShift) + d);
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (uint64_t i = 0; i < nrandom; ++i) {
        x += 0x9e3779b97f4a7c15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        one((int64_t)((z ^ (z >> 31)) & 0x7fffffffull));
    }
    if (checked) *checked = n;
    return bad;
}

static thread_local hclib_hip_uts_launch_t g_last_launch{-1, 0, 0, 0, 0, 0, 0, 0, 0};

extern "C" int hclib_hip_uts_last_launch(hclib_hip_uts_launch_t *out) {
    if (!out) {
        set_error("hclib_hip_uts_last_launch: null output");
        return HCLIB_HIP_EINVAL;
    }
    *out = g_last_launch;
    return g_last_launch.mode < 0 ? HCLIB_HIP_EINVAL : HCLIB_HIP_OK;
}

extern "C" int hclib_hip_uts_search(const hclib_hip_uts_params_t *params, int shard, int nshards,
                                    int split_depth, hclib_hip_uts_result_t *result,
                                    uint64_t *level_hist, int max_levels) {
    if (!params || !result || nshards < 1 || shard < 0 || shard >= nshards || max_levels < 0 ||
        max_levels > (env_int("HCLIB_HIP_UTS_TRACE", 0) == 2 ? 4 * 65536 : 65536) || (nshards > 1 && split_depth < 1)) {
        set_error("hclib_hip_uts_search: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = mod();
    // The rule / threshold tables are pure functions of the parameters and
    // cost ~1 ms of libm on the host for a GEO tree (100 threshold searches
    // per depth): the last set and its device copy are kept for the next
    // search of the same tree (every call returns with the stream drained, so
    // no launch still reads them when they are replaced)
    static struct {
        bool have = false;
        int device = -1;
        hclib_hip_uts_params_t p;
        UtsTables T;
        void *dmem = nullptr;
    } tab;
    if (!tab.have || tab.device != m.device || memcmp(&tab.p, params, sizeof(tab.p)) != 0) {
        if (tab.dmem && tab.device == m.device) (void)hipFree(tab.dmem);
        tab.have = false;
        tab.dmem = nullptr;
        HX_TRY(build_tables(*params, tab.T));
        const size_t rb = tab.T.rules.size() * sizeof(int4), tb = tab.T.thr.size() * 4;
        HX_HIP(hipMalloc(&tab.dmem, ((rb + 255) & ~(size_t)255) + ((tb + 255) & ~(size_t)255) + kUtsBuckets + 256));
        char *dp = (char *)tab.dmem;
        HX_HIP(hipMemcpy(dp, tab.T.rules.data(), rb, hipMemcpyHostToDevice));
        HX_HIP(hipMemcpy(dp + ((rb + 255) & ~(size_t)255), tab.T.thr.data(), tb, hipMemcpyHostToDevice));
        uint8_t nb[kUtsBuckets] = {0};
        if (tab.T.thr.size() >= 128) build_buckets(tab.T.thr.data(), nb);
        HX_HIP(hipMemcpy(dp + ((rb + 255) & ~(size_t)255) + ((tb + 255) & ~(size_t)255), nb, kUtsBuckets,
                         hipMemcpyHostToDevice));
        tab.p = *params;
        tab.device = m.device;
        tab.have = true;
    }
    const UtsTables &T = tab.T;
    int4 *d_rules = (int4 *)tab.dmem;
    uint32_t *d_thr = (uint32_t *)((char *)tab.dmem + ((T.rules.size() * sizeof(int4) + 255) & ~(size_t)255));
    const uint32_t *d_nb = (const uint32_t *)((char *)d_thr + ((T.thr.size() * 4 + 255) & ~(size_t)255));

    // the optional per-level histogram
    const size_t hb = (size_t)max_levels * 8;
    void *dmem = nullptr;
    if (max_levels) HX_HIP(hipMalloc(&dmem, hb));
    unsigned long long *d_hist = (unsigned long long *)dmem;
    const int trace_kind = max_levels > 0 ? env_int("HCLIB_HIP_UTS_TRACE", 0) : 0;
    const bool trace = trace_kind != 0;
    if (max_levels) HX_HIP(hipMemsetAsync(d_hist, trace ? 0xff : 0, hb, m.stream));
    // FEAT 3 (diagnostic): the chain to follow, k_1..k_D of scripts/critpath/uts_chain.c
    uint32_t *d_chain = nullptr;
    if (trace_kind == 2) {
        std::vector<uint32_t> chain;
        const char *path = getenv("HCLIB_HIP_UTS_CHAIN");
        if (FILE *f = path ? fopen(path, "rb") : nullptr) {
            uint32_t w;
            while (fread(&w, 4, 1, f) == 1) chain.push_back(w);
            fclose(f);
        }
        if (chain.empty() || chain[0] + 1 != chain.size() || (size_t)max_levels < 4 * chain.size()) {
            (void)hipFree(dmem);
            set_error("hclib_hip_uts_search: chain trace needs HCLIB_HIP_UTS_CHAIN and max_levels >= 4 (D + 1)");
            return HCLIB_HIP_EINVAL;
        }
        HX_HIP(hipMalloc(&d_chain, chain.size() * 4));
        HX_HIP(hipMemcpy(d_chain, chain.data(), chain.size() * 4, hipMemcpyHostToDevice));
    }

    UtsCtx ctx;
    memcpy(ctx.root, T.root, sizeof(ctx.root));
    ctx.root_nc = T.root_nc;
    ctx.nrules = (int)T.rules.size();
    ctx.stationary = T.stationary;
    ctx.gran = params->compute_gran < 1 ? 1 : params->compute_gran;
    ctx.m = params->non_leaf_bf;
    ctx.shard = shard;
    ctx.nshards = nshards;
    ctx.split = split_depth;
    ctx.hist_levels = max_levels;
    ctx.rules = d_rules;
    ctx.thr = d_thr;
    ctx.hist = max_levels ? d_hist : nullptr;
    ctx.chain = d_chain;

    ctx.lds_tables = (T.rules.size() <= kUtsLdsRules && T.thr.size() <= kUtsLdsThr) ? 1 : 0;
    ctx.bin_thr = 0;
    ctx.nthr = (int)T.thr.size();
    // one GEO table for depths 1..D-1, constant 0 children from D on
    int geo_depth = 0;
    {
        const int nr = (int)T.rules.size();
        int d = 1;
        while (d < nr && T.rules[d].x == 2 && T.rules[d].z == 0) ++d;
        bool rest_zero = d > 1 && T.stationary;
        for (int e = d; e < nr && rest_zero; ++e) rest_zero = T.rules[e].x == 0 && T.rules[e].y == 0;
        if (rest_zero && T.thr.size() >= 128) geo_depth = d;
    }
    ctx.geo_depth = geo_depth;
    ctx.nb = d_nb;

    PoolView pool;
    // 128 chunk deques (8 per XCD slice of 16): T3L 28.64 -> 28.57 ms and
    // 28.73 -> 28.58, T1XL 31.19 -> 31.00, T1 0.206 -> 0.202 (means of
    // interleaved rounds, profiles/r05/sweep_dq_*.log, sweep_t3l_j.log); 32
    // is a millisecond slower on T3L
    const uint32_t nq = (uint32_t)env_int("HCLIB_HIP_DEQUES", 128);
    HX_TRY(make_pool(nq, (uint32_t)env_int("HCLIB_HIP_DEQUE_CAP", 4096),
                     (uint32_t)env_int("HCLIB_HIP_CHUNK", 64), UtsKind<kUtsBin, 0>::kWords, &pool));
    const bool bin = params->type == 0 && T.rules.size() == 2 && T.rules[1].x == 1 && T.stationary;
    const bool geo_fixed = !bin && geo_depth > 0 && env_int("HCLIB_HIP_UTS_GEO_FIXED", 1);
    // waves per CU: span-bound BIN trees run fastest with 2 (fewer idle
    // pollers, fewer hand-offs); GEO trees are throughput-bound and fill 8
    // (the 512-item rings leave room for them) once they are large — a
    // small tree (T1, ~4 M nodes in 1 ms) loses more to spreading its few
    // first levels over 2048 waves than it gains (profiles/r02/
    // sweep_t1xl_waves_geo.log: T1XL 90 -> 52 ms from 4 to 8, T1 1.0 ->
    // 1.45 ms). Size: uts_expected_nodes.
    // Rule-table trees (other shapes, HYBRID) of a few million nodes run
    // fastest with 4 (T2 1.80 -> 1.36 ms, T4 1.05 -> 0.86, T5 1.07 -> 0.96;
    // T2L still wants 8: profiles/r02/geo_spill.log)
    // sharded launches of a rank attached to a global region share work
    const bool global = nshards > 1 && m.gview.hdr != nullptr && max_levels == 0;
    // fixed-shape trees start seeded (breadth-first, hx_sched.h seed_levels)
    const bool seed_on = geo_fixed && !global && env_int("HCLIB_HIP_UTS_SEED", 1);
    // BIN shards: the grid expands the replicated top levels breadth-first to
    // the split depth (hx_sched.h seed_levels, the shard filter inside the
    // seeding) and then runs the plain kernel of a whole-tree search. With
    // the filter in the worker loop instead (FEAT = 1) the shard holding
    // T3L's deep chain ran 2.3-2.7 ms slower than the whole tree, although
    // below the split the filter executes nothing: the FEAT = 1 body
    // compiles the span-bound narrow loop worse (the FEAT = 0 kernel on the
    // same shard: +0.05-0.14 ms; profiles/r06/shard_big_a.log)
    const bool bin_seed = bin && nshards > 1 && !global && max_levels == 0 && split_depth >= 1 &&
                          split_depth + 1 < kSeedMaxLevels && env_int("HCLIB_HIP_UTS_SEED", 1);
    // BIN trees: four worker waves per CU in one workgroup (one per SIMD;
    // three siblings to hand work to through LDS before the HBM deques):
    // T3L 29.08 -> 28.76 ms mean of 6 interleaved rounds against two per CU
    // in pairs, T3 2.78 -> 2.76 (profiles/r05/sweep_wpg_t3l.log,
    // sweep_wpg_t3.log; the critical chain's HBM hand-offs 560 -> 295,
    // t3l_chain_wpg.jsonl). Launches that share work across ranks keep 2
    int wpc_default = bin && !global ? 4 : 2, ring_default = 512;
    if (!bin) {
        const double est = uts_expected_nodes(*params);
        if (seed_on) {
            // seeded: every wave starts busy, so even a small tree fills 8
            // waves per CU on 512-item rings once its seeding is cheap (round
            // 5: T1 0.234 -> 0.220 ms at 8 waves per CU and 16 slots per wave,
            // profiles/r05/sweep_t1_d.log; round 4 had 4 per CU, 0.28 vs 0.61
            // ms unseeded on 2 / 256, profiles/r04/seed*_t1.log)
            wpc_default = 8;
            ring_default = 512;
        } else {
            wpc_default = est >= 3e7 ? 8 : (geo_fixed ? 2 : 4);
            // an unseeded small tree runs faster on 256-item rings (one piece
            // per task: the frontier fans out by range splitting), a fixed-shape
            // one at 2 waves per CU: T1 0.98 -> 0.70 ms; a large one slower
            // (T1XL 52 -> 70 ms), profiles/r02/sweep_t1_ring_waves.log,
            // sweep_t1xl_ring_waves.log, geo_lds_tail.log
            ring_default = est >= 3e7 ? 512 : 256;
        }
    }
    const int grid = env_int("HCLIB_HIP_GRID", 0) > 0
                         ? env_int("HCLIB_HIP_GRID", 0)
                         : m.num_cus * env_int("HCLIB_HIP_WAVES_PER_CU", wpc_default);
    SchedConfig cfg;
    cfg.spill_hi = (uint32_t)env_int("HCLIB_HIP_SPILL_HI", 512);
    // BIN trees with the narrow-frontier loop give work away from 72 items
    // (just over one batch: a wave keeps at most ~one batch of a narrow
    // frontier, T3L 36.3 -> 35.0 ms, profiles/r02/t3l_knobs.log). GEO trees
    // keep far more before feeding hungry waves (fewer, fuller hand-offs;
    // profiles/r02/geo_spill.log): 224 with rule tables (T2 2.82 -> 1.71 ms,
    // T5 1.40 -> 1.00, T2L 6.33 -> 5.20) and on the fixed-shape 512-item rings
    // at one piece per task (T1XL 37.2 ms, T1L 3.77; profiles/r02/
    // pieces_tune.log; 336 at five pieces), 128 on 256-item rings (T1)
    const int ring_used = geo_fixed && !(nshards > 1 || max_levels > 0) ? env_int("HCLIB_HIP_UTS_RING", ring_default) : 512;
    // BIN trees: 66 since the register carry went through LDS (T3L 30.64 ->
    // 30.20 ms same-box against 72, profiles/r04/sc_ab_t3l*.log, t3l3_spill.log);
    // it must stay above one batch (64) or the narrow loop never runs
    int spill_lo_default = bin ? 66 : (geo_fixed && ring_used < 512) ? 128 : 224;
    // seeded fixed-shape trees (below) start with every wave busy, so a wave
    // keeps more before it feeds others: T1 0.285 -> 0.248 ms at 336, T1L
    // 2.70 -> 2.38, T1XL's 8-way shards 4.94 -> 4.75 at 448
    // (profiles/r04/seed5_*.log, seed6_*.log)
    const bool seeded = seed_on && ring_used >= 512;
    if (seeded) spill_lo_default = uts_expected_nodes(*params) >= 3e7 ? 448 : 336;
    cfg.spill_lo = (uint32_t)env_int("HCLIB_HIP_SPILL_LO", spill_lo_default);
    cfg.spin_limit = (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    cfg.nwaves = (uint32_t)grid;
    cfg.stamps = (uint32_t)env_int("HCLIB_HIP_STAMPS", 0);
    // hunger read every 32 batches, every 8 while many waves are hungry
    // (scripts/sweep_uts.py: T1 1.37 -> 1.07 ms, T1XL 101 -> 97 ms, T3L even)
    // (fixed-shape GEO trees on 512-item rings every 64: T1XL 51.5 -> 49.9 ms,
    // T1L even, T2L slower; profiles/r02/geo_knobs.log)
    // hunger read interval: 64 batches on BIN trees (T3L 29.34 -> 29.23 ms mean of 7 interleaved rounds, and
    // -0.14 ms in two shorter sweeps: profiles/r05/sweep_h64sp1_t3l.log,
    // sweep_wpg4_t3l.log, sweep_spills_t3l.log), 32 otherwise
    // ... except small fixed-shape trees (expected < 3e7 nodes), which run
    // a few dozen batches per wave: 32 (T1 0.210 -> 0.200-0.201 ms mean of 6
    // and 8 interleaved rounds; T1L wants 64: 2.44 vs 2.48 ms;
    // profiles/r05/sweep_t1_g.log, sweep_t1_h.log, sweep_t1l_h.log)
    // ... and large fixed-shape trees every 128 (T1XL 31.15 -> 30.77 ms, T1L
    // 2.417 -> 2.383, means of 4-5 interleaved rounds, sweep_t1xl_l.log,
    // sweep_t1l_l.log)
    const bool small_fixed = geo_fixed && uts_expected_nodes(*params) < 3e7;
    const bool large_fixed = geo_fixed && ring_used >= 512 && !small_fixed;
    cfg.hunger = (uint32_t)env_int("HCLIB_HIP_HUNGER", large_fixed ? 128 : bin ? 64 : 32);
    cfg.carry = (uint32_t)env_int("HCLIB_HIP_CARRY", 2);
    cfg.backoff = (uint32_t)env_int("HCLIB_HIP_BACKOFF", 16);
    cfg.defer = (uint32_t)env_int("HCLIB_HIP_DEFER", 1);
    // dual batches (two nodes per lane while a wave holds > 64 items; kinds
    // whose ring fits two batches' pushes: the fixed-shape GEO trees on
    // 512-item rings)
    cfg.dual = (uint32_t)env_int("HCLIB_HIP_UTS_DUAL", 1);
    cfg.spills = (uint32_t)env_int("HCLIB_HIP_SPILLS_PER_BATCH", 0);
    // breadth-first seeding (hx_sched.h seed_levels) for fixed-shape GEO
    // trees: the grid expands the top levels together and shares the level
    // that reaches HCLIB_HIP_SEED_PER_WAVE slots per wave out evenly, instead
    // of growing the busy set from one root by hand-offs
    SeedCfg seed{0, 0, (uint32_t)UtsKind<kUtsBin, 0>::kWords, 0};
    if (seeded) {
        // slots per wave: a few for a small tree (one level fewer to expand),
        // more for a large one (finer shares, less stealing later;
        // profiles/r04/seed3_*.log, seed4_*.log)
        // (16 for small trees since round 5: one level deeper, T1 0.234 ->
        // 0.220 ms, profiles/r05/sweep_t1_d.log; a level holds at most ~b x
        // the target, so 32 keeps a wave's share of a b = 4 level within
        // half its ring)
        const int per_wave = env_int("HCLIB_HIP_SEED_PER_WAVE", uts_expected_nodes(*params) >= 3e7 ? 32 : 16);
        seed.target = (uint32_t)(grid * per_wave);
        seed.max_levels = (uint32_t)env_int("HCLIB_HIP_SEED_LEVELS", 20);
        // wave 0 alone runs the levels of at most 128 slots (its ring's room
        // is 224): a level of 189 (T1's depth 3) is cheaper on the grid
        // (T1 median 0.2051-0.2067 -> 0.1976-0.2011 ms over 18 + 40 launches,
        // T1L 2.490 -> 2.465; profiles/r06/sweep_t1_solo*.log)
        seed.solo_cap = (uint32_t)env_int("HCLIB_HIP_SEED_SOLO", 128);
        // a shard's share is only known past its split (level d holds the
        // slots of depth d + 1, filtered when they run), so the seeding goes
        // on to the split — where the levels up to it fit the seeding's
        // buffers (expected sizes n(d) = prod b_k): the unfiltered level
        // (n(split) slots) within half the level buffer, and this shard's
        // share of the level past it within a quarter of each wave's ring
        // (hx_sched.h seed_levels: the buffer holds 8 x target + 65,536
        // slots, a wave takes at most CAP / 2 items). Deeper splits seed
        // only to the target and filter in the worker loop (FEAT = 1).
        if (nshards > 1) {
            double n_split = 1.0, n_next = 1.0;
            for (int d = 0; d <= split_depth && d < 64; ++d) {
                if (d < split_depth) n_split *= geo_bi(*params, d) > 0 ? geo_bi(*params, d) : 0.0;
                n_next *= geo_bi(*params, d) > 0 ? geo_bi(*params, d) : 0.0;
            }
            const double cap = 8.0 * seed.target + 65536.0;
            const bool fits = split_depth + 1 < kSeedMaxLevels && split_depth < (int)seed.max_levels &&
                              n_split <= 0.5 * cap && n_next / nshards <= (double)grid * (512 / 8);
            seed.min_levels = fits ? (uint32_t)split_depth : 0u;
        }
    } else if (bin_seed) {
        // exactly the split's levels: a BIN level holds ~b0 slots (critical
        // branching, sd ~ sqrt(b0 d m^2 q (1 - q))), far inside the buffer
        seed.target = 1;
        seed.max_levels = (uint32_t)split_depth;
        seed.min_levels = (uint32_t)split_depth;
    }
    HX_TRY(reset_sched(pool, 1, global, (uint32_t)grid, seed.target ? &seed : nullptr));
    HX_HIP(hipEventRecord(m.ev0, m.stream));
    // a sharded search whose seeding reaches past its split (every seeded
    // fixed-shape shard with split < the seeding's level bound) filters its
    // shard inside the seeding (UtsKind::seed_process) and then runs the
    // plain kernel; otherwise the worker loop itself filters (FEAT = 1)
    const bool seed_past_split = seed.target && nshards > 1 &&
                                 seed.min_levels == (uint32_t)split_depth;
    const bool feat = max_levels > 0 || (nshards > 1 && (global || !seed_past_split));
    if (bin) ctx.bin_thr = (uint32_t)T.rules[1].y;
    const int mode = bin ? kUtsBin : geo_fixed ? kUtsGeoFixed : (ctx.lds_tables ? kUtsRulesLds : kUtsRulesGlobal);
    typedef void (*uts_kernel_t)(UtsCtx, PoolView, SchedGlobals *, SchedConfig);
    static const uts_kernel_t kernels[4][2] = {
        {k_uts_search<kUtsRulesGlobal, 0>, k_uts_search<kUtsRulesGlobal, 1>},
        {k_uts_search<kUtsRulesLds, 0>, k_uts_search<kUtsRulesLds, 1>},
        {k_uts_search<kUtsBin, 0>, k_uts_search<kUtsBin, 1>},
        {k_uts_search<kUtsGeoFixed, 0>, k_uts_search<kUtsGeoFixed, 1>},
    };
    uts_kernel_t kern = kernels[mode][feat ? 1 : 0];
    if (trace) {
        if (mode != kUtsBin || nshards > 1) {
            (void)hipFree(dmem);
            if (d_chain) (void)hipFree(d_chain);
            set_error("hclib_hip_uts_search: the depth trace is for unsharded BIN trees");
            return HCLIB_HIP_EINVAL;
        }
        kern = trace_kind == 2 ? k_uts_search<kUtsBin, 3> : k_uts_search<kUtsBin, 2>;
    }
    if (global) {
        static const uts_kernel_t gkernels[4] = {
            k_uts_search<kUtsRulesGlobal, 1, 512, true>, k_uts_search<kUtsRulesLds, 1, 512, true>,
            k_uts_search<kUtsBin, 1, 1024, true>, k_uts_search<kUtsGeoFixed, 1, 512, true>};
        kern = gkernels[mode];
    }
    // ring-size variants of the fixed-shape GEO search: whole-tree launches
    // only (ring_used: sharded and histogram launches size spill_lo and the
    // seeding's fit check for 512-item rings)
    if (mode == kUtsGeoFixed && !feat && !global) {
        if (ring_used == 256) kern = k_uts_search<kUtsGeoFixed, 0, 256>;
        else if (ring_used == 1024) kern = k_uts_search<kUtsGeoFixed, 0, 1024>;
    }
    // BIN trees: the worker waves of a CU share a workgroup and hand work
    // to each other through LDS before the HBM deques (two: T3L 34.0 ->
    // 33.5-33.7 ms, profiles/r02/inbox_ab.log; four since round 5, see
    // wpc_default; HCLIB_HIP_WPG = 1, 2 or 4)
    int wpg = 1;
    if (mode == kUtsBin && !global && (!trace || trace_kind == 2)) {
        wpg = env_int("HCLIB_HIP_WPG", 4);
        if (wpg != 2 && wpg != 4) wpg = 1;
        if (grid % wpg) wpg = 1;
        if (trace_kind == 2 && wpg == 2) kern = k_uts_search<kUtsBin, 3, 1024, false, 2>;
        else if (trace_kind == 2 && wpg == 4) kern = k_uts_search<kUtsBin, 3, 1024, false, 4>;
        else if (wpg == 2) kern = feat ? k_uts_search<kUtsBin, 1, 1024, false, 2> : k_uts_search<kUtsBin, 0, 1024, false, 2>;
        else if (wpg == 4) kern = feat ? k_uts_search<kUtsBin, 1, 1024, false, 4> : k_uts_search<kUtsBin, 0, 1024, false, 4>;
    }
    {
        int ring_k = mode == kUtsBin ? 1024 : 512;
        if (mode == kUtsGeoFixed && !feat && !global && (ring_used == 256 || ring_used == 1024)) ring_k = ring_used;
        g_last_launch = hclib_hip_uts_launch_t{mode, trace ? 1 + trace_kind : (feat || global ? 1 : 0), wpg, grid, ring_k,
                                               seed.target ? 1 : 0, (int)seed.target, (int)cfg.spill_lo,
                                               grid / (m.num_cus > 0 ? m.num_cus : 1)};
    }
    HX_TRY(check_resident((const void *)kern, grid / wpg, 64 * wpg, 0, "hclib_hip_uts_search"));
    hipLaunchKernelGGL(kern, dim3(grid / wpg), dim3(64 * wpg), 0, m.stream, ctx, pool, m.globals, cfg);
    HX_HIP(hipGetLastError());
    HX_HIP(hipEventRecord(m.ev1, m.stream));
    SchedGlobals gl;
    int rc = finish_sched(&gl, "hclib_hip_uts_search");
    float ms = 0;
    (void)hipEventElapsedTime(&ms, m.ev0, m.ev1);
    if (rc == HCLIB_HIP_OK && max_levels) {
        std::vector<unsigned long long> h(max_levels);
        HX_HIP(hipMemcpy(h.data(), d_hist, hb, hipMemcpyDeviceToHost));
        for (int i = 0; i < max_levels; ++i) level_hist[i] = h[i];
    }
    (void)hipFree(dmem);
    if (d_chain) (void)hipFree(d_chain);
    if (rc != HCLIB_HIP_OK) return rc;
    result->nodes = gl.counters[0];
    result->leaves = gl.counters[1];
    result->max_depth = gl.maxes[0];
    result->batches = gl.counters[kCtrBatches];
    result->chunks_pushed = gl.counters[kCtrPushed];
    result->chunks_stolen = gl.counters[kCtrStolen];
    result->kernel_ms = ms;
    const double busy = (double)gl.counters[kCtrBusyCycles],
                 idle = (double)gl.counters[kCtrIdleCycles];
    result->busy_frac = (busy + idle) > 0 ? busy / (busy + idle) : 0.0;
    // s_memtime ticks at the shader clock, calibrated against the 100 MHz
    // s_memrealtime over the same wave lifetimes
    const double mhz = gl.counters[kCtrRealTicks]
                           ? 100.0 * (double)gl.counters[kCtrClockTicks] / (double)gl.counters[kCtrRealTicks]
                           : 2400.0;
    result->us_per_batch = gl.counters[kCtrBatches] ? busy / gl.counters[kCtrBatches] / mhz : 0.0;
    return HCLIB_HIP_OK;
}
