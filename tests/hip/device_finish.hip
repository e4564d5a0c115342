// Nested finish inside device tasks (include/hclib_hip/hx_finish.h) through
// hclib::hip::run_tasks with task kinds defined in this file:
//
//  * FibFinishKind — test/fib/fib.c:57-71 as the reference writes it:
//      fib(n) { if (n < 2) return n; FINISH { async fib(n-1); async fib(n-2); }
//               return lhs + rhs; }
//    every call a task, every FINISH a scope, `lhs + rhs` the continuation
//    run by the last child out. fib(0..27) against fib_iter (fib.c:38-46),
//    2 fib(n+1) - 1 tasks and fib(n+1) - 1 continuations.
//
//  * NestedFinishKind — test/cpp/nested_finish.cpp: 100 iterations of
//      async { finish { async { finish { async { finish { async { finish {
//        async { leaf } } } } } } } } }
//    Each leaf and each continuation takes a ticket from one global
//    sequence counter; for every iteration the leaf must come before the
//    innermost continuation and each continuation before the one around it
//    (a finish ends only after everything inside it), and every level must
//    complete exactly 100 times. The iterations sit in one top-level scope
//    opened on the host (finish_arena::preopen) whose value must be 100.
//
// Prints "Check results: OK" (tests/test_device_api.py).
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "hclib_hip_cpp.h"

#define CHECK(c, ...)                                              \
    do {                                                           \
        if (!(c)) {                                                \
            fprintf(stderr, "FAILED %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                          \
            fprintf(stderr, "\n");                                 \
            exit(1);                                               \
        }                                                          \
    } while (0)

// --------------------------------------------------------------- fib
struct FibFinishCtx {
    int n;
    hx::FinishArena fin;
};

struct FibFinishKind {
    static constexpr int kTmplWords = 2;  // {n + 1 of the parent call, parent scope}
    static constexpr int kWords = 4;
    static constexpr bool kPure = false;
    static constexpr bool kBoundedChildren = true;
    using Ctx = FibFinishCtx;
    struct Acc {
        unsigned long long tasks = 0, conts = 0;
        __device__ void flush(hx::SchedGlobals *g) {
            const unsigned long long t = hx::wave_sum(tasks), c = hx::wave_sum(conts);
            if (hx::lane_id() == 0) {
                hx::add_agent(&g->counters[0], t);
                hx::add_agent(&g->counters[1], c);
            }
        }
    };
    __device__ static int roots(const Ctx &c, Acc &, uint32_t *tmpl) {
        tmpl[0] = (uint32_t)c.n + 1;
        tmpl[1] = hx::kScopeRoot;
        return 1;
    }
    __device__ static int process(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k, uint32_t *child,
                                  uint32_t *err, bool) {
        acc.tasks += 1;
        const int n = (int)t[0] - 1 - (int)k;
        const uint32_t scope = hx::finish_open(c.fin, n >= 2, t[1], 2, 0, err);
        if (n < 2) {
            // return n; the continuation of every enclosing finish that this
            // check-out closes is `return lhs + rhs` (the scope's sum)
            acc.conts += hx::finish_check_out(c.fin, t[1], (unsigned long long)n,
                                              [](uint32_t, unsigned long long sum) { return sum; });
            return 0;
        }
        child[0] = (uint32_t)n;
        child[1] = scope;
        return scope == hx::kScopeRoot ? 0 : 2;
    }
};

// ------------------------------------------------------ nested finish
constexpr int kIters = 100;
constexpr int kDepth = 4;  // finishes per iteration

struct NestCtx {
    hx::FinishArena fin;
    unsigned int *seq;       // global ticket counter
    unsigned int *leaf_seq;  // [kIters]
    unsigned int *cont_seq;  // [kIters * kDepth]
    unsigned int *done;      // [kDepth] continuations per level
};

struct NestedFinishKind {
    static constexpr int kTmplWords = 2;  // {depth << 16 | iteration, parent scope}
    static constexpr int kWords = 4;
    static constexpr bool kPure = false;
    static constexpr bool kBoundedChildren = true;
    using Ctx = NestCtx;
    struct Acc {
        __device__ void flush(hx::SchedGlobals *) {}
    };
    // the launch's root: kIters iterations, each checking out of scope 0 (the
    // host-opened top-level finish of the hclib::launch body)
    __device__ static int roots(const Ctx &, Acc &, uint32_t *tmpl) {
        tmpl[0] = 0;
        tmpl[1] = 0;
        return kIters;
    }
    __device__ static int process(const Ctx &c, Acc &, const uint32_t *t, uint32_t k, uint32_t *child,
                                  uint32_t *err, bool) {
        // a root item k is iteration k at depth 0; others carry their own
        const bool top = t[0] == 0 && t[1] == 0 && k < (uint32_t)kIters;
        const uint32_t d = top ? 0u : t[0] >> 16, it = top ? k : t[0] & 0xffffu;
        const uint32_t parent = top ? 0u : t[1];
        // async { finish { async ... } }: open the finish with one task in it
        const bool opens = d < (uint32_t)kDepth;
        const uint32_t scope = hx::finish_open(c.fin, opens, parent, 1, it << 8 | d, err);
        if (opens) {
            child[0] = (d + 1) << 16 | it;
            child[1] = scope;
            return scope == hx::kScopeRoot ? 0 : 1;
        }
        // the innermost async: "Howdy from inside a finish within nested finishes"
        c.leaf_seq[it] = atomicAdd(c.seq, 1u);
        hx::finish_check_out(c.fin, parent, 1ull, [&](uint32_t cw, unsigned long long sum) {
            if (cw == hx::kScopeRoot) return sum;  // never: scope 0's cont is the top marker
            const uint32_t cd = cw & 0xffu, ci = cw >> 8;
            if (cd < (uint32_t)kDepth) {
                c.cont_seq[ci * kDepth + cd] = atomicAdd(c.seq, 1u);
                atomicAdd(&c.done[cd], 1u);
            }
            return sum;
        });
        return 0;
    }
};

static unsigned long long fib_iter(int n) {  // test/fib/fib.c:38-46
    unsigned long long a = 0, b = 1;
    for (int i = 0; i < n; ++i) {
        const unsigned long long t = a + b;
        a = b;
        b = t;
    }
    return a;
}

int main() {
    CHECK(hclib_hip_init(0) == HCLIB_HIP_OK, "hclib_hip_init: %s", hclib_hip_last_error());
    hclib::hip::task_config tc;
    tc.spill_lo = 32;
    for (int n = 0; n <= 27; ++n) {
        hclib::hip::finish_arena fin((uint32_t)fib_iter(n + 1) + 1);
        CHECK(fin.ok(), "finish_arena");
        hclib::hip::task_stats st;
        const int rc = hclib::hip::run_tasks<FibFinishKind>(FibFinishCtx{n, fin.view()}, &st, tc);
        CHECK(rc == HCLIB_HIP_OK, "run_tasks<FibFinishKind>(%d): %s", n, hclib_hip_last_error());
        const unsigned long long v = fin.root_value(), want = fib_iter(n);
        CHECK(v == want, "fib(%d) = %llu, want %llu", n, v, want);
        CHECK(st.counters[0] == 2 * fib_iter(n + 1) - 1, "fib(%d): %llu tasks", n,
              (unsigned long long)st.counters[0]);
        CHECK(st.counters[1] == fib_iter(n + 1) - 1 && fin.scopes_opened() == fib_iter(n + 1) - 1,
              "fib(%d): %llu continuations, %u scopes", n, (unsigned long long)st.counters[1], fin.scopes_opened());
        if (n == 27) printf("fib(27) = %llu: %llu tasks, %llu finish continuations (%.3f ms)\n", v,
                            (unsigned long long)st.counters[0], (unsigned long long)st.counters[1], st.kernel_ms);
    }

    // nested finish
    hclib::hip::finish_arena fin(1 + kIters * kDepth);
    CHECK(fin.ok(), "finish_arena");
    // scope 0: the launch body's finish around the kIters asyncs
    CHECK(fin.preopen({(uint32_t)kIters}, {hx::kScopeRoot}, {hx::kScopeRoot}) == HCLIB_HIP_OK, "preopen");
    unsigned int *dm = nullptr;
    const size_t words = 1 + kIters + kIters * kDepth + kDepth;
    CHECK(hipMalloc((void **)&dm, words * 4) == hipSuccess, "hipMalloc");
    CHECK(hipMemset(dm, 0, words * 4) == hipSuccess, "hipMemset");
    NestCtx nc{fin.view(), dm, dm + 1, dm + 1 + kIters, dm + 1 + kIters + kIters * kDepth};
    hclib::hip::task_stats st;
    const int rc = hclib::hip::run_tasks<NestedFinishKind>(nc, &st, tc);
    CHECK(rc == HCLIB_HIP_OK, "run_tasks<NestedFinishKind>: %s", hclib_hip_last_error());
    std::vector<unsigned int> h(words);
    CHECK(hipMemcpy(h.data(), dm, words * 4, hipMemcpyDeviceToHost) == hipSuccess, "copy");
    const unsigned int *leaf = &h[1], *cont = &h[1 + kIters], *done = &h[1 + kIters + kIters * kDepth];
    CHECK(h[0] == kIters * (1 + kDepth), "%u tickets", h[0]);
    for (int d = 0; d < kDepth; ++d) CHECK(done[d] == (unsigned)kIters, "level %d: %u continuations", d, done[d]);
    for (int i = 0; i < kIters; ++i) {
        CHECK(leaf[i] < cont[i * kDepth + kDepth - 1], "iteration %d: innermost finish ended before its async", i);
        for (int d = kDepth - 1; d > 0; --d)
            CHECK(cont[i * kDepth + d] < cont[i * kDepth + d - 1], "iteration %d: finish %d ended before finish %d",
                  i, d - 1, d);
    }
    CHECK(fin.root_value() == (uint64_t)kIters, "top-level scope value %llu", (unsigned long long)fin.root_value());
    CHECK(fin.scopes_opened() == 1 + kIters * kDepth, "%u scopes", fin.scopes_opened());
    printf("nested finish: %d iterations x %d nested finishes, every finish after its inner tasks\n", kIters, kDepth);
    (void)hipFree(dm);
    printf("Check results: OK\n");
    return 0;
}
