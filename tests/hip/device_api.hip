// The device side of the C++ API (include/hclib_hip_cpp.h) on MI355X:
//  * hclib::hip::forasync{1,2,3}D with __device__ lambdas, FLAT and
//    RECURSIVE: visit counts equal the reference tiling's
//    (forasync1D_flat / _recursive / _runner, src/hclib.c:110-190, 316-351),
//    restated here on the host independently of the library;
//  * hclib::hip::run_tasks<Kind> with two user-defined task kinds compiled
//    in this file: the fib call tree of test/fib/fib.c (fib(n) = sum of the
//    leaf values, 2*fib(n+1)-1 tasks) and N-Queens (solutions and partial
//    placements checked against a serial host search).
// Prints "Check results: OK" (tests/test_device_api.py).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hclib_hip_cpp.h"

#define CHECK(c, ...)                                        \
    do {                                                     \
        if (!(c)) {                                          \
            fprintf(stderr, "FAILED %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                    \
            fprintf(stderr, "\n");                           \
            exit(1);                                         \
        }                                                    \
    } while (0)

// ------------------------------------------------ reference tiling (host)
static void ref_runner(int low, int high, int stride, std::vector<int> &cnt) {
    for (int i = low; i < high; i += stride) cnt[i]++;
}
static void ref_recursive(int low, int high, int stride, int tile, std::vector<int> &cnt) {
    if ((high - low) > tile) {
        int mid = (high + low) / 2;
        ref_recursive(mid, high, stride, tile, cnt);
        ref_recursive(low, mid, stride, tile, cnt);
    } else {
        ref_runner(low, high, stride, cnt);
    }
}
static void ref_flat1d(int low, int high, int stride, int tile, std::vector<int> &cnt) {
    int nb_chunks = high / tile, size = tile * nb_chunks, low0;
    for (low0 = low; low0 < size; low0 += tile) ref_runner(low0, low0 + tile, stride, cnt);
    if (size < high) ref_runner(low0, high, stride, cnt);
}

static void check_forasync1d(int low, int high, int tile, int stride, int mode) {
    const int ext = high + tile + 64;
    std::vector<int> want(ext, 0), got(ext, 0);
    if (mode == FORASYNC_MODE_RECURSIVE) ref_recursive(low, high, stride, tile, want);
    else ref_flat1d(low, high, stride, tile, want);
    int *d = nullptr;
    CHECK(hipMalloc((void **)&d, ext * sizeof(int)) == hipSuccess, "hipMalloc");
    CHECK(hipMemset(d, 0, ext * sizeof(int)) == hipSuccess, "hipMemset");
    hclib::loop_domain_1d dom(low, high, 1, stride);
    dom.get_internal()->tile = tile;
    int rc = hclib::hip::forasync1D(&dom, [=] __device__(int i) { atomicAdd(&d[i], 1); }, mode);
    CHECK(rc == HCLIB_HIP_OK, "forasync1D: %s", hclib_hip_last_error());
    CHECK(hipMemcpy(got.data(), d, ext * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess, "copy");
    (void)hipFree(d);
    CHECK(got == want, "forasync1D {%d,%d,%d,%d} mode %d differs from the reference tiling", low, high, stride,
          tile, mode);
}

template <int ND>
static void check_forasync_nd(int mode) {
    const int E0 = 37, E1 = 29, E2 = ND == 3 ? 11 : 1, n = E0 * E1 * E2;
    int *d = nullptr;
    CHECK(hipMalloc((void **)&d, n * sizeof(int)) == hipSuccess, "hipMalloc");
    CHECK(hipMemset(d, 0, n * sizeof(int)) == hipSuccess, "hipMemset");
    int rc;
    if (ND == 2) {
        hclib::loop_domain_2d dom(E0, E1);
        dom.get_internal()[0].tile = 5;
        dom.get_internal()[1].tile = 8;
        rc = hclib::hip::forasync2D(&dom, [=] __device__(int i, int j) { atomicAdd(&d[i * E1 + j], 1); }, mode);
    } else {
        hclib::loop_domain_3d dom(0, E0, 6, 0, E1, 4, 0, E2, 3);
        rc = hclib::hip::forasync3D(&dom, [=] __device__(int i, int j, int k) {
            atomicAdd(&d[(i * E1 + j) * E2 + k], 1);
        }, mode);
    }
    CHECK(rc == HCLIB_HIP_OK, "forasync%dD: %s", ND, hclib_hip_last_error());
    std::vector<int> got(n);
    CHECK(hipMemcpy(got.data(), d, n * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess, "copy");
    (void)hipFree(d);
    for (int i = 0; i < n; ++i) CHECK(got[i] == 1, "forasync%dD index %d visited %d times", ND, i, got[i]);
}

// ------------------------------------------------------ fib as a kind
// template {m}: child k is fib(m-1-k) (test/fib/fib.c:57-71); a leaf adds n
struct FibCountCtx {
    int n;
};
struct FibCountKind {
    static constexpr int kTmplWords = 2;
    static constexpr int kWords = 4;
    static constexpr bool kPure = true;
    static constexpr bool kBoundedChildren = true;
    using Ctx = FibCountCtx;
    struct Acc {
        uint32_t tasks = 0, sum = 0;
        __device__ void flush(hx::SchedGlobals *g) {
            const unsigned long long t = hx::wave_sum((unsigned long long)tasks),
                                     s = hx::wave_sum((unsigned long long)sum);
            if (hx::lane_id() == 0) {
                hx::add_agent(&g->counters[0], t);
                hx::add_agent(&g->counters[1], s);
            }
        }
    };
    __device__ static int roots(const Ctx &c, Acc &, uint32_t *t) {
        t[0] = (uint32_t)c.n + 1;
        t[1] = 0;
        return 1;
    }
    __device__ static int process(const Ctx &, Acc &acc, const uint32_t *t, uint32_t k, uint32_t *child,
                                  uint32_t *, bool valid) {
        const int m = (int)t[0] - 1 - (int)k;
        acc.tasks += valid ? 1u : 0u;
        if (m < 2) {
            acc.sum += valid ? (uint32_t)m : 0u;
            return 0;
        }
        child[0] = (uint32_t)m;
        child[1] = 0;
        return valid ? 2 : 0;
    }
};

// ---------------------------------------------------- N-Queens as a kind
// template {cols, left diagonals, right diagonals, row, -, -}; child k puts
// the row's queen in column k (bitmask formulation)
struct QueensCtx {
    int n;
};
struct QueensKind {
    static constexpr int kTmplWords = 6;
    static constexpr int kWords = 8;
    static constexpr bool kPure = true;
    static constexpr bool kBoundedChildren = true;
    using Ctx = QueensCtx;
    struct Acc {
        uint32_t sols = 0, nodes = 0;
        __device__ void flush(hx::SchedGlobals *g) {
            const unsigned long long s = hx::wave_sum((unsigned long long)sols),
                                     n = hx::wave_sum((unsigned long long)nodes);
            if (hx::lane_id() == 0) {
                hx::add_agent(&g->counters[0], s);
                hx::add_agent(&g->counters[1], n);
            }
        }
    };
    __device__ static int roots(const Ctx &c, Acc &, uint32_t *t) {
        for (int i = 0; i < 6; ++i) t[i] = 0;
        return c.n;
    }
    __device__ static int process(const Ctx &c, Acc &acc, const uint32_t *t, uint32_t k, uint32_t *child,
                                  uint32_t *, bool valid) {
        const uint32_t mask = (1u << c.n) - 1u, bit = 1u << k;
        const bool ok = valid && !((t[0] | t[1] | t[2]) & bit);
        acc.nodes += ok ? 1u : 0u;
        const bool last = t[3] + 1 == (uint32_t)c.n;
        acc.sols += (ok && last) ? 1u : 0u;
        child[0] = t[0] | bit;
        child[1] = ((t[1] | bit) << 1) & mask;
        child[2] = (t[2] | bit) >> 1;
        child[3] = t[3] + 1;
        child[4] = 0;
        child[5] = 0;
        return (ok && !last) ? c.n : 0;
    }
};

// ------------------------------------------- worker identity in a kind
// UTS.cpp:104-106,220-221 keep per-worker state indexed by
// hclib_get_current_worker(): here every task adds itself to its worker's
// tally (hx::current_worker(), one wave = one worker)
struct WorkerCtx {
    int n;
    unsigned int *tally;  // [num_workers]
    unsigned int *bad;    // ids outside [0, num_workers)
};
struct WorkerKind {
    static constexpr int kTmplWords = 2;
    static constexpr int kWords = 4;
    static constexpr bool kPure = false;  // the tallies are side effects
    static constexpr bool kBoundedChildren = true;
    using Ctx = WorkerCtx;
    struct Acc {
        __device__ void flush(hx::SchedGlobals *) {}
    };
    __device__ static int roots(const Ctx &c, Acc &, uint32_t *t) {
        t[0] = (uint32_t)c.n + 1;
        t[1] = 0;
        return 1;
    }
    __device__ static int process(const Ctx &c, Acc &, const uint32_t *t, uint32_t k, uint32_t *child, uint32_t *,
                                  bool) {
        const int w = hx::current_worker(), nw = hx::num_workers();
        if (w < 0 || w >= nw) atomicAdd(c.bad, 1u);
        else atomicAdd(&c.tally[w], 1u);
        const int m = (int)t[0] - 1 - (int)k;
        if (m < 2) return 0;
        child[0] = (uint32_t)m;
        child[1] = 0;
        return 2;
    }
};

static void host_queens(int n, int row, uint32_t cols, uint32_t ld, uint32_t rd, unsigned long long &sols,
                        unsigned long long &nodes) {
    const uint32_t mask = (1u << n) - 1u;
    for (int k = 0; k < n; ++k) {
        const uint32_t bit = 1u << k;
        if ((cols | ld | rd) & bit) continue;
        nodes++;
        if (row + 1 == n) sols++;
        else host_queens(n, row + 1, cols | bit, ((ld | bit) << 1) & mask, (rd | bit) >> 1, sols, nodes);
    }
}

int main() {
    CHECK(hclib_hip_init(0) == HCLIB_HIP_OK, "hclib_hip_init: %s", hclib_hip_last_error());
    // device forasync: the reference's iteration sets, including the FLAT
    // low != 0 overrun ({10, 100, 1, 33} runs 10..108)
    const int c1[][4] = {{0, 1000, 33, 1}, {10, 100, 33, 1}, {5, 777, 60, 3}, {0, 1 << 20, 1024, 1},
                         {0, 1, 4, 1},     {3, 4099, 1, 7}};
    for (auto &c : c1)
        for (int mode : {FORASYNC_MODE_FLAT, FORASYNC_MODE_RECURSIVE}) check_forasync1d(c[0], c[1], c[2], c[3], mode);
    for (int mode : {FORASYNC_MODE_FLAT, FORASYNC_MODE_RECURSIVE}) {
        check_forasync_nd<2>(mode);
        check_forasync_nd<3>(mode);
    }
    printf("device forasync 1-D/2-D/3-D FLAT/RECURSIVE: reference iteration sets\n");

    // fib(n) through a user kind
    for (int n : {0, 1, 2, 10, 25}) {
        hclib::hip::task_stats st;
        int rc = hclib::hip::run_tasks<FibCountKind>(FibCountCtx{n}, &st);
        CHECK(rc == HCLIB_HIP_OK, "run_tasks<FibCountKind>: %s", hclib_hip_last_error());
        unsigned long long a = 0, b = 1;
        for (int i = 0; i < n; ++i) {
            unsigned long long t = a + b;
            a = b;
            b = t;
        }
        // fib(n) = a; tasks = 2 * fib(n + 1) - 1
        CHECK(st.counters[1] == a, "fib(%d) = %llu, want %llu", n, (unsigned long long)st.counters[1], a);
        CHECK(st.counters[0] == 2 * b - 1, "fib(%d) tasks %llu, want %llu", n,
              (unsigned long long)st.counters[0], 2 * b - 1);
        printf("fib(%d) = %llu in %llu device tasks (%.3f ms)\n", n, a, (unsigned long long)st.counters[0],
               st.kernel_ms);
    }
    // N-Queens through a user kind (n <= 8: uniform pushes; n > 8: split ranges)
    for (int n = 1; n <= 12; ++n) {
        hclib::hip::task_stats st;
        int rc = hclib::hip::run_tasks<QueensKind>(QueensCtx{n}, &st);
        CHECK(rc == HCLIB_HIP_OK, "run_tasks<QueensKind>: %s", hclib_hip_last_error());
        unsigned long long sols = 0, nodes = 0;
        host_queens(n, 0, 0, 0, 0, sols, nodes);
        CHECK(st.counters[0] == sols && st.counters[1] == nodes, "queens(%d): %llu/%llu, want %llu/%llu", n,
              (unsigned long long)st.counters[0], (unsigned long long)st.counters[1], sols, nodes);
        if (n >= 10) printf("queens(%d) = %llu solutions, %llu placements (%.3f ms)\n", n, sols, nodes, st.kernel_ms);
    }
    // worker identity: every task tallied under a valid worker id, spread
    // over many workers (fib(24): 150,049 tasks)
    {
        const int nw = hclib_hip_num_workers();
        unsigned int *d = nullptr;
        CHECK(nw > 0 && hipMalloc((void **)&d, (size_t)(nw + 1) * 4) == hipSuccess &&
                  hipMemset(d, 0, (size_t)(nw + 1) * 4) == hipSuccess,
              "tally buffer");
        hclib::hip::task_config tc;
        tc.spill_lo = 32;
        hclib::hip::task_stats st;
        int rc = hclib::hip::run_tasks<WorkerKind>(WorkerCtx{24, d, d + nw}, &st, tc);
        CHECK(rc == HCLIB_HIP_OK, "run_tasks<WorkerKind>: %s", hclib_hip_last_error());
        std::vector<unsigned int> h((size_t)nw + 1);
        CHECK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) == hipSuccess, "copy tally");
        unsigned long long total = 0;
        int used = 0;
        for (int w = 0; w < nw; ++w) {
            total += h[w];
            used += h[w] ? 1 : 0;
        }
        CHECK(h[nw] == 0, "%u tasks saw a worker id outside [0, %d)", h[nw], nw);
        CHECK(total == 2 * 75025ull - 1, "tallied %llu tasks, want %llu", total, 2 * 75025ull - 1);
        CHECK(used > 1, "only %d worker(s) ran tasks", used);
        printf("worker identity: %llu tasks on %d of %d device workers\n", total, used, nw);
        (void)hipFree(d);
    }
    printf("Check results: OK\n");
    return 0;
}
