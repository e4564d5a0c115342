// Dynamic device dataflow (include/hclib_hip/hx_dyn.h) through
// hclib::hip::run_dyn, with task kinds defined in this file:
//
//  * fib with data-driven tasks — test/fib/fib.c:113-141 as the reference
//    writes it: fib(n, res) puts n, or creates two promises, asyncs fib(n-1)
//    and fib(n-2) into them and async_awaits a sum task on both that puts
//    their sum into res. Every task, promise and await is created on the
//    device while the launch runs. fib(0..22) against fib_iter, with the
//    task / promise / put counts the program implies.
//
//  * the Smith-Waterman tile program of smith_waterman.cpp:171-232: a root
//    task creates the three promises of every tile (right column, bottom
//    row, bottom-right corner, :177-190) and async_awaits every tile on its
//    left / up / diagonal neighbours' promises (:227-229; boundary promises,
//    which the reference puts before the loop, :141-165, are not awaited);
//    a tile computes its cells from its neighbours' published rows and puts
//    its three promises (:212-226). Random sequences on 12 x 9 tiles of
//    64 x 64, the score against a serial host DP.
//
//  * the errors: a second put on a promise (single assignment) and a task
//    that awaits a promise nothing puts (deadlock) return HCLIB_HIP_EDEVICE.
//
// Prints "Check results: OK" (tests/test_device_api.py).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

using hx::DynWave;
using hx::kDynOpen;

// ------------------------------------------------------------------ fib
enum : uint32_t { kMain = 0, kFib = 1, kSum = 2 };

struct FibCtx {
    int n;
};

struct FibDdtKind {
    using Ctx = FibCtx;
    static constexpr bool kSc1Payload = true;
    // payload: {kind, a, b, c}: main {n}, fib {n, res}, sum {p1, p2, res}
    __device__ static void run(const Ctx &c, DynWave &w, uint32_t, const uint32_t *pay) {
        const uint32_t kind = pay[0];
        const int lane = hx::lane_id();
        if (kind == kMain) {  // the launch body: res = promise(); async fib(n, res)
            const uint32_t res = hx::dyn_promises(w, 1);
            const uint32_t p[4] = {kFib, (uint32_t)c.n, res, 0};
            hx::dyn_async_await<true>(w, lane == 0, p, nullptr, 0);
            return;
        }
        if (kind == kFib) {
            const int n = (int)pay[1];
            const uint32_t res = pay[2];
            if (n < 2) {
                hx::dyn_put<true>(w, res, (unsigned long long)n);
                return;
            }
            const uint32_t p = hx::dyn_promises(w, 2);  // lhs, rhs
            // lanes 0, 1: fib(n-1) -> p, fib(n-2) -> p+1; lane 2: sum awaiting both
            uint32_t pl[4], fut[2] = {kDynOpen, kDynOpen};
            int nf = 0;
            if (lane == 0) {
                pl[0] = kFib, pl[1] = (uint32_t)(n - 1), pl[2] = p, pl[3] = 0;
            } else if (lane == 1) {
                pl[0] = kFib, pl[1] = (uint32_t)(n - 2), pl[2] = p + 1, pl[3] = 0;
            } else {
                pl[0] = kSum, pl[1] = p, pl[2] = p + 1, pl[3] = res;
                fut[0] = p, fut[1] = p + 1, nf = 2;
            }
            hx::dyn_async_await<true>(w, lane < 3, pl, fut, nf);
            return;
        }
        // sum: both futures are satisfied
        const unsigned long long v = hx::dyn_get(w, pay[1]) + hx::dyn_get(w, pay[2]);
        hx::dyn_put<true>(w, pay[3], v);
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

// ------------------------------------------------------------------- SW
constexpr int kT = 64;  // tile width = height

// alignment_score_matrix (smith_waterman.cpp:36-43) for codes 1..4
__host__ __device__ inline int sw_score(int a, int b) {
    return a == b ? 4 : ((a + b) % 2 == 1 ? -2 : 0);  // A-C, A-T, C-G, G-T: -2; A-G, C-T: 0
}

struct SwCtx {
    const int8_t *s1, *s2;  // coded 1..4
    int ntw, nth;
    int *bottom;  // [tiles][kT] H of each tile's bottom row
    int *right;   // [tiles][kT] H of each tile's right column
};

struct SwDynKind {
    using Ctx = SwCtx;
    static constexpr bool kSc1Payload = true;
    // payload: {kind, tile}; kind 0: the root, 1: a tile
    __device__ static void run(const Ctx &c, DynWave &w, uint32_t, const uint32_t *pay) {
        const int lane = hx::lane_id();
        const uint32_t nt = (uint32_t)(c.ntw * c.nth);
        if (pay[0] == 0) {
            // the tile program: three promises per tile, then one async_await per tile
            const uint32_t base = hx::dyn_promises(w, 3 * nt);
            for (uint32_t t0 = 0; t0 < nt; t0 += 64) {
                const uint32_t t = t0 + (uint32_t)lane;
                const int i = (int)(t / (uint32_t)c.ntw), j = (int)(t % (uint32_t)c.ntw);
                uint32_t fut[3] = {kDynOpen, kDynOpen, kDynOpen};
                if (j > 0) fut[0] = base + 3 * (t - 1) + 0;                            // left's right column
                if (i > 0) fut[1] = base + 3 * (t - (uint32_t)c.ntw) + 1;              // up's bottom row
                if (i > 0 && j > 0) fut[2] = base + 3 * (t - (uint32_t)c.ntw - 1) + 2;  // diagonal's corner
                const uint32_t pl[2] = {1u, t};
                hx::dyn_async_await<true>(w, t < nt, pl, fut, 3);
            }
            return;
        }
        const uint32_t t = pay[1];
        const int i = (int)(t / (uint32_t)c.ntw), j = (int)(t % (uint32_t)c.ntw);
        const int R0 = i * kT, C0 = j * kT;  // matrix index of the row / column above / left of the tile
        // inputs: H(R0 + r, C0) for this lane's row, H(R0, C0 + q) for the top
        // row, H(R0, C0) the corner (boundaries: H(r, 0) = -r, H(0, q) = -q)
        const int row = R0 + lane + 1;
        const int left0 = j == 0 ? -row : hx::ld_agent(&c.right[(size_t)(t - 1) * kT + lane]);
        const int corner = (i == 0) ? -C0 : (j == 0 ? -R0 : (int)hx::dyn_get(w, 3 * (t - (uint32_t)c.ntw - 1) + 2));
        const int a = c.s2[row - 1];
        // lane r computes column q = s - r at step s: the cell above is lane
        // r-1's value from step s-1 (lane 0: the top row), the diagonal the
        // value above one column back (first column: the left column one row
        // up, lane 0: the corner)
        const int left_up = __shfl_up(left0, 1, 64);
        int left = left0, up_prev = lane == 0 ? corner : left_up, out = left0;
        for (int s = 0; s < kT + 63; ++s) {
            const int from_up = __shfl_up(out, 1, 64);
            const int q = s - lane;
            if (q < 0 || q >= kT) continue;
            int up = from_up;
            if (lane == 0)
                up = i == 0 ? -(C0 + q + 1) : hx::ld_agent(&c.bottom[(size_t)(t - (uint32_t)c.ntw) * kT + q]);
            const int sc = sw_score(a, c.s1[C0 + q]);
            int v = left - 1;
            v = v > up - 1 ? v : up - 1;
            v = v > up_prev + sc ? v : up_prev + sc;
            left = v;
            out = v;
            up_prev = up;
            if (lane == 63) hx::st_agent(&c.bottom[(size_t)t * kT + q], v);
        }
        const int h = left;
        hx::st_agent(&c.right[(size_t)t * kT + lane], h);
        const int last = __shfl(h, 63, 64);
        // right column, bottom row, corner (:212-226)
        hx::dyn_put<true>(w, 3 * t + 0, 0ull);
        hx::dyn_put<true>(w, 3 * t + 1, 0ull);
        hx::dyn_put<true>(w, 3 * t + 2, (unsigned long long)(uint32_t)last);
    }
};

static int sw_host(const std::vector<int8_t> &s1, const std::vector<int8_t> &s2) {
    const size_t n = s1.size(), m = s2.size();
    std::vector<int> prev(n + 1), cur(n + 1);
    for (size_t q = 0; q <= n; ++q) prev[q] = -(int)q;
    for (size_t r = 1; r <= m; ++r) {
        cur[0] = -(int)r;
        for (size_t q = 1; q <= n; ++q) {
            int v = prev[q - 1] + sw_score(s2[r - 1], s1[q - 1]);
            v = v > prev[q] - 1 ? v : prev[q] - 1;
            v = v > cur[q - 1] - 1 ? v : cur[q - 1] - 1;
            cur[q] = v;
        }
        std::swap(prev, cur);
    }
    return prev[n];
}

// -------------------------------------------------------------- errors
struct BadKind {
    using Ctx = int;  // 0: double put, 1: await a promise nothing puts
    static constexpr bool kSc1Payload = true;
    __device__ static void run(const Ctx &mode, DynWave &w, uint32_t, const uint32_t *pay) {
        if (pay[0] != 0) return;  // the stuck task (never runs)
        const uint32_t p = hx::dyn_promises(w, 2);
        if (mode == 0) {
            hx::dyn_put<true>(w, p, 1ull);
            hx::dyn_put<true>(w, p, 2ull);
        } else {
            const uint32_t pl[1] = {1u}, fut[1] = {p + 1};
            hx::dyn_async_await<true>(w, hx::lane_id() == 0, pl, fut, 1);
        }
    }
};

int main() {
    CHECK(hclib_hip_init(0) == HCLIB_HIP_OK, "hclib_hip_init: %s", hclib_hip_last_error());
    hclib::hip::dyn_caps caps;
    caps.tasks = 200000;
    caps.promises = 200000;
    caps.wait_nodes = 200000;
    for (int n = 0; n <= 22; ++n) {
        hclib_hip_dyn_stats_t st;
        const int rc = hclib::hip::run_dyn<FibDdtKind>(FibCtx{n}, 4, {kMain, 0, 0, 0}, caps, &st);
        CHECK(rc == HCLIB_HIP_OK, "run_dyn<FibDdtKind>(%d): %s", n, hclib_hip_last_error());
        const std::vector<uint64_t> res = hclib::hip::dyn_datum(0, 1);
        CHECK(!res.empty() && res[0] == fib_iter(n), "fib(%d) = %llu, want %llu", n,
              res.empty() ? 0ull : (unsigned long long)res[0], fib_iter(n));
        // fib calls: 2 fib(n+1) - 1; each inner call (fib(n+1) - 1 of them)
        // creates 2 promises and one sum task
        const unsigned long long calls = 2 * fib_iter(n + 1) - 1, inner = fib_iter(n + 1) - 1;
        CHECK(st.tasks == 1 + calls + inner && st.created == calls + inner, "fib(%d): %llu tasks run, %llu created", n,
              (unsigned long long)st.tasks, (unsigned long long)st.created);
        CHECK(st.promises == 1 + 2 * inner && st.puts == 1 + 2 * inner, "fib(%d): %llu promises, %llu puts", n,
              (unsigned long long)st.promises, (unsigned long long)st.puts);
        if (n == 22)
            printf("fib(22) = %llu with data-driven device tasks: %llu tasks, %llu promises (%.3f ms)\n",
                   (unsigned long long)res[0], (unsigned long long)st.tasks, (unsigned long long)st.promises,
                   st.kernel_ms);
    }

    // Smith-Waterman tile program
    const int ntw = 12, nth = 9;
    std::vector<int8_t> s1(ntw * kT), s2(nth * kT);
    srand(7);
    for (auto &x : s1) x = (int8_t)(1 + rand() % 4);
    for (auto &x : s2) x = (int8_t)(1 + rand() % 4);
    int8_t *d1 = nullptr, *d2 = nullptr;
    int *dbot = nullptr, *dright = nullptr;
    const int nt = ntw * nth;
    CHECK(hipMalloc((void **)&d1, s1.size()) == hipSuccess && hipMalloc((void **)&d2, s2.size()) == hipSuccess &&
              hipMalloc((void **)&dbot, (size_t)nt * kT * 4) == hipSuccess &&
              hipMalloc((void **)&dright, (size_t)nt * kT * 4) == hipSuccess,
          "hipMalloc");
    CHECK(hipMemcpy(d1, s1.data(), s1.size(), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d2, s2.data(), s2.size(), hipMemcpyHostToDevice) == hipSuccess,
          "copy");
    hclib_hip_dyn_stats_t st;
    int rc = hclib::hip::run_dyn<SwDynKind>(SwCtx{d1, d2, ntw, nth, dbot, dright}, 2, {0u, 0u}, caps, &st);
    CHECK(rc == HCLIB_HIP_OK, "run_dyn<SwDynKind>: %s", hclib_hip_last_error());
    const std::vector<uint64_t> corner = hclib::hip::dyn_datum(3 * (nt - 1) + 2, 1);
    const int score = corner.empty() ? -1 : (int)(uint32_t)corner[0], want = sw_host(s1, s2);
    CHECK(score == want, "SW score %d, want %d", score, want);
    CHECK(st.tasks == (uint64_t)nt + 1 && st.created == (uint64_t)nt && st.puts == 3ull * nt &&
              st.promises == 3ull * nt,
          "SW: %llu tasks, %llu created, %llu puts", (unsigned long long)st.tasks, (unsigned long long)st.created,
          (unsigned long long)st.puts);
    printf("Smith-Waterman %d x %d tiles as device async_awaits: score %d (host DP %d), %llu releases (%.3f ms)\n",
           ntw, nth, score, want, (unsigned long long)st.releases, st.kernel_ms);
    (void)hipFree(d1);
    (void)hipFree(d2);
    (void)hipFree(dbot);
    (void)hipFree(dright);

    // errors
    caps.spin_limit_ms = 300;
    rc = hclib::hip::run_dyn<BadKind>(0, 1, {0u}, caps);
    CHECK(rc == HCLIB_HIP_EDEVICE && strstr(hclib_hip_last_error(), "single assignment"), "double put: %d %s", rc,
          hclib_hip_last_error());
    printf("double put: %s\n", hclib_hip_last_error());
    rc = hclib::hip::run_dyn<BadKind>(1, 1, {0u}, caps);
    CHECK(rc == HCLIB_HIP_EDEVICE && strstr(hclib_hip_last_error(), "deadlock"), "unput future: %d %s", rc,
          hclib_hip_last_error());
    printf("unput future: %s\n", hclib_hip_last_error());
    printf("Check results: OK\n");
    return 0;
}
