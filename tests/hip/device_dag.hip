// Device promises / futures (include/hclib_hip/hx_dag.h through
// hclib::hip::dag + run_dag) on MI355X, checked against serial host
// evaluations of the same graphs:
//  * chain      — task i awaits promise i and puts i+1 (test/c/promise/
//                 asyncAwait1.c's chain, 20,000 long);
//  * wavefront  — a 192 x 192 grid, each cell awaiting its left, up and
//                 diagonal promises like a Smith-Waterman tile
//                 (test/smithwaterman/smith_waterman.cpp:174-229), boundary
//                 promises put before the launch (:141-165); the body also
//                 reads its left neighbour's PLAIN store, so the put's release
//                 and the taker's acquire are exercised for ordinary data;
//  * random     — 40,000 tasks awaiting 0..8 earlier promises each (more
//                 than MAX_NUM_WAITS = 4, duplicates allowed);
//  * fan-out    — one promise awaited by 30,000 tasks (lane-parallel release);
//  * errors     — a second put on a promise (the reference's single-
//                 assignment HASSERT, src/hclib-promise.c:206-207) and a task
//                 whose promise nothing puts (end_finish deadlock) both come
//                 back as HCLIB_HIP_EDEVICE, without hanging.
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

typedef unsigned long long u64;

__host__ __device__ inline u64 mix(u64 x) {  // splitmix64 finaliser
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__device__ inline u64 wave_xor(u64 v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v ^= __shfl_xor(v, d, 64);
    return v;
}

// ------------------------------------------------------------- chain
struct ChainKind {
    struct Ctx {
        int dummy;
    };
    __device__ static void run(const Ctx &, hx::DagWave &w, uint32_t t, const uint32_t *) {
        const u64 d = hx::dag_get(w, t);
        hx::dag_put(w, t + 1, d * 6364136223846793005ull + 1442695040888963407ull + t);
    }
};

// --------------------------------------------------------- wavefront
struct GridKind {
    struct Ctx {
        u64 *out;  // (G+1) x (G+1) plain copies of every cell value
        int G;
        unsigned *bad;
    };
    __device__ static void run(const Ctx &c, hx::DagWave &w, uint32_t t, const uint32_t *pl) {
        const int i = (int)pl[0], j = (int)pl[1], W = c.G + 1;
        const u64 up = hx::dag_get(w, (uint32_t)((i - 1) * W + j));
        const u64 dg = hx::dag_get(w, (uint32_t)((i - 1) * W + j - 1));
        const u64 left = c.out[i * W + j - 1];  // plain load of a plain store
        if (hx::lane_id() == 0 && left != hx::dag_get(w, (uint32_t)(i * W + j - 1))) atomicAdd(c.bad, 1u);
        const u64 lane = (u64)hx::lane_id();
        const u64 r = wave_xor(mix(up + lane) ^ mix(left * (lane + 1)) ^ mix(dg - lane));
        if (hx::lane_id() == 0) c.out[i * W + j] = r;
        hx::dag_put(w, (uint32_t)(i * W + j), r);
    }
};

static u64 grid_cell(u64 up, u64 left, u64 dg) {
    u64 r = 0;
    for (u64 lane = 0; lane < 64; ++lane) r ^= mix(up + lane) ^ mix(left * (lane + 1)) ^ mix(dg - lane);
    return r;
}

// ------------------------------------------------------------ random
constexpr int kRandMax = 8;
struct RandKind {
    struct Ctx {
        int dummy;
    };
    // payload: {t, k, p0..p7}
    __device__ static void run(const Ctx &, hx::DagWave &w, uint32_t t, const uint32_t *pl) {
        const int k = (int)pl[1], lane = hx::lane_id();
        u64 v = lane < k ? hx::dag_get(w, pl[2 + lane]) : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        hx::dag_put(w, t, mix(v + 0x1234567ull * t));
    }
};

// ----------------------------------------------------------- fan-out
struct FanKind {
    struct Ctx {
        int dummy;
    };
    __device__ static void run(const Ctx &, hx::DagWave &w, uint32_t t, const uint32_t *) {
        if (t == 0) hx::dag_put(w, 0, 12345);
        else hx::dag_put(w, t, hx::dag_get(w, 0) + 7ull * t);
    }
};

// ------------------------------------------------------------ errors
struct DoublePutKind {
    struct Ctx {
        int dummy;
    };
    __device__ static void run(const Ctx &, hx::DagWave &w, uint32_t t, const uint32_t *) { hx::dag_put(w, 0, t); }
};

// ----------------------------------- workgroup tasks with reserved slots
// A tagged, reserving Kind (hx_dag.h kTagged / kReserve) on run_dag_group:
// outputs are tagged words {1 << 32 | value} its readers poll, the put is
// split around the body and takes one ready slot per waiter entry. Task 0's
// promise has `fan` (> 64) waiters: the reserved put's long-list form.
struct ReserveKind {
    static constexpr int kPutN = 1;
    static constexpr bool kSc1Payload = true;
    static constexpr bool kTagged = true;
    static constexpr bool kReserve = true;
    struct Ctx {
        u64 *out;     // tagged output word per task
        int dbl;      // 1: task 1 also puts promise 0 (a second put)
        unsigned *bad;
    };
    __device__ static u64 wait_tag(const u64 *p) {
        u64 v = 0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (((v = hx::ld_agent(p)) >> 32) == 0 && __builtin_amdgcn_s_memrealtime() - t0 < 100000000ull)
            __builtin_amdgcn_s_sleep(1);
        return v;
    }
    __device__ static bool run_group(const Ctx &c, uint32_t t, const uint32_t *pl, int wave) {
        if (wave != 0) return true;
        // payload: {value source task or ~0}
        u64 v = 12345;
        if (pl[0] != 0xffffffffu) {
            const u64 in = wait_tag(&c.out[pl[0]]);
            if ((in >> 32) == 0 && hx::lane_id() == 0) atomicAdd(c.bad, 1u);
            v = (u64)(uint32_t)in + 7ull * t;
        }
        if (hx::lane_id() == 0) hx::st_agent(&c.out[t], (1ull << 32) | (uint32_t)v);
        return true;
    }
    __device__ static void promises(const Ctx &c, uint32_t t, uint32_t (&p)[1]) { p[0] = (c.dbl && t == 1) ? 0 : t; }
    __device__ static void datums(const Ctx &, uint32_t t, unsigned long long (&d)[1]) { d[0] = t; }
};

static void report(const char *what, const hclib_hip_dag_stats_t &st) {
    printf("%-10s %8llu tasks %8llu puts %8llu releases  %8.3f ms  %.1f M tasks/s\n", what,
           (unsigned long long)st.tasks, (unsigned long long)st.puts, (unsigned long long)st.releases, st.kernel_ms,
           st.tasks / (st.kernel_ms * 1e3));
}

int main() {
    CHECK(hclib_hip_init(0) == HCLIB_HIP_OK, "hclib_hip_init: %s", hclib_hip_last_error());
    {  // chain
        const uint32_t N = 20000;
        hclib::hip::dag g(1);
        for (uint32_t p = 0; p <= N; ++p) g.promise();
        g.put(0, 99);
        for (uint32_t i = 0; i < N; ++i) g.async_await(&i, {i});
        hclib_hip_dag_stats_t st;
        int rc = hclib::hip::run_dag<ChainKind>(ChainKind::Ctx{0}, g, &st);
        CHECK(rc == HCLIB_HIP_OK, "chain: %s", hclib_hip_last_error());
        u64 d = 99;
        for (uint32_t i = 0; i < N; ++i) {
            d = d * 6364136223846793005ull + 1442695040888963407ull + i;
            CHECK(g.satisfied(i + 1) && g.datum(i + 1) == d, "chain: promise %u", i + 1);
        }
        CHECK(st.tasks == N && st.puts == N && st.releases == N - 1, "chain stats");
        report("chain", st);
    }
    {  // wavefront
        const int G = 192, W = G + 1;
        hclib::hip::dag g(2);
        std::vector<u64> want((size_t)W * W);
        for (int p = 0; p < W * W; ++p) g.promise();
        for (int k = 0; k < W; ++k) {  // boundary row / column, put before the launch
            want[k] = mix(1000 + k);
            want[(size_t)k * W] = mix(5000 + k);
            g.put(k, want[k]);
            g.put(k * W, want[(size_t)k * W]);
        }
        for (int i = 1; i <= G; ++i)
            for (int j = 1; j <= G; ++j) {
                const uint32_t pl[2] = {(uint32_t)i, (uint32_t)j};
                g.async_await(pl, {(uint32_t)((i - 1) * W + j - 1), (uint32_t)((i - 1) * W + j),
                                   (uint32_t)(i * W + j - 1)});
                want[(size_t)i * W + j] =
                    grid_cell(want[(size_t)(i - 1) * W + j], want[(size_t)i * W + j - 1], want[(size_t)(i - 1) * W + j - 1]);
            }
        u64 *out = nullptr;
        unsigned *bad = nullptr;
        CHECK(hipMalloc((void **)&out, want.size() * 8) == hipSuccess && hipMalloc((void **)&bad, 4) == hipSuccess,
              "hipMalloc");
        CHECK(hipMemcpy(out, want.data(), want.size() * 8, hipMemcpyHostToDevice) == hipSuccess, "copy");
        CHECK(hipMemset(bad, 0, 4) == hipSuccess, "memset");
        hclib_hip_dag_stats_t st;
        int rc = hclib::hip::run_dag<GridKind>(GridKind::Ctx{out, G, bad}, g, &st);
        CHECK(rc == HCLIB_HIP_OK, "wavefront: %s", hclib_hip_last_error());
        std::vector<u64> got(want.size());
        unsigned nbad = 0;
        CHECK(hipMemcpy(got.data(), out, got.size() * 8, hipMemcpyDeviceToHost) == hipSuccess, "copy back");
        CHECK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost) == hipSuccess, "copy back");
        CHECK(nbad == 0, "wavefront: %u plain loads saw a stale left value", nbad);
        for (int i = 1; i <= G; ++i)
            for (int j = 1; j <= G; ++j) {
                const size_t c = (size_t)i * W + j;
                CHECK(g.datum((uint32_t)c) == want[c] && got[c] == want[c], "wavefront: cell (%d, %d)", i, j);
            }
        CHECK(st.tasks == (u64)G * G && st.puts == (u64)G * G, "wavefront stats");
        (void)hipFree(out);
        (void)hipFree(bad);
        report("wavefront", st);
    }
    {  // random
        const uint32_t N = 40000;
        hclib::hip::dag g(2 + kRandMax);
        std::vector<u64> want(N);
        u64 s = 7;
        for (uint32_t t = 0; t < N; ++t) g.promise();
        for (uint32_t t = 0; t < N; ++t) {
            uint32_t pl[2 + kRandMax] = {t, 0};
            s = mix(s);
            const uint32_t k = t < 8 ? 0 : (uint32_t)(s % (kRandMax + 1));
            u64 sum = 0;
            for (uint32_t q = 0; q < k; ++q) {
                s = mix(s);
                const uint32_t back = 1 + (uint32_t)(s % (t < 3000 ? t : 3000));
                pl[2 + q] = (q > 0 && (s >> 40) % 7 == 0) ? pl[1 + q] : t - back;  // some duplicates
                sum += want[pl[2 + q]];
            }
            pl[1] = k;
            g.async_await(pl, pl + 2, (int)k);
            want[t] = mix(sum + 0x1234567ull * t);
        }
        hclib_hip_dag_stats_t st;
        int rc = hclib::hip::run_dag<RandKind>(RandKind::Ctx{0}, g, &st);
        CHECK(rc == HCLIB_HIP_OK, "random: %s", hclib_hip_last_error());
        for (uint32_t t = 0; t < N; ++t) CHECK(g.datum(t) == want[t], "random: promise %u", t);
        CHECK(st.tasks == N && st.puts == N, "random stats");
        report("random", st);
    }
    {  // fan-out
        const uint32_t N = 30001;
        hclib::hip::dag g(0);
        for (uint32_t t = 0; t < N; ++t) g.promise();
        g.async_await(nullptr, nullptr, 0);
        for (uint32_t t = 1; t < N; ++t) g.async_await(nullptr, {0u});
        hclib_hip_dag_stats_t st;
        int rc = hclib::hip::run_dag<FanKind>(FanKind::Ctx{0}, g, &st);
        CHECK(rc == HCLIB_HIP_OK, "fan-out: %s", hclib_hip_last_error());
        for (uint32_t t = 1; t < N; ++t) CHECK(g.datum(t) == 12345ull + 7ull * t, "fan-out: promise %u", t);
        CHECK(st.releases == N - 1, "fan-out releases %llu", (unsigned long long)st.releases);
        report("fan-out", st);
    }
    {  // workgroup tasks, reserved ready slots, a 200-waiter promise and a chain
        const uint32_t fan = 200, chain = 300, N = 1 + fan + chain;
        hclib::hip::dag g(1);
        for (uint32_t t = 0; t < N; ++t) g.promise();
        const uint32_t root = 0xffffffffu;
        g.async_await(&root, nullptr, 0);
        for (uint32_t t = 1; t <= fan; ++t) {
            const uint32_t src = 0;
            g.async_await(&src, {0u});
        }
        for (uint32_t t = fan + 1; t < N; ++t) {  // each awaits the previous task (one waiter per promise)
            const uint32_t src = t - 1;
            g.async_await(&src, {t - 1});
        }
        u64 *out = nullptr;
        unsigned *bad = nullptr;
        CHECK(hipMalloc((void **)&out, N * 8) == hipSuccess && hipMalloc((void **)&bad, 4) == hipSuccess, "hipMalloc");
        CHECK(hipMemset(out, 0, N * 8) == hipSuccess && hipMemset(bad, 0, 4) == hipSuccess, "memset");
        hclib_hip_dag_stats_t st;
        for (int waves = 1; waves <= 2; ++waves) {
            CHECK(hipMemset(out, 0, N * 8) == hipSuccess, "memset");
            int rc = hclib::hip::run_dag_groups<ReserveKind>(ReserveKind::Ctx{out, 0, bad}, g, &st, 1, waves);
            CHECK(rc == HCLIB_HIP_OK, "reserved: %s", hclib_hip_last_error());
            std::vector<u64> got(N);
            unsigned nbad = 0;
            CHECK(hipMemcpy(got.data(), out, N * 8, hipMemcpyDeviceToHost) == hipSuccess, "copy back");
            CHECK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost) == hipSuccess, "copy back");
            CHECK(nbad == 0, "reserved: %u untagged inputs", nbad);
            std::vector<uint32_t> want(N);
            for (uint32_t t = 0; t < N; ++t) {
                // task t reads task pl[0]'s output: 0 for the fan, t - 1 along the chain
                want[t] = t == 0 ? 12345u : (uint32_t)(want[t <= fan ? 0 : t - 1] + 7ull * t);
                CHECK(got[t] == ((1ull << 32) | want[t]), "reserved: task %u got %llx want %x", t,
                      (unsigned long long)got[t], want[t]);
                CHECK(g.satisfied(t) && g.datum(t) == t, "reserved: promise %u", t);
            }
            CHECK(st.tasks == N && st.puts == N && st.releases == N - 1, "reserved stats %llu %llu %llu",
                  (unsigned long long)st.tasks, (unsigned long long)st.puts, (unsigned long long)st.releases);
            report(waves == 1 ? "reserved1" : "reserved2", st);
        }
        // a second put on the 200-waiter promise: found (slots past the list
        // or a satisfied count of 2), promptly, without a hang
        CHECK(hipMemset(out, 0, N * 8) == hipSuccess, "memset");
        int rc = hclib::hip::run_dag_groups<ReserveKind>(ReserveKind::Ctx{out, 1, bad}, g, &st, 1, 1, 2000);
        CHECK(rc == HCLIB_HIP_EDEVICE && strstr(hclib_hip_last_error(), "single assignment"),
              "reserved double put: rc %d (%s)", rc, hclib_hip_last_error());
        printf("reserved double put -> %s (%.3f ms)\n", hclib_hip_last_error(), st.kernel_ms);
        (void)hipFree(out);
        (void)hipFree(bad);
    }
    {  // a second put on one promise
        hclib::hip::dag g(0);
        g.promise();
        g.async_await(nullptr, nullptr, 0);
        g.async_await(nullptr, nullptr, 0);
        int rc = hclib::hip::run_dag<DoublePutKind>(DoublePutKind::Ctx{0}, g);
        CHECK(rc == HCLIB_HIP_EDEVICE && strstr(hclib_hip_last_error(), "single assignment"),
              "double put: rc %d (%s)", rc, hclib_hip_last_error());
        printf("double put -> %s\n", hclib_hip_last_error());
    }
    {  // a future nothing satisfies
        hclib::hip::dag g(0);
        g.promise();
        g.promise();
        g.async_await(nullptr, {0u});
        int rc = hclib::hip::run_dag<FanKind>(FanKind::Ctx{0}, g, nullptr, 1, 200);
        CHECK(rc == HCLIB_HIP_EDEVICE && strstr(hclib_hip_last_error(), "deadlock"), "deadlock: rc %d (%s)", rc,
              hclib_hip_last_error());
        printf("unsatisfied future -> %s\n", hclib_hip_last_error());
    }
    printf("Check results: OK\n");
    return 0;
}
