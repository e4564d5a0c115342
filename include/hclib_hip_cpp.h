/*
 * hclib_hip_cpp.h — the device side of HClib's C++ API on MI355X
 * (compile with hipcc --offload-arch=gfx950; link libhclib_amd.so).
 *
 * The reference's C++ layer runs lambdas on CPU workers
 * (inc/hclib-async.h:161-166, inc/hclib-forasync.h:519-530). On the GPU a
 * lambda must be device code, compiled into the caller's translation unit,
 * so the device API is templates over the caller's functors:
 *
 *   hclib::hip::forasync{1,2,3}D(loop, [=] __device__ (int i[, j[, k]]) {...}, mode)
 *       hclib::forasync{1,2,3}D with a __device__ lambda: one grid-stride
 *       launch over exactly the reference's iteration set for `mode`
 *       (include/hclib_forasync_sets.h). Blocking, like the reference's
 *       finish-wrapped forasync; the _nb forms return after enqueueing.
 *
 *   hclib::hip::dag + run_dag<Kind>(ctx, graph, &stats)
 *       hclib::promise_t / async_await for device tasks: the host declares
 *       promises and tasks (each with a payload and the futures it awaits,
 *       inc/hclib-async.h:247-355); one persistent launch runs the graph,
 *       task bodies read futures with hx::dag_get and satisfy promises with
 *       hx::dag_put, which releases waiters through dependency counters
 *       (include/hclib_hip/hx_dag.h). Blocking, like a finish around the
 *       asyncs; afterwards graph.datum(p) is each promise's value.
 *
 *   hclib::hip::finish_arena + hx::finish_open / hx::finish_check_out
 *       nested finish scopes inside device tasks (include/hclib_hip/
 *       hx_finish.h): the code after a finish is a continuation that the
 *       last task to leave the scope runs inline.
 *
 *   hclib::hip::run_tasks<Kind>(ctx, &stats)
 *       a user-defined device task kind on the persistent work-stealing
 *       megakernel (include/hclib_hip/hx_sched.h): the GPU form of
 *       `hclib::launch` + recursive `hclib::async` inside one `finish`. A
 *       task is a template of Kind::kTmplWords u32 words; running child k of
 *       a task may create one new task with n children (the Kind concept is
 *       documented at the top of hx_sched.h). The launch-wide finish is the
 *       scheduler's `outstanding` counter; run_tasks returns when it drains.
 *
 * Errors: negative HCLIB_HIP_* codes with hclib_hip_last_error(), as the
 * module C ABI (include/hclib_hip.h).
 */
#ifndef HCLIB_HIP_CPP_H_
#define HCLIB_HIP_CPP_H_

#include <hip/hip_runtime.h>

#include <initializer_list>
#include <vector>

#include "hclib_cpp.h"
#include "hclib_hip.h"
#include "hclib_hip/hx_dag.h"
#include "hclib_hip/hx_dyn.h"
#include "hclib_hip/hx_finish.h"
#include "hclib_hip/hx_sched.h"

namespace hclib {
namespace hip {

// ------------------------------------------- device loop bodies of the caller
// forasync_device(body, dim, domain, mode, stream): the reference's forasync
// iteration set (hclib_hip_forasync_plan) swept by a kernel compiled here,
// in the caller's translation unit; body(i, j, k) is a __device__ callable
// (j, k = 0 below dim 2, 3). Asynchronous on `stream`.
namespace detail {
__device__ __forceinline__ int sweep_index(const hclib_hip_sweep_plan_t &p, int d, int64_t t) {
    int lo = 0, hi = p.nruns[d] - 1;
    while (lo < hi) {  // the last run with prefix <= t
        const int mid = (lo + hi + 1) >> 1;
        if (p.prefix[d][mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    const hclib_hip_run_t r = p.runs[d][lo];
    return r.first + (int)(t - p.prefix[d][lo]) * r.stride;
}
template <class Body>
__global__ __launch_bounds__(256) void k_user_sweep(Body body, hclib_hip_sweep_plan_t p) {
    const int64_t n1 = p.ndim > 1 ? p.prefix[1][p.nruns[1]] : 1, n2 = p.ndim > 2 ? p.prefix[2][p.nruns[2]] : 1;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < p.total; t += step) {
        const int64_t t2 = t % n2, r = t / n2, t1 = r % n1, t0 = r / n1;
        body(sweep_index(p, 0, t0), p.ndim > 1 ? sweep_index(p, 1, t1) : 0, p.ndim > 2 ? sweep_index(p, 2, t2) : 0);
    }
}
}  // namespace detail

template <class Body>
int forasync_device(const Body &body, int dim, hclib_loop_domain_t *domain, int mode, void *stream) {
    static_assert(sizeof(hclib_loop_domain_t) == sizeof(hclib_hip_loop_domain_t), "hclib_loop_domain_t layout");
    hclib_hip_sweep_plan_t p;
    int rc = hclib_hip_forasync_plan(dim, (hclib_hip_loop_domain_t *)domain, mode, stream, &p);
    if (rc || p.total == 0) return rc;
    int64_t grid = (p.total + 255) / 256;
    const int64_t cap = (int64_t)(hclib_hip_num_cus() > 0 ? hclib_hip_num_cus() : 1) * 16;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(detail::k_user_sweep<Body>, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, body, p);
    if (hipGetLastError() != hipSuccess) rc = HCLIB_HIP_EHIP;
    const int rr = hclib_hip_forasync_plan_release(&p, stream);
    return rc ? rc : rr;
}

}  // namespace hip
}  // namespace hclib

// The kind table (include/hclib.h): register, before main, a launcher for a
// host function of the program. `fp` is the function the program passes to
// hclib_async / spawn (a device task kind) or to hclib_forasync (a device
// loop body); `launcher` is int (void *args) resp. int (void *args, int dim,
// hclib_loop_domain_t *domain, int mode, void *stream), defined in this
// translation unit (typically run_tasks<Kind> / run_dag<Kind> /
// forasync_device around the program's own device code).
#define HCLIB_HIP_KIND_CAT2(a, b) a##b
#define HCLIB_HIP_KIND_CAT(a, b) HCLIB_HIP_KIND_CAT2(a, b)
#define HCLIB_HIP_DEVICE_ASYNC(fp, launcher)                                                        \
    static const int HCLIB_HIP_KIND_CAT(hclib_hip_kind_reg_, __LINE__) =                            \
        (hclib_hip_register_device_async((generic_frame_ptr)(fp), #fp, (launcher)), 0)
#define HCLIB_HIP_DEVICE_FORASYNC(fct, launcher)                                                    \
    static const int HCLIB_HIP_KIND_CAT(hclib_hip_body_reg_, __LINE__) =                            \
        (hclib_hip_register_device_forasync((void *)(fct), #fct, (launcher)), 0)

namespace hclib {
namespace hip {

// ------------------------------------------------------- device forasync
struct RunTable {
    const hclib_sets::Run *runs;
    const int64_t *prefix;  // prefix[r] = iterations before run r
    int nruns;
};

__device__ __forceinline__ int run_idx(const RunTable &t, int64_t i) {
    int lo = 0, hi = t.nruns - 1;
    while (lo < hi) {  // last run whose prefix <= i
        const int mid = (lo + hi + 1) >> 1;
        if (t.prefix[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    const hclib_sets::Run r = t.runs[lo];
    return r.first + (int)(i - t.prefix[lo]) * r.stride;
}

// one unit-stride or strided run: no table
template <typename F>
__global__ __launch_bounds__(256) void k_forasync_run(hclib_sets::Run r, F f) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < r.count; t += step)
        f(r.first + (int)t * r.stride);
}

// the cartesian product of 1-3 run tables; the innermost index varies
// fastest so consecutive lanes touch consecutive indices
template <int ND, typename F>
__global__ __launch_bounds__(256) void k_forasync_runs(RunTable t0, RunTable t1, RunTable t2, int64_t n1,
                                                       int64_t n2, int64_t total, F f) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += step) {
        if constexpr (ND == 1) {
            f(run_idx(t0, t));
        } else if constexpr (ND == 2) {
            f(run_idx(t0, t / n1), run_idx(t1, t % n1));
        } else {
            const int64_t r = t / n2;
            f(run_idx(t0, r / n1), run_idx(t1, r % n1), run_idx(t2, t % n2));
        }
    }
}

namespace detail {

inline int num_workers() {
    const int n = hclib_hip_num_workers();
    return n > 0 ? n : 1;
}

inline std::vector<hclib_sets::Run> dim_runs(hclib_loop_domain_t *d, int ndim, int mode) {
    hclib_sets::resolve_tile(&d->tile, d->low, d->high, num_workers());
    const hclib_sets::Domain dd{d->low, d->high, d->stride, d->tile};
    return hclib_sets::runs(dd, ndim, mode);
}

inline int grid_for(int64_t total) {
    int64_t g = (total + 255) / 256;
    const int64_t cap = (int64_t)(hclib_hip_num_cus() > 0 ? hclib_hip_num_cus() : 256) * 8;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

// Upload the run tables of `nd` dimensions, launch, and (blocking) wait.
template <int ND, typename F>
int launch_runs(std::vector<hclib_sets::Run> *r, F f, hipStream_t s, bool blocking) {
    int64_t n[3] = {1, 1, 1}, total = 1;
    for (int d = 0; d < ND; ++d) {
        n[d] = hclib_sets::count(r[d]);
        total *= n[d];
    }
    if (total == 0) return HCLIB_HIP_OK;
    bool single = false;
    if constexpr (ND == 1) {
        if (r[0].size() == 1) {
            hipLaunchKernelGGL(k_forasync_run<F>, dim3(grid_for(total)), dim3(256), 0, s, r[0][0], f);
            single = true;
        }
    }
    if (!single) {
        size_t bytes = 0;
        for (int d = 0; d < ND; ++d) bytes += r[d].size() * (sizeof(hclib_sets::Run) + 8) + 8 + 64;
        std::vector<char> h(bytes);
        char *dbuf = nullptr;
        if (hipMalloc((void **)&dbuf, bytes) != hipSuccess) return HCLIB_HIP_ENOMEM;
        RunTable t[3] = {};
        size_t off = 0;
        for (int d = 0; d < ND; ++d) {
            std::vector<int64_t> pre(r[d].size() + 1, 0);
            for (size_t i = 0; i < r[d].size(); ++i) pre[i + 1] = pre[i] + r[d][i].count;
            memcpy(&h[off], r[d].data(), r[d].size() * sizeof(hclib_sets::Run));
            t[d].runs = (const hclib_sets::Run *)(dbuf + off);
            off += (r[d].size() * sizeof(hclib_sets::Run) + 15) & ~(size_t)15;
            memcpy(&h[off], pre.data(), pre.size() * 8);
            t[d].prefix = (const int64_t *)(dbuf + off);
            off += (pre.size() * 8 + 15) & ~(size_t)15;
            t[d].nruns = (int)r[d].size();
        }
        if (hipMemcpyAsync(dbuf, h.data(), bytes, hipMemcpyHostToDevice, s) != hipSuccess) return HCLIB_HIP_EHIP;
        hipLaunchKernelGGL((k_forasync_runs<ND, F>), dim3(grid_for(total)), dim3(256), 0, s, t[0], t[1], t[2],
                           ND > 1 ? n[1] : 1, ND > 2 ? n[2] : 1, total, f);
        if (blocking) {
            if (hipStreamSynchronize(s) != hipSuccess) return HCLIB_HIP_EHIP;
            (void)hipFree(dbuf);
        } else {
            (void)hipFreeAsync(dbuf, s);  // the table outlives the launch on its stream
        }
    }
    if (hipGetLastError() != hipSuccess) return HCLIB_HIP_EHIP;
    if (blocking && hipStreamSynchronize(s) != hipSuccess) return HCLIB_HIP_EHIP;
    return HCLIB_HIP_OK;
}

template <int ND, typename F>
int forasync(hclib_loop_domain_t *loop, F f, int mode, hipStream_t s, bool blocking) {
    if (hclib_hip_init(0) != HCLIB_HIP_OK) return HCLIB_HIP_ENODEV;
    std::vector<hclib_sets::Run> r[3];
    for (int d = 0; d < ND; ++d) {
        if (loop[d].stride < 1) return HCLIB_HIP_EINVAL;
        r[d] = dim_runs(&loop[d], ND, mode);
    }
    return launch_runs<ND>(r, f, s, blocking);
}

}  // namespace detail

template <typename F>
int forasync1D(hclib::loop_domain_1d *loop, F f, int mode = FORASYNC_MODE_RECURSIVE, hipStream_t s = nullptr) {
    return detail::forasync<1>(loop->get_internal(), f, mode, s, true);
}
template <typename F>
int forasync1D_nb(hclib::loop_domain_1d *loop, F f, int mode = FORASYNC_MODE_RECURSIVE, hipStream_t s = nullptr) {
    return detail::forasync<1>(loop->get_internal(), f, mode, s, false);
}
template <typename F>
int forasync2D(hclib::loop_domain_2d *loop, F f, int mode = FORASYNC_MODE_RECURSIVE, hipStream_t s = nullptr) {
    return detail::forasync<2>(loop->get_internal(), f, mode, s, true);
}
template <typename F>
int forasync2D_nb(hclib::loop_domain_2d *loop, F f, int mode = FORASYNC_MODE_RECURSIVE, hipStream_t s = nullptr) {
    return detail::forasync<2>(loop->get_internal(), f, mode, s, false);
}
template <typename F>
int forasync3D(hclib::loop_domain_3d *loop, F f, int mode = FORASYNC_MODE_RECURSIVE, hipStream_t s = nullptr) {
    return detail::forasync<3>(loop->get_internal(), f, mode, s, true);
}
template <typename F>
int forasync3D_nb(hclib::loop_domain_3d *loop, F f, int mode = FORASYNC_MODE_RECURSIVE, hipStream_t s = nullptr) {
    return detail::forasync<3>(loop->get_internal(), f, mode, s, false);
}

// ------------------------------------------------- user device task kinds
template <class Kind, int CAP>
__global__ __launch_bounds__(64) void k_run_tasks(typename Kind::Ctx ctx, hx::PoolView pool, hx::SchedGlobals *g,
                                                  hx::SchedConfig cfg) {
    __shared__ hx::WaveStack<Kind, CAP> st;
    hx::run_worker<Kind, CAP>(ctx, pool, g, cfg, st, blockIdx.x == 0);
}

// Device finish scopes for a task kind (hx_finish.h): `capacity` scopes in
// device memory plus the bump allocator and the outermost scope's value. A
// kind keeps view() in its Ctx; tasks open scopes with hx::finish_open and
// check out with hx::finish_check_out (continuations run inline).
class finish_arena {
  public:
    explicit finish_arena(uint32_t capacity) : cap_(capacity) {
        const size_t sb = sizeof(hx::FinishScope) * (size_t)capacity;
        off_ = (sb + 255) & ~(size_t)255;
        if (hipMalloc(&mem_, off_ + 256) != hipSuccess) mem_ = nullptr;
        reset();
    }
    ~finish_arena() {
        if (mem_) (void)hipFree(mem_);
    }
    finish_arena(const finish_arena &) = delete;
    finish_arena &operator=(const finish_arena &) = delete;
    bool ok() const { return mem_ != nullptr; }
    // every scope free again, no value at the root (ordered on the null stream)
    void reset() {
        if (mem_) (void)hipMemset((char *)mem_ + off_, 0, 256);
    }
    // pre-open scope ids [0, n) before a launch (e.g. a top-level finish the
    // root tasks check out of): scope i has counts[i] tasks, parent[i]
    int preopen(const std::vector<uint32_t> &counts, const std::vector<uint32_t> &parents,
                const std::vector<uint32_t> &conts) {
        const size_t n = counts.size();
        if (n > cap_ || parents.size() != n || conts.size() != n) return HCLIB_HIP_EINVAL;
        std::vector<hx::FinishScope> h(n);
        for (size_t i = 0; i < n; ++i) h[i] = hx::FinishScope{(unsigned long long)counts[i] << 56, parents[i], conts[i]};
        uint32_t next = (uint32_t)n;
        if (hipMemcpy(mem_, h.data(), n * sizeof(hx::FinishScope), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy((char *)mem_ + off_, &next, 4, hipMemcpyHostToDevice) != hipSuccess)
            return HCLIB_HIP_EHIP;
        return HCLIB_HIP_OK;
    }
    hx::FinishArena view() const {
        hx::FinishArena a;
        a.scopes = (hx::FinishScope *)mem_;
        a.next = (uint32_t *)((char *)mem_ + off_);
        a.cap = cap_;
        a.root_value = (unsigned long long *)((char *)mem_ + off_ + 64);
        return a;
    }
    // the value the outermost scope handed up (after the launch)
    uint64_t root_value() const {
        uint64_t v = 0;
        (void)hipMemcpy(&v, (char *)mem_ + off_ + 64, 8, hipMemcpyDeviceToHost);
        return v;
    }
    uint32_t scopes_opened() const {
        uint32_t n = 0;
        (void)hipMemcpy(&n, (char *)mem_ + off_, 4, hipMemcpyDeviceToHost);
        return n;
    }

  private:
    uint32_t cap_;
    size_t off_ = 0;
    void *mem_ = nullptr;
};

struct task_stats {
    uint64_t counters[16];  // [0..7] the kind's Acc::flush counters, [8..15] scheduler
    uint64_t maxes[4];      // the kind's atomic maxima
    double kernel_ms;
};

struct task_config {
    int waves_per_cu = 4;       // resident waves (workers) per CU
    uint32_t chunk = 64;        // items per stolen chunk
    uint32_t spill_hi = 512;    // ring occupancy that always spills
    uint32_t spill_lo = 32;     // occupancy from which items go to hungry waves
    uint32_t hunger = 8;        // batches between reads of the hunger signal
    uint32_t spin_limit_ms = 20000;
};

// hclib::launch + async/finish of a device kind: wave 0 seeds Kind::roots,
// the megakernel runs until every task (and every queued chunk) is done.
template <class Kind, int CAP = 1024>
int run_tasks(const typename Kind::Ctx &ctx, task_stats *stats = nullptr, const task_config &c = task_config()) {
    hclib_hip_sched_launch_t L;
    int rc = hclib_hip_sched_begin((uint32_t)Kind::kWords, c.chunk, c.waves_per_cu, &L);
    if (rc != HCLIB_HIP_OK) return rc;
    hx::PoolView pool;
    pool.hdr = (hx::QueueHdr *)L.hdr;
    pool.seq = L.seq;
    pool.cnt = L.cnt;
    pool.data = L.data;
    pool.nq = L.nq;
    pool.cap = L.cap;
    pool.chunk = L.chunk;
    hx::SchedConfig cfg;
    cfg.spill_hi = c.spill_hi;
    cfg.spill_lo = c.spill_lo;
    cfg.spin_limit = c.spin_limit_ms;
    cfg.nwaves = (uint32_t)L.grid;
    cfg.stamps = 0;
    cfg.hunger = c.hunger;
    hipLaunchKernelGGL((k_run_tasks<Kind, CAP>), dim3(L.grid), dim3(64), 0, (hipStream_t)L.stream, ctx, pool,
                       (hx::SchedGlobals *)L.globals, cfg);
    task_stats local;
    task_stats *s = stats ? stats : &local;
    return hclib_hip_sched_end("hclib::hip::run_tasks", s->counters, s->maxes, &s->kernel_ms);
}

// ------------------------------------------------ device promise DAG
class dag;
// Run every task of `g` on the GPU and wait (the enclosing finish ends).
// Errors: a double put or a task nothing releases -> HCLIB_HIP_EDEVICE.
template <class Kind>
int run_dag(const typename Kind::Ctx &ctx, dag &g, hclib_hip_dag_stats_t *stats = nullptr, int waves_per_cu = 4,
            uint32_t spin_limit_ms = 0);
// The same with workgroup tasks (hx::run_dag_group): every task runs on all
// `waves_per_group` waves of one workgroup (Kind::run_group), puts split
// around the body (kPutN / promises / datums) and, for tagged Kinds,
// reserved ready slots (kReserve; include/hclib_hip/hx_dag.h).
template <class Kind>
int run_dag_groups(const typename Kind::Ctx &ctx, dag &g, hclib_hip_dag_stats_t *stats = nullptr,
                   int groups_per_cu = 1, int waves_per_group = 1, uint32_t spin_limit_ms = 0);

// Host-side graph builder: the device counterpart of creating promises with
// hclib_promise_create and tasks with hclib_async(fn, arg, futures, n).
class dag {
  public:
    explicit dag(uint32_t payload_words) : words_(payload_words) { await_off_.push_back(0); }

    // hclib_promise_create: a new promise id
    uint32_t promise() {
        preput_.push_back(0);
        pre_datum_.push_back(0);
        return (uint32_t)preput_.size() - 1;
    }
    // hclib_promise_put before the launch (e.g. the boundary promises of
    // test/smithwaterman/smith_waterman.cpp:141-165)
    void put(uint32_t p, uint64_t datum) {
        preput_.at(p) = 1;
        pre_datum_.at(p) = datum;
    }
    // hclib_async(..., futures, n): a task with `payload_words` words of
    // payload that runs once every awaited promise is put
    uint32_t async_await(const uint32_t *payload, const uint32_t *futures, int n) {
        payload_.insert(payload_.end(), payload, payload + words_);
        for (int i = 0; i < n; ++i) await_ids_.push_back(futures[i]);
        await_off_.push_back((uint32_t)await_ids_.size());
        return (uint32_t)await_off_.size() - 2;
    }
    uint32_t async_await(const uint32_t *payload, std::initializer_list<uint32_t> futures) {
        std::vector<uint32_t> f(futures);
        return async_await(payload, f.data(), (int)f.size());
    }
    uint32_t num_tasks() const { return (uint32_t)await_off_.size() - 1; }
    uint32_t num_promises() const { return (uint32_t)preput_.size(); }
    // after run_dag: hclib_future_get / hclib_future_is_satisfied
    uint64_t datum(uint32_t p) const { return datum_.at(p); }
    bool satisfied(uint32_t p) const { return sat_.at(p) != 0; }

    template <class Kind>
    friend int run_dag(const typename Kind::Ctx &ctx, dag &g, hclib_hip_dag_stats_t *stats, int waves_per_cu,
                       uint32_t spin_limit_ms);
    template <class Kind>
    friend int run_dag_groups(const typename Kind::Ctx &ctx, dag &g, hclib_hip_dag_stats_t *stats, int groups_per_cu,
                              int waves_per_group, uint32_t spin_limit_ms);

  private:
    uint32_t words_;
    std::vector<uint32_t> payload_, await_off_, await_ids_;
    std::vector<uint8_t> preput_, sat_;
    std::vector<uint64_t> pre_datum_, datum_;
};

template <class Kind>
__global__ __launch_bounds__(64) void k_run_dag(typename Kind::Ctx ctx, hx::DagView v) {
    hx::run_dag_worker<Kind>(ctx, v);
}

template <class Kind>
int run_dag(const typename Kind::Ctx &ctx, dag &g, hclib_hip_dag_stats_t *stats, int waves_per_cu,
            uint32_t spin_limit_ms) {
    hclib_hip_dag_launch_t L;
    int rc = hclib_hip_dag_begin(g.num_tasks(), g.num_promises(), g.words_, g.payload_.data(), g.await_off_.data(),
                                 g.await_ids_.data(), g.preput_.data(), g.pre_datum_.data(), waves_per_cu,
                                 spin_limit_ms, &L);
    if (rc != HCLIB_HIP_OK) return rc;
    const hx::DagView v = *(const hx::DagView *)L.view;
    hipLaunchKernelGGL((k_run_dag<Kind>), dim3(L.grid), dim3(64), 0, (hipStream_t)L.stream, ctx, v);
    g.datum_.assign(g.num_promises(), 0);
    g.sat_.assign(g.num_promises(), 0);
    hclib_hip_dag_stats_t local;
    return hclib_hip_dag_end("hclib::hip::run_dag", g.datum_.data(), g.sat_.data(), stats ? stats : &local);
}

template <class Kind>
__global__ __launch_bounds__(1024) void k_run_dag_groups(typename Kind::Ctx ctx, hx::DagView v) {
    hx::run_dag_group<Kind>(ctx, v, nullptr);
}

template <class Kind>
int run_dag_groups(const typename Kind::Ctx &ctx, dag &g, hclib_hip_dag_stats_t *stats, int groups_per_cu,
                   int waves_per_group, uint32_t spin_limit_ms) {
    if (waves_per_group < 1 || waves_per_group > 16) {
        fprintf(stderr, "hclib::hip::run_dag_groups: 1..16 waves per group\n");
        return HCLIB_HIP_EINVAL;
    }
    hclib_hip_dag_launch_t L;
    int rc = hclib_hip_dag_begin(g.num_tasks(), g.num_promises(), g.words_, g.payload_.data(), g.await_off_.data(),
                                 g.await_ids_.data(), g.preput_.data(), g.pre_datum_.data(), groups_per_cu,
                                 spin_limit_ms, &L);
    if (rc != HCLIB_HIP_OK) return rc;
    const hx::DagView v = *(const hx::DagView *)L.view;
    hipLaunchKernelGGL((k_run_dag_groups<Kind>), dim3(L.grid), dim3(64 * waves_per_group), 0, (hipStream_t)L.stream,
                       ctx, v);
    g.datum_.assign(g.num_promises(), 0);
    g.sat_.assign(g.num_promises(), 0);
    hclib_hip_dag_stats_t local;
    return hclib_hip_dag_end("hclib::hip::run_dag_groups", g.datum_.data(), g.sat_.data(), stats ? stats : &local);
}

// ------------------------------------------------- dynamic device dataflow
// run_dyn<Kind>(ctx, roots, caps): the root tasks (payload_words u32 each,
// `roots` holds nroots * payload_words words) run on the persistent waves
// and create promises and async_await tasks as they go
// (include/hclib_hip/hx_dyn.h); returns when every created task has run, or
// HCLIB_HIP_EDEVICE (double put, pool exhausted, deadlock). dyn_datum reads
// promises back afterwards.
struct dyn_caps {
    uint32_t tasks = 1u << 20, promises = 1u << 20, wait_nodes = 1u << 21;
    int waves_per_cu = 4;
    uint32_t spin_limit_ms = 0;  // 0: HCLIB_HIP_SPIN_LIMIT_MS or 20 s
};

template <class Kind>
__global__ __launch_bounds__(64) void k_run_dyn(typename Kind::Ctx ctx, hx::DynView v) {
    hx::run_dyn_worker<Kind>(ctx, v);
}

template <class Kind>
int run_dyn(const typename Kind::Ctx &ctx, uint32_t payload_words, const std::vector<uint32_t> &roots,
            const dyn_caps &caps = dyn_caps(), hclib_hip_dyn_stats_t *stats = nullptr) {
    const uint32_t nroots = payload_words ? (uint32_t)(roots.size() / payload_words) : (uint32_t)roots.size();
    hclib_hip_dyn_launch_t L;
    int rc = hclib_hip_dyn_begin(payload_words, roots.data(), nroots, caps.tasks, caps.promises, caps.wait_nodes,
                                 caps.waves_per_cu, caps.spin_limit_ms, &L);
    if (rc != HCLIB_HIP_OK) return rc;
    const hx::DynView v = *(const hx::DynView *)L.view;
    hipLaunchKernelGGL((k_run_dyn<Kind>), dim3(L.grid), dim3(64), 0, (hipStream_t)L.stream, ctx, v);
    hclib_hip_dyn_stats_t local;
    return hclib_hip_dyn_end("hclib::hip::run_dyn", stats ? stats : &local);
}

inline std::vector<uint64_t> dyn_datum(uint32_t first, uint32_t n) {
    std::vector<uint64_t> d(n, 0);
    if (hclib_hip_dyn_datum(first, n, d.data(), nullptr) != HCLIB_HIP_OK) d.clear();
    return d;
}

}  // namespace hip
}  // namespace hclib

#endif  // HCLIB_HIP_CPP_H_
