// hclib_api.hip — the HClib C API (include/hclib.h) on top of modules/hip.
//
// The host side of the MI355X runtime is a single control thread: the
// scheduler that matters runs on the GPU. This file keeps the reference's
// task model exactly where it is observable — finish counters
// (src/hclib-runtime.c:431-446, 1219-1313), promises with waiter lists and
// chained registration over a task's futures (src/hclib-promise.c:132-245),
// forasync tile-size rules (src/hclib.c:452-473) — and routes the work:
//   * device task kinds (fib, UTS) -> one persistent megakernel launch each
//     (uts.hip / fib.hip), their results written back into the task's own
//     argument struct when the task completes;
//   * device loop bodies -> one grid-stride sweep launch (forasync.hip);
//   * any other function -> a host task run by the control thread, help-first
//     inside end_finish / future_wait (the reference's work-shift,
//     src/hclib-runtime.c:1067-1119; no fibers needed with one thread).
// Errors abort with a message, like HASSERT / log_die in the reference.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/hclib.h"
#include "../../include/hclib_forasync_sets.h"
#include "hx_host.h"
#include "hx_module.h"

using hxh::die;

// finish_t, src/inc/hclib-finish.h:6-10
struct finish_t {
    finish_t *parent;
    int counter;
    hclib_promise_t *finish_dep;
};

static_assert(sizeof(hclib_task_t) == 96, "hclib_task_t keeps the reference's 96-byte layout");

namespace {

#define SENTINEL ((hclib_task_t *)0x1)
#define SATISFIED ((hclib_task_t *)0x2)

struct Runtime {
    bool launched = false;
    bool hip = false;
    std::vector<hclib_task_t *> ready;  // LIFO, like the owner end of a deque
    // the kind table: device task kinds and device loop bodies by the host
    // function that names them; built-in (fib, UTS, the library's loop
    // bodies, by id) or a user launcher from the program's own HIP object
    struct DevKind {
        int builtin = 0;
        hclib_hip_async_launcher_t launch = nullptr;
        std::string name;
    };
    struct DevBody {
        int builtin = 0;
        hclib_hip_forasync_launcher_t launch = nullptr;
        std::string name;
    };
    std::map<generic_frame_ptr, DevKind> kinds;
    std::map<void *, DevBody> bodies;
    // memory callbacks per locale type (src/hclib-mem.c:13-50)
    struct MemFuncs {
        hclib_module_alloc_impl_func_type alloc = nullptr;
        hclib_module_realloc_impl_func_type realloc = nullptr;
        hclib_module_free_impl_func_type free = nullptr;
        hclib_module_memset_impl_func_type memset = nullptr;
        hclib_module_copy_impl_func_type copy = nullptr;
        int copy_priority = 0;
    };
    std::map<int, MemFuncs> mem;
    bool mem_builtins = false;
    double user_timer = 0.0;  // hclib_user_harness_timer
    // stats (HCLIB_STATS analogue, src/hclib-runtime.c:83-104)
    unsigned long long host_tasks = 0, device_tasks = 0, end_finishes = 0, forasyncs = 0;
    unsigned long long spawned = 0, future_waits = 0, end_finishes_nb = 0, yields = 0, yield_iters = 0;
    unsigned long long device_items = 0, device_batches = 0, device_chunks_pushed = 0, device_chunks_stolen = 0;
    double device_ms = 0;
    std::vector<hclib_hip_wave_stats_t> waves;  // per device wave, summed over launches
};

Runtime &rt() {
    static Runtime r;
    return r;
}

// the finish scope and the task the host worker is running
inline finish_t *&current_finish() { return hxh::worker0()->current_finish; }
inline hclib_task_t *current_task() { return (hclib_task_t *)hxh::worker0()->curr_task; }

void check_in(finish_t *f) {
    if (f) f->counter++;
}

void check_out(finish_t *f) {
    if (f && --f->counter == 0 && f->finish_dep) hclib_promise_put(f->finish_dep, f);
}

// _register_if_promise_not_ready, src/hclib-promise.c:132-166
bool register_if_not_ready(hclib_task_t *t, hclib_future_t *fut) {
    hclib_promise_t *p = fut->owner;
    if (p->wait_list_head == SATISFIED) return false;
    t->next_waiter = p->wait_list_head;
    p->wait_list_head = t;
    return true;
}

// register_on_all_promise_dependencies, src/hclib-promise.c:171-195: every
// inline slot (a NULL slot is skipped, not a terminator), then the
// NULL-terminated waiting_on_extra
bool register_all(hclib_task_t *t) {
    while (t->waiting_on_index < MAX_NUM_WAITS - 1) {
        t->waiting_on_index++;
        hclib_future_t *f = t->waiting_on[t->waiting_on_index];
        if (f && register_if_not_ready(t, f)) return false;
    }
    if (t->waiting_on_extra) {
        while (true) {
            hclib_future_t *f = t->waiting_on_extra[t->waiting_on_index - MAX_NUM_WAITS + 1];
            if (!f) break;
            t->waiting_on_index++;
            if (register_if_not_ready(t, f)) return false;
        }
    }
    return true;
}

void make_ready(hclib_task_t *t) { rt().ready.push_back(t); }

int check_hip(int rc, const char *what) {
    if (rc != HCLIB_HIP_OK) die("%s failed: %s", what, hclib_hip_last_error());
    return rc;
}

// bind the hip module (modules/hip) to `device` (-1: the process's default,
// HCLIB_HIP_DEVICE or LOCAL_RANK). One GPU per process: a second device is
// an error, as one rank drives one GPU in the multi-GPU launch.
void ensure_gpu(const char *who, int device = -1) {
    if (device < 0) device = hx::env_int("HCLIB_HIP_DEVICE", hx::env_int("LOCAL_RANK", 0));
    const int have = hclib_hip_device();  // bound by an earlier call or by the hip module's callbacks
    if (have < 0) {
        if (hclib_hip_init(device) != HCLIB_HIP_OK)
            die("%s: the hip module could not bind a gfx950 device: %s", who, hclib_hip_last_error());
    } else if (have != device) {
        die("%s: this process drives GPU %d; GPU %d needs a process of its own", who, have, device);
    }
    rt().hip = true;
}

// the device a task at `locale` runs on (-1: the process's default)
int device_of(hclib_locale_t *locale) {
    const int d = hxh::locale_device(locale);
    return d;
}

// the megakernel's scheduler counters of the launch that just ended
// (include/hclib_hip.h: [13] batches, [14] chunks pushed, [15] chunks stolen)
void add_sched_counters(Runtime &R) {
    uint64_t c[16];
    hclib_hip_last_sched_counters(c);
    R.device_batches += c[13];
    R.device_chunks_pushed += c[14];
    R.device_chunks_stolen += c[15];
    const int n = hclib_hip_last_wave_stats(nullptr, 0);
    std::vector<hclib_hip_wave_stats_t> w((size_t)n);
    hclib_hip_last_wave_stats(w.data(), n);
    if (R.waves.size() < w.size()) R.waves.resize(w.size(), hclib_hip_wave_stats_t{});
    for (size_t i = 0; i < w.size(); ++i) {
        hclib_hip_wave_stats_t &a = R.waves[i];
        a.executed += w[i].executed;
        a.spawned += w[i].spawned;
        a.batches += w[i].batches;
        a.chunks_pushed += w[i].chunks_pushed;
        a.chunks_stolen += w[i].chunks_stolen;
        a.items_stolen += w[i].items_stolen;
        a.xcd = w[i].xcd;
        for (int x = 0; x < 8; ++x) a.stolen_from[x] += w[i].stolen_from[x];
    }
}

const Runtime::DevKind *kind_of(generic_frame_ptr fp) {
    Runtime &R = rt();
    if (R.kinds.empty()) return nullptr;
    auto k = R.kinds.find(fp);
    return k == R.kinds.end() ? nullptr : &k->second;
}

// run one device task kind to completion and write its outputs back
void run_device_task(hclib_task_t *t, const Runtime::DevKind &dk) {
    Runtime &R = rt();
    ensure_gpu("device task", device_of(t->locale));
    R.device_tasks++;
    if (dk.launch) {  // a user kind: its launcher runs it on the bound GPU
        check_hip(dk.launch(t->args), dk.name.c_str());
        add_sched_counters(R);
        return;
    }
    const int kind = dk.builtin;
    switch (kind) {
    case HCLIB_HIP_KIND_FIB: {
        // FibArgs of test/fib/fib.c:50-53: { int n; long res; }
        struct FibArgs {
            int n;
            long res;
        } *a = (FibArgs *)t->args;
        int64_t v = 0;
        hclib_hip_fib_result_t r;
        check_hip(hclib_hip_fib(a->n, &v, &r), "hclib_hip_fib");
        a->res = (long)v;
        R.device_items += r.tasks;
        add_sched_counters(R);
        R.device_ms += r.kernel_ms;
        break;
    }
    case HCLIB_HIP_KIND_UTS: {
        hclib_hip_uts_task_t *a = (hclib_hip_uts_task_t *)t->args;
        hclib_hip_uts_params_t p;
        p.type = a->type;
        p.shape_fn = a->shape_fn;
        p.gen_mx = a->gen_mx;
        p.root_id = a->root_id;
        p.non_leaf_bf = a->non_leaf_bf;
        p.compute_gran = a->compute_gran;
        p.b_0 = a->b_0;
        p.non_leaf_prob = a->non_leaf_prob;
        p.shift_depth = a->shift_depth;
        hclib_hip_uts_result_t r;
        check_hip(hclib_hip_uts_search(&p, 0, 1, 0, &r, nullptr, 0), "hclib_hip_uts_search");
        a->nodes = r.nodes;
        a->leaves = r.leaves;
        a->max_depth = r.max_depth;
        R.device_items += r.nodes;
        add_sched_counters(R);
        R.device_ms += r.kernel_ms;
        break;
    }
    default:
        die("unknown device task kind %d", kind);
    }
}

// the root task of hclib_launch: its record carries the user's function and
// argument (hclib_get_curr_task_info reports them, as the reference's root
// async does, src/hclib-runtime.c:1472) but it runs on a context of its own
hclib_task_t *g_root_task = nullptr;
void run_root(hclib_task_t *t);

// execute_task, src/hclib-runtime.c:448-478
void execute(hclib_task_t *t) {
    Runtime &R = rt();
    hclib_worker_state *ws = hxh::worker0();
    finish_t *saved = ws->current_finish;
    void *saved_task = ws->curr_task;
    ws->current_finish = t->current_finish;
    ws->curr_task = t;
    if (t == g_root_task) {
        R.host_tasks++;
        run_root(t);
    } else if (const Runtime::DevKind *dk = kind_of(t->_fp)) {
        run_device_task(t, *dk);
    } else {
        R.host_tasks++;
        t->_fp(t->args);
    }
    ws->curr_task = saved_task;
    ws->current_finish = saved;
    check_out(t->current_finish);
    free(t->waiting_on_extra);
    if (t != g_root_task) free(t);
}

// Device work in flight on the module stream that belongs to a finish scope
// (a device forasync): the scope stays checked in until the work's event
// completes, like the pending operations modules/cuda polls
// (modules/common/hclib-module-common.h:10-90). The host worker completes
// them while it helps: finished ones first, and when it has no ready task
// left it waits for the oldest.
struct DeviceOp {
    hipEvent_t ev;
    finish_t *finish;
    void (*done)(void *);
    void *arg;
};
std::vector<DeviceOp> &pending() {
    static std::vector<DeviceOp> p;
    return p;
}

void complete_op(size_t i) {
    DeviceOp op = pending()[i];
    pending().erase(pending().begin() + (ptrdiff_t)i);
    (void)hipEventDestroy(op.ev);
    if (op.done) op.done(op.arg);
    check_out(op.finish);
}

// returns true if any operation completed
bool poll_pending(bool wait_oldest) {
    std::vector<DeviceOp> &P = pending();
    if (P.empty()) return false;
    if (wait_oldest) {
        if (hipEventSynchronize(P[0].ev) != hipSuccess) die("device work of a finish scope failed");
        complete_op(0);
        return true;
    }
    bool any = false;
    for (size_t i = 0; i < P.size();) {
        const hipError_t e = hipEventQuery(P[i].ev);
        if (e == hipSuccess) {
            complete_op(i);
            any = true;
        } else if (e == hipErrorNotReady) {
            ++i;
        } else {
            die("device work of a finish scope failed: %s", hipGetErrorString(e));
        }
    }
    return any;
}

// register device work just enqueued on `stream` with the current finish
void add_device_op(hipStream_t stream, void (*done)(void *), void *arg) {
    DeviceOp op{nullptr, current_finish(), done, arg};
    if (hipEventCreateWithFlags(&op.ev, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(op.ev, stream) != hipSuccess)
        die("cannot record device work");
    check_in(op.finish);
    pending().push_back(op);
}

// find_and_run_task with one worker: complete finished device work, pop
// the newest ready task; with nothing ready, wait for the oldest device work
bool run_one() {
    Runtime &R = rt();
    // an operation completed here may have put the promise the caller waits
    // on: that is progress, even with nothing left to run or wait for
    if (poll_pending(false) && R.ready.empty()) return true;
    if (R.ready.empty()) return poll_pending(true);
    hclib_task_t *t = R.ready.back();
    R.ready.pop_back();
    execute(t);
    return true;
}

// spawn_handler, src/hclib-runtime.c:572-617: check in on the current
// finish (escaping tasks do not), copy the futures (extras into a
// NULL-terminated waiting_on_extra), schedule once all are satisfied
void spawn_handler(hclib_task_t *t, hclib_locale_t *locale, hclib_future_t **futures, int nfutures,
                   int escaping) {
    Runtime &R = rt();
    if (!R.launched) die("a task was spawned outside hclib_launch");
    if (!t) die("spawn: NULL task");
    if (escaping) {
        t->current_finish = nullptr;
    } else {
        check_in(current_finish());
        t->current_finish = current_finish();
    }
    if (locale) t->locale = locale;
    R.spawned++;
    if (nfutures > 0) {
        const int inl = nfutures > MAX_NUM_WAITS ? MAX_NUM_WAITS : nfutures;
        memcpy(t->waiting_on, futures, (size_t)inl * sizeof(*futures));
        if (nfutures > MAX_NUM_WAITS) {
            const int extra = nfutures - MAX_NUM_WAITS;
            t->waiting_on_extra = (hclib_future_t **)malloc((size_t)(extra + 1) * sizeof(hclib_future_t *));
            if (!t->waiting_on_extra) die("out of memory");
            memcpy(t->waiting_on_extra, futures + MAX_NUM_WAITS, (size_t)extra * sizeof(*futures));
            t->waiting_on_extra[extra] = nullptr;
        }
        t->waiting_on_index = -1;
    }
    // is_eligible_to_schedule, src/hclib-runtime.c:540-551
    if (!t->waiting_on[0] || register_all(t)) make_ready(t);
}

hclib_task_t *new_task(generic_frame_ptr fp, void *arg, int non_blocking) {
    hclib_task_t *t = (hclib_task_t *)calloc(1, sizeof(hclib_task_t));
    if (!t) die("out of memory");
    t->_fp = fp;
    t->args = arg;
    t->non_blocking = non_blocking;
    return t;
}

}  // namespace

namespace {
// The root task runs on a context of its own, as the reference's does (a
// LiteCtx fiber, src/hclib-runtime.c:1460-1478). Its stack is mmap'd with a
// PROT_NONE guard page below it (the reference's OVERFLOW_PROTECT pad,
// src/inc/litectx.h:68,117): every host task runs nested on it (help-first
// inside end_finish / future_wait), and an overflow must fault, not corrupt
// the heap. It stays mapped until the launch ends, so tasks that outlive the
// root body and still read its locals (test/cpp/promise/future5.cpp) see
// them intact.
constexpr size_t kRootStack = 8u << 20;  // touched lazily
ucontext_t g_root_ret, g_root_ctx;
void *g_root_map = nullptr;
size_t g_root_map_len = 0;
void root_trampoline() { g_root_task->_fp(g_root_task->args); }
void run_root(hclib_task_t *) {
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    g_root_map_len = kRootStack + page;
    g_root_map = mmap(nullptr, g_root_map_len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                      -1, 0);
    if (g_root_map == MAP_FAILED || mprotect(g_root_map, page, PROT_NONE) != 0 || getcontext(&g_root_ctx) != 0)
        die("hclib_launch: cannot create the root context");
    g_root_ctx.uc_stack.ss_sp = (char *)g_root_map + page;
    g_root_ctx.uc_stack.ss_size = kRootStack;
    g_root_ctx.uc_link = &g_root_ret;
    makecontext(&g_root_ctx, root_trampoline, 0);
    if (swapcontext(&g_root_ret, &g_root_ctx) != 0) die("hclib_launch: cannot enter the root context");
}
}  // namespace

extern "C" {

// ------------------------------------------------------------ lifecycle
// hclib_entrypoint, src/hclib-runtime.c:319-401: load the modules named in
// deps, their pre-init functions, the locality graph, their post-init
// functions, then the root finish
void hclib_init(const char **deps, int ndeps, const int instrument) {
    (void)instrument;
    Runtime &R = rt();
    if (R.launched) die("hclib_init called twice");
    hxh::load_dependencies(deps, ndeps);
    hclib_call_module_pre_init_functions();
    hxh::bind_worker0();  // builds the graph, makes current_ws() answer here
    hclib_call_module_post_init_functions();
    R.launched = true;
    current_finish() = nullptr;
    hclib_start_finish();  // root finish (src/hclib-runtime.c:400)
}

void hclib_finalize(const int instrument) {
    (void)instrument;
    Runtime &R = rt();
    hclib_end_finish();
    hclib_call_finalize_functions();
    R.launched = false;
    const char *stats = getenv("HCLIB_STATS");
    if (stats && *stats && strcmp(stats, "0")) hclib_print_runtime_stats(stdout);
}

void hclib_launch(async_fct_t fct_ptr, void *arg, const char **deps, int ndeps) {
    const char *prof = getenv("HCLIB_PROFILE_LAUNCH_BODY");
    hclib_init(deps, ndeps, 0);
    const unsigned long long t0 = hclib_current_time_ns();
    hclib_task_t root;
    memset(&root, 0, sizeof(root));
    root._fp = fct_ptr;
    root.args = arg;
    g_root_task = &root;
    spawn_handler(&root, hclib_get_closest_locale(), nullptr, 0, 0);
    hclib_finalize(0);  // ends the root finish: the root task runs here
    g_root_task = nullptr;
    if (g_root_map) munmap(g_root_map, g_root_map_len);
    g_root_map = nullptr;
    const unsigned long long t1 = hclib_current_time_ns();
    if (prof && *prof) printf("\nHCLIB TIME %llu ns\n", t1 - t0);
}

unsigned long long hclib_current_time_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (unsigned long long)ts.tv_sec * 1000000000ull + ts.tv_nsec;
}

unsigned long long hclib_current_time_ms(void) { return hclib_current_time_ns() / 1000000ull; }

// ---------------------------------------------------------------- tasks
// inc/hclib-async-struct.h:49-54, src/hclib-runtime.c:619-644
void spawn(hclib_task_t *task) { spawn_handler(task, nullptr, nullptr, 0, 0); }
void spawn_at(hclib_task_t *task, hclib_locale_t *locale) { spawn_handler(task, locale, nullptr, 0, 0); }
void spawn_await_at(hclib_task_t *task, hclib_future_t **futures, const int nfutures, hclib_locale_t *locale) {
    spawn_handler(task, locale, futures, nfutures, 0);
}
void spawn_await(hclib_task_t *task, hclib_future_t **futures, const int nfutures) {
    spawn_handler(task, nullptr, futures, nfutures, 0);
}

// src/hclib.c:34-57
void hclib_async(generic_frame_ptr fp, void *arg, hclib_future_t **futures, const int nfutures,
                 hclib_locale_t *locale) {
    spawn_handler(new_task(fp, arg, 0), locale, futures, nfutures, 0);
}

void hclib_async_nb(generic_frame_ptr fp, void *arg, hclib_locale_t *locale) {
    spawn_handler(new_task(fp, arg, 1), locale, nullptr, 0, 0);
}

// hclib_yield, src/hclib-runtime.c:1142-1217, with the control thread as the
// only host worker: run ready tasks, newest first, until none is left or a
// blocking one has run (the reference breaks after it swaps to a blocking
// task's context).
void hclib_yield(hclib_locale_t *locale) {
    (void)locale;
    Runtime &R = rt();
    if (!R.launched) die("hclib_yield called outside hclib_launch");
    R.yields++;
    while (!R.ready.empty()) {
        const int nb = R.ready.back()->non_blocking;
        R.yield_iters++;
        run_one();
        if (!nb) break;
    }
}

namespace {
struct FutureWrapper {
    hclib_promise_t event;
    future_fct_t fp;
    void *in;
};
void future_caller(void *raw) {  // src/hclib.c:65-69
    FutureWrapper *w = (FutureWrapper *)raw;
    void *r = w->fp(w->in);
    hclib_promise_put(&w->event, r);
}
}  // namespace

hclib_future_t *hclib_async_future(future_fct_t fp, void *arg, hclib_future_t **futures,
                                   const int nfutures, hclib_locale_t *locale) {
    FutureWrapper *w = (FutureWrapper *)malloc(sizeof(FutureWrapper));
    hclib_promise_init(&w->event);
    w->fp = fp;
    w->in = arg;
    hclib_async(future_caller, w, futures, nfutures, locale);
    return &w->event.future;
}

// hclib_start_finish, src/hclib-runtime.c:1219-1247
void hclib_start_finish(void) {
    finish_t *f = (finish_t *)calloc(1, sizeof(finish_t));
    if (!f) die("out of memory");
    f->counter = 1;
    f->parent = current_finish();
    check_in(f->parent);
    current_finish() = f;
}

// hclib_end_finish + help_finish, src/hclib-runtime.c:1249-1277, 1067-1119
void hclib_end_finish(void) {
    Runtime &R = rt();
    finish_t *f = current_finish();
    if (!f) die("hclib_end_finish without a matching start");
    R.end_finishes++;
    while (f->counter > 1) {
        if (!run_one())
            die("end_finish: %d task(s) wait on promises that nothing can put (deadlock)",
                f->counter - 1);
    }
    current_finish() = f->parent;
    check_out(f->parent);
    free(f);
}

// src/hclib-runtime.c:1280-1313
void hclib_end_finish_nonblocking_helper(hclib_promise_t *event) {
    Runtime &R = rt();
    R.end_finishes_nb++;
    finish_t *f = current_finish();
    if (!f) die("hclib_end_finish_nonblocking without a matching start");
    f->finish_dep = event;
    current_finish() = f->parent;
    check_out(f);  // the owner's check-out; puts `event` when the scope drains
    check_out(f->parent);
}

hclib_future_t *hclib_end_finish_nonblocking(void) {
    hclib_promise_t *e = hclib_promise_create();
    hclib_end_finish_nonblocking_helper(e);
    return &e->future;
}

}  // extern "C"

namespace {

// A host loop body (a C function pointer the GPU cannot run) is lowered the
// way the reference lowers every forasync (src/hclib.c:110-473): one task
// per tile, registered with the enclosing finish, each running
// forasync{1,2,3}D_runner's loop nest over its tile. The tiles are the runs
// of include/hclib_forasync_sets.h, so the iteration set (including the
// FLAT low != 0 overrun quirk) is the reference's.
struct HostTile {
    void *fct;
    void *argv;
    int dim;
    hclib_sets::Run r[3];
};

void host_tile_runner(void *raw) {  // forasync{1,2,3}D_runner, src/hclib.c:110-156
    HostTile *t = (HostTile *)raw;
    const hclib_sets::Run &a = t->r[0], &b = t->r[1], &c = t->r[2];
    for (int i = 0; i < a.count; ++i) {
        const int x = a.first + i * a.stride;
        if (t->dim == 1) {
            ((forasync1D_Fct_t)t->fct)(t->argv, x);
            continue;
        }
        for (int j = 0; j < b.count; ++j) {
            const int y = b.first + j * b.stride;
            if (t->dim == 2) {
                ((forasync2D_Fct_t)t->fct)(t->argv, x, y);
                continue;
            }
            for (int k = 0; k < c.count; ++k)
                ((forasync3D_Fct_t)t->fct)(t->argv, x, y, c.first + k * c.stride);
        }
    }
    free(t);
}

void forasync_host(void *fct, void *argv, int dim, hclib_loop_domain_t *domain, int mode) {
    Runtime &R = rt();
    R.forasyncs++;
    std::vector<hclib_sets::Run> runs[3];
    for (int d = 0; d < dim; ++d) {
        if (domain[d].stride < 1) die("hclib_forasync: stride must be >= 1");
        // tile == -1 -> auto, written back (src/hclib.c:455-461)
        hclib_sets::resolve_tile(&domain[d].tile, domain[d].low, domain[d].high,
                                 hclib_get_num_workers());
        const hclib_sets::Domain dd{domain[d].low, domain[d].high, domain[d].stride, domain[d].tile};
        runs[d] = hclib_sets::runs(dd, dim, mode == FORASYNC_MODE_RECURSIVE ? 1 : 0);
    }
    const hclib_sets::Run one{0, 1, 1, 0};
    const size_t n1 = dim > 1 ? runs[1].size() : 1, n2 = dim > 2 ? runs[2].size() : 1;
    for (const hclib_sets::Run &a : runs[0])
        for (size_t j = 0; j < n1; ++j)
            for (size_t k = 0; k < n2; ++k) {
                HostTile *t = (HostTile *)malloc(sizeof(HostTile));
                if (!t) die("out of memory");
                t->fct = fct;
                t->argv = argv;
                t->dim = dim;
                t->r[0] = a;
                t->r[1] = dim > 1 ? runs[1][j] : one;
                t->r[2] = dim > 2 ? runs[2][k] : one;
                spawn_handler(new_task(host_tile_runner, t, 0), nullptr, nullptr, 0, 0);
            }
}

}  // namespace

namespace {
struct IotaOp {
    int *host;
    size_t n;
    int *dev_ran, *dev_err;
};
void iota_done(void *raw) {
    IotaOp *op = (IotaOp *)raw;
    int nerr = 0;
    if (hipMemcpy(op->host, op->dev_ran, op->n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&nerr, op->dev_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        die("hclib_forasync: copy-back failed");
    (void)hipFree(op->dev_ran);
    (void)hipFree(op->dev_err);
    free(op);
    if (nerr) die("forasync body check failed at %d indices", nerr);
}
}  // namespace

extern "C" {

// ------------------------------------------------------------- forasync
void hclib_forasync(void *fct, void *argv, int dim, hclib_loop_domain_t *domain,
                    forasync_mode_t mode) {
    Runtime &R = rt();
    if (!R.launched) die("hclib_forasync called outside hclib_launch");
    if (dim < 1 || dim > 3) die("hclib_forasync: dim %d not in 1..3", dim);
    auto b = R.bodies.find(fct);
    if (b == R.bodies.end()) {  // a host loop body: host tile tasks
        forasync_host(fct, argv, dim, domain, mode);
        return;
    }
    ensure_gpu("hclib_forasync");
    R.forasyncs++;
    static_assert(sizeof(hclib_loop_domain_t) == sizeof(hclib_hip_loop_domain_t), "layout");
    hclib_hip_loop_domain_t *d = (hclib_hip_loop_domain_t *)domain;
    hipStream_t st = hx::mod().stream;
    int rc;
    if (b->second.launch) {
        // a user body: its launcher enqueues the sweep on the module stream;
        // it completes with the enclosing finish, as the built-in bodies do
        rc = b->second.launch(argv, dim, domain, (int)mode, st);
        check_hip(rc, b->second.name.c_str());
        add_device_op(st, nullptr, nullptr);
        return;
    }
    if (b->second.builtin == HCLIB_HIP_BODY_IOTA_CHECK) {
        // test/c/forasync1DCh.c passes a plain host int array: the sweep runs
        // on a device copy, copied back when the sweep completes
        hclib_hip_loop_domain_t dd = d[0];
        const int nw = hclib_hip_num_workers() > 0 ? hclib_hip_num_workers() : 1;
        if (dd.tile == -1) dd.tile = ((dd.high - dd.low) + nw - 1) / nw;
        const size_t extent = (size_t)(dd.high + (dd.tile > 0 ? dd.tile : 1));
        IotaOp *op = (IotaOp *)calloc(1, sizeof(IotaOp));
        if (!op) die("out of memory");
        op->host = (int *)argv;
        op->n = (size_t)dd.high;
        if (hipMalloc((void **)&op->dev_ran, extent * sizeof(int)) != hipSuccess ||
            hipMalloc((void **)&op->dev_err, sizeof(int)) != hipSuccess)
            die("hclib_forasync: device allocation failed");
        if (hipMemcpyAsync(op->dev_ran, argv, op->n * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(op->dev_err, 0, sizeof(int), st) != hipSuccess)
            die("hclib_forasync: upload failed");
        hclib_hip_iota_args_t ia = {op->dev_ran, op->dev_err};
        rc = hclib_hip_forasync(b->second.builtin, &ia, dim, d, mode, st);
        check_hip(rc, "hclib_hip_forasync");
        add_device_op(st, iota_done, op);
    } else {
        // the sweep belongs to the enclosing finish: it completes there (or
        // in whatever helps first), the host thread does not wait for it here
        rc = hclib_hip_forasync(b->second.builtin, argv, dim, d, mode, st);
        check_hip(rc, "hclib_hip_forasync");
        add_device_op(st, nullptr, nullptr);
    }
}

hclib_future_t *hclib_forasync_future(void *fct, void *argv, int dim,
                                      hclib_loop_domain_t *domain, forasync_mode_t mode) {
    hclib_start_finish();  // src/hclib.c:466-473
    hclib_forasync(fct, argv, dim, domain, mode);
    return hclib_end_finish_nonblocking();
}

// ------------------------------------------------------------- promises
void hclib_promise_init(hclib_promise_t *p) {
    p->satisfied = 0;
    p->datum = nullptr;
    p->wait_list_head = SENTINEL;
    p->future.owner = p;
}

hclib_promise_t *hclib_promise_create(void) {
    hclib_promise_t *p = (hclib_promise_t *)malloc(sizeof(hclib_promise_t));
    if (!p) die("out of memory");
    hclib_promise_init(p);
    return p;
}

hclib_future_t *hclib_get_future_for_promise(hclib_promise_t *p) { return &p->future; }

hclib_promise_t **hclib_promise_create_n(size_t n, int null_terminated) {
    hclib_promise_t **ps = (hclib_promise_t **)malloc(sizeof(hclib_promise_t *) * n);
    const size_t lg = null_terminated ? n - 1 : n;
    for (size_t i = 0; i < lg; ++i) ps[i] = hclib_promise_create();
    if (null_terminated) ps[lg] = nullptr;
    return ps;
}

void hclib_promise_free_n(hclib_promise_t **ps, size_t n, int null_terminated) {
    const size_t lg = null_terminated ? n - 1 : n;
    for (size_t i = 0; i < lg; ++i) hclib_promise_free(ps[i]);
    free(ps);
}

void hclib_promise_free(hclib_promise_t *p) { free(p); }

void *hclib_future_get(hclib_future_t *f) {
    if (!f->owner->satisfied) die("hclib_future_get on an unsatisfied future");
    return f->owner->datum;
}

// hclib_promise_put, src/hclib-promise.c:203-245
void hclib_promise_put(hclib_promise_t *p, void *datum) {
    if (p->satisfied) die("violated single assignment property for promises");
    p->datum = datum;
    p->satisfied = 1;
    hclib_task_t *list = p->wait_list_head;
    p->wait_list_head = SATISFIED;
    while (list != SENTINEL) {
        hclib_task_t *next = list->next_waiter;
        if (register_all(list)) make_ready(list);
        list = next;
    }
}

// hclib_future_wait, src/hclib-runtime.c:983-1025 (help while waiting)
void *hclib_future_wait(hclib_future_t *f) {
    rt().future_waits++;
    while (!f->owner->satisfied) {
        if (!run_one()) die("future_wait: the future can never be satisfied (deadlock)");
    }
    return f->owner->datum;
}

int hclib_future_is_satisfied(hclib_future_t *f) { return f->owner->satisfied; }

}  // extern "C"

// ------------------------------------------- locales and memory operations
namespace {

// "sysmem" callbacks (the reference's system module registers the same
// libc calls for its sysmem locale)
void *host_alloc(size_t n, hclib_locale_t *) { return malloc(n ? n : 1); }
void *host_realloc(void *p, size_t n, hclib_locale_t *) { return realloc(p, n ? n : 1); }
void host_free(void *p, hclib_locale_t *) { free(p); }
void host_memset(void *p, int v, size_t n, hclib_locale_t *) { memset(p, v, n); }
void host_copy(hclib_locale_t *, void *d, hclib_locale_t *, void *s, size_t n) { memcpy(d, s, n); }

Runtime::MemFuncs &mem_of(int type) {
    Runtime &R = rt();
    if (!R.mem_builtins) {
        R.mem_builtins = true;
        Runtime::MemFuncs &h = R.mem[0];
        h.alloc = host_alloc;
        h.realloc = host_realloc;
        h.free = host_free;
        h.memset = host_memset;
        h.copy = host_copy;
        h.copy_priority = MAY_USE;
        // a GPU locale type's callbacks come from the hip plug-in module
        // (hclib_amd/csrc/modules/hclib_hip_module.hip), registered in its
        // post-init like the reference's modules/cuda
    }
    return R.mem[type];
}

hclib_locale_t *check_locale(hclib_locale_t *l, const char *who) {
    if (!l) die("%s: NULL locale", who);
    return l;
}

struct MemTask {  // malloc_struct / realloc_struct / memset_struct / copy_struct
    int op;       // 0 alloc, 1 realloc, 2 memset, 3 copy
    void *ptr;
    size_t nbytes;
    int pattern;
    hclib_locale_t *locale, *src_locale;
    void *src;
    hclib_future_t *src_fut;
    hclib_promise_t *promise;
    Runtime::MemFuncs *fn;
    hclib_module_copy_impl_func_type copy;
};

// allocate_kernel / reallocate_kernel / memset_kernel / copy_kernel,
// src/hclib-mem.c:59-191
void mem_task(void *raw) {
    MemTask *m = (MemTask *)raw;
    void *out = nullptr;
    switch (m->op) {
    case 0: out = m->fn->alloc(m->nbytes, m->locale); break;
    case 1: out = m->fn->realloc(m->ptr, m->nbytes, m->locale); break;
    case 2: m->fn->memset(m->ptr, m->pattern, m->nbytes, m->locale); break;
    default:
        m->copy(m->locale, m->ptr, m->src_locale, m->src ? m->src : hclib_future_get(m->src_fut), m->nbytes);
        break;
    }
    hclib_promise_put(m->promise, out);
    free(m);
}

hclib_future_t *spawn_mem(MemTask *m, hclib_future_t **futures, int nfutures) {
    m->promise = hclib_promise_create();
    hclib_future_t *f = hclib_get_future_for_promise(m->promise);
    hclib_async(mem_task, m, futures, nfutures, m->locale);
    return f;
}

MemTask *new_mem_task(int op, hclib_locale_t *l) {
    MemTask *m = (MemTask *)calloc(1, sizeof(MemTask));
    if (!m) die("out of memory");
    m->op = op;
    m->locale = l;
    m->fn = &mem_of(l->type);
    return m;
}

}  // namespace

extern "C" {

// hclib_register_*_func, src/hclib-mem.c:23-50 (alloc/realloc/free/memset are MAY_USE)
void hclib_register_alloc_func(int t, hclib_module_alloc_impl_func_type f) { mem_of(t).alloc = f; }
void hclib_register_realloc_func(int t, hclib_module_realloc_impl_func_type f) { mem_of(t).realloc = f; }
void hclib_register_free_func(int t, hclib_module_free_impl_func_type f) { mem_of(t).free = f; }
void hclib_register_memset_func(int t, hclib_module_memset_impl_func_type f) { mem_of(t).memset = f; }
void hclib_register_copy_func(int t, hclib_module_copy_impl_func_type f, int priority) {
    mem_of(t).copy = f;
    mem_of(t).copy_priority = priority;
}

hclib_future_t *hclib_allocate_at(size_t nbytes, hclib_locale_t *locale) {
    MemTask *m = new_mem_task(0, check_locale(locale, "hclib_allocate_at"));
    if (!m->fn->alloc) die("hclib_allocate_at: no allocator for locale type %d", locale->type);
    m->nbytes = nbytes;
    return spawn_mem(m, nullptr, 0);
}

hclib_future_t *hclib_reallocate_at(void *ptr, size_t new_nbytes, hclib_locale_t *locale) {
    MemTask *m = new_mem_task(1, check_locale(locale, "hclib_reallocate_at"));
    if (!m->fn->realloc) die("hclib_reallocate_at: no reallocator for locale type %d", locale->type);
    m->ptr = ptr;
    m->nbytes = new_nbytes;
    return spawn_mem(m, nullptr, 0);
}

hclib_future_t *hclib_memset_at(void *ptr, int pattern, size_t nbytes, hclib_locale_t *locale) {
    MemTask *m = new_mem_task(2, check_locale(locale, "hclib_memset_at"));
    if (!m->fn->memset) die("hclib_memset_at: no memset for locale type %d", locale->type);
    m->ptr = ptr;
    m->pattern = pattern;
    m->nbytes = nbytes;
    return spawn_mem(m, nullptr, 0);
}

void hclib_free_at(void *ptr, hclib_locale_t *locale) {  // src/hclib-mem.c:148-154 (synchronous)
    Runtime::MemFuncs &f = mem_of(check_locale(locale, "hclib_free_at")->type);
    if (!f.free) die("hclib_free_at: no free for locale type %d", locale->type);
    f.free(ptr, locale);
}

// src/hclib-mem.c:193-241: the MUST_USE side's copy wins; both MUST_USE is an error
hclib_future_t *hclib_async_copy(hclib_locale_t *dst_locale, void *dst, hclib_locale_t *src_locale, void *src,
                                 size_t nbytes, hclib_future_t **futures, const int nfutures) {
    check_locale(dst_locale, "hclib_async_copy");
    check_locale(src_locale, "hclib_async_copy");
    Runtime::MemFuncs &d = mem_of(dst_locale->type), &sm = mem_of(src_locale->type);
    hclib_module_copy_impl_func_type cb;
    if (!d.copy && !sm.copy) die("hclib_async_copy: no copy function for locale types %d, %d", dst_locale->type,
                                 src_locale->type);
    if (!d.copy) cb = sm.copy;
    else if (!sm.copy) cb = d.copy;
    else if (d.copy == sm.copy) cb = d.copy;
    else {
        if (d.copy_priority == MUST_USE && sm.copy_priority == MUST_USE)
            die("hclib_async_copy: both locales' copy functions are MUST_USE");
        cb = sm.copy_priority == MUST_USE ? sm.copy : d.copy;
    }
    MemTask *m = new_mem_task(3, dst_locale);
    m->ptr = dst;
    m->src_locale = src_locale;
    m->nbytes = nbytes;
    m->copy = cb;
    if (src == HCLIB_ASYNC_COPY_USE_FUTURE_AS_SRC) {
        if (nfutures != 1) die("hclib_async_copy: a future source needs exactly one future");
        m->src = nullptr;
        m->src_fut = futures[0];
    } else {
        m->src = src;
    }
    return spawn_mem(m, futures, nfutures);
}

}  // extern "C"

extern "C" {

// -------------------------------------------------------------- queries
// src/hclib-runtime.c:1365-1368 (workers_backlog, src/hclib-locality-graph.c:
// 742-758): tasks queued on the calling worker's deques. Here the caller is
// the host control thread, whose deque is the help-first ready list; device
// tasks live in the megakernel's queues only while a launch runs.
size_t hclib_current_worker_backlog(void) { return rt().ready.size(); }

// src/hclib-locality-graph.c:760-768: tasks queued at `locale` over every
// worker's deque there. Here: the ready host tasks placed at it (a task
// spawned without a locale sits at the closest locale, the reference's
// default push place, src/hclib-runtime.c:518-521)
unsigned locale_num_tasks(hclib_locale_t *locale) {
    if (!locale) die("locale_num_tasks: NULL locale");
    hclib_locale_t *dflt = hclib_get_closest_locale();
    unsigned n = 0;
    for (hclib_task_t *t : rt().ready) n += (t->locale ? t->locale : dflt) == locale;
    return n;
}

// src/hclib-locality-graph.c:807-813: append to the locale's idle functions
void locale_register_idle_task(hclib_locale_t *locale, void (*fp)(void)) {
    if (!locale || !fp) die("locale_register_idle_task: NULL argument");
    void (**grown)(void) =
        (void (**)(void))realloc((void *)locale->idle_funcs, (locale->n_idle_funcs + 1) * sizeof(void (*)(void)));
    if (!grown) die("locale_register_idle_task: out of memory");
    locale->idle_funcs = grown;
    locale->idle_funcs[locale->n_idle_funcs++] = fp;
}

// src/hclib-locality-graph.c:815-827: every idle function of every locale on
// the worker's steal path, in path order
void locale_run_idle_tasks(hclib_worker_state *ws) {
    if (!ws || !ws->paths || !ws->paths->steal_path) die("locale_run_idle_tasks: worker has no paths");
    const hclib_locality_path *steal = ws->paths->steal_path;
    for (unsigned i = 0; i < steal->path_length; ++i) {
        hclib_locale_t *l = steal->locales[i];
        for (unsigned j = 0; j < l->n_idle_funcs; ++j) l->idle_funcs[j]();
    }
}

// src/hclib-runtime.c:1319-1321: recorded; HCLIB_STATS prints it
void hclib_user_harness_timer(double dur) { rt().user_timer = dur; }

// src/hclib-runtime.c:480-486: used / capacity of the caller's deque
void hclib_default_queue_capacity(int *used, int *capacity) {
    if (used) *used = (int)rt().ready.size();
    if (capacity) *capacity = 1 << 20;  // INIT_DEQUE_CAPACITY of the reference
}

// src/hclib.c:475-480: function and argument of the running task (the
// root task's when called from the hclib_launch entrypoint)
void hclib_get_curr_task_info(void (**fp_out)(void *), void **args_out) {
    hclib_task_t *t = current_task();
    if (!t) die("hclib_get_curr_task_info: no task is running");
    if (fp_out) *fp_out = t->_fp;
    if (args_out) *args_out = t->args;
}

// src/hclib-runtime.c:1340-1363: run fp(data) on the main context. The host
// control thread is the main context here (no fibers), so it runs in place.
void hclib_run_on_main_ctx(void (*fp)(void *), void *data) {
    if (!fp) die("hclib_run_on_main_ctx: null function");
    fp(data);
}

// src/hclib.c:16-30 and src/hclib-runtime.c:231-239, 396: loop distribution
// functions; id 0 (HCLIB_DEFAULT_LOOP_DIST) places every tile at the central
// place
static hclib_locale_t *default_dist_func(const int, const hclib_loop_domain_t *, const hclib_loop_domain_t *,
                                         const int) {
    return hclib_get_central_place();
}
static std::vector<loop_dist_func> &dist_funcs() {
    static std::vector<loop_dist_func> v{default_dist_func};
    return v;
}
unsigned hclib_register_dist_func(loop_dist_func func) {
    if (!func) die("hclib_register_dist_func: null function");
    dist_funcs().push_back(func);
    return (unsigned)dist_funcs().size() - 1;
}
loop_dist_func hclib_lookup_dist_func(unsigned id) {
    if (id >= dist_funcs().size()) die("hclib_lookup_dist_func: no function %u", id);
    return dist_funcs()[id];
}

// the GPU locale standing for HIP device `index` (the first one of the graph)
hclib_locale_t *hclib_hip_gpu_locale(int index) {
    // asking for a GPU locale means using it: a host without a gfx950 device
    // (or without the hip module loaded) fails here, loudly
    if (hxh::gpu_type() == ~0u)
        die("hclib_hip_gpu_locale: no GPU locale type (load the \"hip\" module: deps {\"system\", \"hip\"})");
    // the locale first: a graph without this device (e.g. LOCAL_RANK=1's,
    // which holds only GPU 1) must not initialise the device before failing
    const int n = hclib_get_num_locales();
    bool any_gpu = false;
    for (int i = 0; i < n; ++i) {
        hclib_locale_t *l = hclib_get_locale(i);
        any_gpu = any_gpu || hxh::locale_device(l) >= 0;
        if (hxh::locale_device(l) == index) {
            ensure_gpu("hclib_hip_gpu_locale", hxh::locale_device(l));
            return l;
        }
    }
    // a graph without any GPU: the module found no device to bind; say why
    // (binding is what failed, and no other GPU of the graph gets touched)
    if (!any_gpu) ensure_gpu("hclib_hip_gpu_locale", index);
    die("hclib_hip_gpu_locale: the locality graph has no locale for GPU %d", index);
}

void hclib_hip_register_async_kind(generic_frame_ptr fp, int kind) {
    if (kind != HCLIB_HIP_KIND_FIB && kind != HCLIB_HIP_KIND_UTS)
        die("hclib_hip_register_async_kind: unknown kind %d (the built-in kinds are HCLIB_HIP_KIND_FIB and "
            "HCLIB_HIP_KIND_UTS; a kind of the program's own registers a launcher with "
            "hclib_hip_register_device_async)", kind);
    Runtime::DevKind k;
    k.builtin = kind;
    k.name = kind == HCLIB_HIP_KIND_FIB ? "fib" : "uts";
    rt().kinds[fp] = k;
}

void hclib_hip_register_forasync_body(void *fct, int body) {
    if (body < HCLIB_HIP_BODY_TRIAD_F32 || body > HCLIB_HIP_BODY_VISIT_COUNT)
        die("hclib_hip_register_forasync_body: unknown body %d (the built-in bodies are "
            "HCLIB_HIP_BODY_TRIAD_F32..HCLIB_HIP_BODY_VISIT_COUNT; a body of the program's own registers a "
            "launcher with hclib_hip_register_device_forasync)", body);
    Runtime::DevBody b;
    b.builtin = body;
    b.name = "built-in body";
    rt().bodies[fct] = b;
}

// the kind table entries of the program's own HIP objects
// (HCLIB_HIP_DEVICE_ASYNC / HCLIB_HIP_DEVICE_FORASYNC, include/hclib_hip_cpp.h)
void hclib_hip_register_device_async(generic_frame_ptr fp, const char *name, hclib_hip_async_launcher_t launch) {
    if (!fp || !launch) die("hclib_hip_register_device_async: null function or launcher");
    Runtime::DevKind k;
    k.launch = launch;
    k.name = name ? name : "device kind";
    rt().kinds[fp] = k;
}

void hclib_hip_register_device_forasync(void *fct, const char *name, hclib_hip_forasync_launcher_t launch) {
    if (!fct || !launch) die("hclib_hip_register_device_forasync: null body or launcher");
    Runtime::DevBody b;
    b.launch = launch;
    b.name = name ? name : "device body";
    rt().bodies[fct] = b;
}

int hclib_hip_device_kind_count(void) { return (int)rt().kinds.size(); }

const char *hclib_hip_device_kind_name(generic_frame_ptr fp) {
    const Runtime::DevKind *k = kind_of(fp);
    return k ? k->name.c_str() : nullptr;
}

// hclib_print_runtime_stats, src/hclib-runtime.c:1370-1410: the reference's
// report layout, one line per worker, then the totals. Worker 0 is the host
// control thread. The device's workers are the megakernel's waves: one line
// per wave of the device launches so far (its own record, summed over
// launches: tasks run, children created, chunks taken from other deques
// and the tasks in them, and from which XCD's deques they came).
void hclib_print_runtime_stats(FILE *fp) {
    Runtime &R = rt();
    fprintf(fp, "===== HClib statistics: =====\n");
    fprintf(fp,
            "  Worker 0: %llu tasks executed, %llu tasks spawned, %llu tasks scheduled, 0 steals, "
            "0 stolen tasks, 0.000000 tasks per steal, stolen from = [ 0 ]\n",
            R.host_tasks + R.device_tasks, R.spawned, R.spawned);
    unsigned long long dev_exec = 0;
    for (size_t i = 0; i < R.waves.size(); ++i) {
        const hclib_hip_wave_stats_t &w = R.waves[i];
        dev_exec += w.executed;
        fprintf(fp,
                "  Device wave %zu (XCD %llu): %llu tasks executed, %llu tasks spawned, %llu batches, "
                "%llu chunks pushed, %llu steals, %llu stolen tasks, %f tasks per steal, stolen from = [ ",
                i, (unsigned long long)w.xcd, (unsigned long long)w.executed, (unsigned long long)w.spawned,
                (unsigned long long)w.batches, (unsigned long long)w.chunks_pushed,
                (unsigned long long)w.chunks_stolen, (unsigned long long)w.items_stolen,
                w.chunks_stolen ? (double)w.items_stolen / (double)w.chunks_stolen : 0.0);
        for (int x = 0; x < 8; ++x) fprintf(fp, "%llu ", (unsigned long long)w.stolen_from[x]);
        fprintf(fp, "]\n");
    }
    if (R.device_tasks)
        fprintf(fp,
                "  Device (%zu waves): %llu device items executed in %llu batches, %llu chunks pushed, "
                "%llu chunks stolen, %f items per batch, %.3f ms\n",
                R.waves.size(), R.device_items, R.device_batches, R.device_chunks_pushed, R.device_chunks_stolen,
                R.device_batches ? (double)R.device_items / (double)R.device_batches : 0.0, R.device_ms);
    fprintf(fp,
            "Total: %llu tasks, %llu end finishes, %llu future waits, %llu non-blocking end finishes, "
            "0 ctx creates, %llu yields, %f iters per yield on average\n",
            R.host_tasks + R.device_tasks + dev_exec, R.end_finishes, R.future_waits, R.end_finishes_nb,
            R.yields, R.yields ? (double)R.yield_iters / (double)R.yields : 0.0);
    if (R.user_timer > 0.0) fprintf(fp, "User harness timer: %f s\n", R.user_timer);
}

}  // extern "C"
