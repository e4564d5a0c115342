// dag.hip — host side of the device promise DAG (include/hclib_hip/hx_dag.h).
//
// begin(): the host half of spawn_await / register_on_all_promise_dependencies
// (src/hclib-runtime.c:596-644, src/hclib-promise.c:132-195) done once for the
// whole graph: each task's dependency counter = its futures on promises not
// yet put; per promise, the tasks awaiting it (CSR, one entry per await); the
// tasks that wait on nothing seed the ready list in task order. Everything is
// uploaded in one copy to one device allocation on the module stream.
// end(): the host half of hclib_end_finish for the launch — wait, read the
// error word, hand the promises' data back.
#include <string.h>

#include <vector>

#include "hx_module.h"
#include "../../include/hclib_hip/hx_dag.h"

namespace hx {
namespace {

struct DagState {
    bool active = false;
    DagView view{};
    void *arena = nullptr;
    size_t arena_bytes = 0;
    uint32_t ntasks = 0, npromises = 0;
    unsigned long long *trace = nullptr;  // HX_DAG_TRACE builds: the per-task timeline
};

DagState g_dag;

size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace
}  // namespace hx

using namespace hx;

extern "C" int hclib_hip_dag_begin(uint32_t ntasks, uint32_t npromises, uint32_t payload_words,
                                   const uint32_t *payload, const uint32_t *await_off,
                                   const uint32_t *await_ids, const uint8_t *preput,
                                   const uint64_t *preput_datum, int waves_per_cu,
                                   uint32_t spin_limit_ms, hclib_hip_dag_launch_t *out) {
    if (!out || (ntasks && !await_off) || (payload_words && ntasks && !payload) || waves_per_cu < 1 ||
        waves_per_cu > 8 || ntasks >= kDagEmpty) {
        set_error("hclib_hip_dag_begin: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    if (g_dag.active) {
        set_error("hclib_hip_dag_begin: a DAG launch is already open (call hclib_hip_dag_end)");
        return HCLIB_HIP_EINVAL;
    }
    const uint32_t nawaits = ntasks ? await_off[ntasks] : 0;
    if (nawaits && !await_ids) {
        set_error("hclib_hip_dag_begin: await_ids is NULL");
        return HCLIB_HIP_EINVAL;
    }
    // counters and the waiter CSR (src/hclib-promise.c:132-195, for all tasks at once)
    std::vector<uint32_t> deps(ntasks, 0), woff(npromises + 1, 0), ready(ntasks, kDagEmpty);
    for (uint32_t t = 0; t < ntasks; ++t) {
        if (await_off[t + 1] < await_off[t]) {
            set_error("hclib_hip_dag_begin: await_off is not monotone at task %u", t);
            return HCLIB_HIP_EINVAL;
        }
        for (uint32_t k = await_off[t]; k < await_off[t + 1]; ++k) {
            const uint32_t p = await_ids[k];
            if (p >= npromises) {
                set_error("hclib_hip_dag_begin: task %u awaits promise %u of %u", t, p, npromises);
                return HCLIB_HIP_EINVAL;
            }
            if (preput && preput[p]) continue;  // satisfied: not registered (:136-139)
            ++deps[t];
            ++woff[p + 1];
        }
    }
    for (uint32_t p = 0; p < npromises; ++p) woff[p + 1] += woff[p];
    std::vector<uint32_t> waiters(woff[npromises] ? woff[npromises] : 1), fill(woff.begin(), woff.end() - 1);
    for (uint32_t t = 0; t < ntasks; ++t)
        for (uint32_t k = await_off[t]; k < await_off[t + 1]; ++k) {
            const uint32_t p = await_ids[k];
            if (!(preput && preput[p])) waiters[fill[p]++] = t;
        }
    uint32_t nready = 0;
    for (uint32_t t = 0; t < ntasks; ++t)
        if (deps[t] == 0) ready[nready++] = t;
    // a group Kind with reserved puts (hx_dag.h kReserve) gives every waiter
    // entry a ready slot of its own: nready + the registered awaits in all
    const uint32_t nslots = nready + woff[npromises];
    if (nslots > ready.size()) ready.resize(nslots, kDagEmpty);
    std::vector<unsigned long long> datum(npromises ? npromises : 1, 0);
    std::vector<uint32_t> sat(npromises ? npromises : 1, 0);
    for (uint32_t p = 0; preput && p < npromises; ++p)
        if (preput[p]) {
            sat[p] = 1;
            datum[p] = preput_datum ? preput_datum[p] : 0;
        }
    // the graph is valid: from here on a device is needed
    HX_TRY(ensure_device());
    Module &m = mod();
    // one arena: ctl lines (head, tail, err), stats, then the arrays
    const size_t o_ctl = 0, o_stats = 1024, o_deps = 1280;
    const size_t o_woff = o_deps + up256((size_t)ntasks * 4 + 4);
    const size_t o_wait = o_woff + up256(woff.size() * 4);
    const size_t o_datum = o_wait + up256(waiters.size() * 4);
    const size_t o_sat = o_datum + up256(datum.size() * 8);
    const size_t o_pay = o_sat + up256(sat.size() * 4);
    const size_t o_ready = o_pay + up256((size_t)ntasks * payload_words * 4 + 4);
    const size_t bytes = o_ready + up256(ready.size() * 4 + 4);
    std::vector<char> h(bytes, 0);
    uint32_t *ctl = (uint32_t *)&h[o_ctl];
    ctl[64] = nready;  // tail
    memcpy(&h[o_deps], deps.data(), deps.size() * 4);
    memcpy(&h[o_woff], woff.data(), woff.size() * 4);
    memcpy(&h[o_wait], waiters.data(), waiters.size() * 4);
    memcpy(&h[o_datum], datum.data(), datum.size() * 8);
    memcpy(&h[o_sat], sat.data(), sat.size() * 4);
    if (ntasks && payload_words) memcpy(&h[o_pay], payload, (size_t)ntasks * payload_words * 4);
    memcpy(&h[o_ready], ready.data(), ready.size() * 4);
    if (bytes > g_dag.arena_bytes) {
        if (g_dag.arena) (void)hipFree(g_dag.arena);
        g_dag.arena = nullptr;
        g_dag.arena_bytes = 0;
        if (hipMalloc(&g_dag.arena, bytes) != hipSuccess) {
            set_error("hclib_hip_dag_begin: hipMalloc(%zu) failed", bytes);
            return HCLIB_HIP_ENOMEM;
        }
        g_dag.arena_bytes = bytes;
    }
    char *d = (char *)g_dag.arena;
    HX_TRY(upload_async(d, h.data(), bytes, m.stream));
    DagView &v = g_dag.view;
    v.head = (uint32_t *)(d + o_ctl);
    v.tail = (uint32_t *)(d + o_ctl + 256);
    v.err = (uint32_t *)(d + o_ctl + 512);
    v.stats = (unsigned long long *)(d + o_stats);
    v.deps = (uint32_t *)(d + o_deps);
    v.waiter_off = (const uint32_t *)(d + o_woff);
    v.waiters = (const uint32_t *)(d + o_wait);
    v.datum = (unsigned long long *)(d + o_datum);
    v.satisfied = (uint32_t *)(d + o_sat);
    v.payload = (const uint32_t *)(d + o_pay);
    v.ready = (uint32_t *)(d + o_ready);
    v.ntasks = ntasks;
    v.nslots = nslots;
    v.npromises = npromises;
    v.payload_words = payload_words;
    v.trace = nullptr;
#if HX_DAG_TRACE
    // diagnostic: per-task timeline (hx_dag.h kDagTraceWords), written to the
    // file HCLIB_HIP_DAG_TRACE names at hclib_hip_dag_end
    if (getenv("HCLIB_HIP_DAG_TRACE") && ntasks) {
        if (g_dag.trace) (void)hipFree(g_dag.trace);
        g_dag.trace = nullptr;
        const size_t tb = (size_t)ntasks * kDagTraceWords * 8;
        if (hipMalloc((void **)&g_dag.trace, tb) == hipSuccess) {
            HX_HIP(hipMemsetAsync(g_dag.trace, 0, tb, m.stream));
            v.trace = g_dag.trace;
        }
    }
#endif
    v.spin_ms = spin_limit_ms ? spin_limit_ms : (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    g_dag.ntasks = ntasks;
    g_dag.npromises = npromises;
    g_dag.active = true;
    HX_HIP(hipEventRecord(m.ev0, m.stream));
    out->view = &g_dag.view;
    out->stream = m.stream;
    const int64_t grid = (int64_t)m.num_cus * waves_per_cu;
    out->grid = (int)(ntasks < grid ? (ntasks ? ntasks : 1) : grid);
    out->ntasks = ntasks;
    out->npromises = npromises;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_dag_end(const char *who, uint64_t *datum_out, uint8_t *satisfied_out,
                                 hclib_hip_dag_stats_t *stats) {
    if (!g_dag.active) {
        set_error("hclib_hip_dag_end: no open DAG launch");
        return HCLIB_HIP_EINVAL;
    }
    g_dag.active = false;
    Module &m = mod();
    const DagView &v = g_dag.view;
    HX_HIP(hipGetLastError());
    HX_HIP(hipEventRecord(m.ev1, m.stream));
    uint32_t err = 0;
    unsigned long long st[6] = {0, 0, 0, 0, 0, 0};
    HX_HIP(hipMemcpyAsync(&err, v.err, 4, hipMemcpyDeviceToHost, m.stream));
    HX_HIP(hipMemcpyAsync(st, v.stats, sizeof(st), hipMemcpyDeviceToHost, m.stream));
    std::vector<uint32_t> sat;
    if (datum_out && g_dag.npromises)
        HX_HIP(hipMemcpyAsync(datum_out, v.datum, (size_t)g_dag.npromises * 8, hipMemcpyDeviceToHost, m.stream));
    // always read back: tagged puts count `satisfied` up without a result,
    // so a double put shows only here (a count of 2), whether or not the
    // caller asked for the satisfied flags
    if (g_dag.npromises) {
        sat.resize(g_dag.npromises);
        HX_HIP(hipMemcpyAsync(sat.data(), v.satisfied, sat.size() * 4, hipMemcpyDeviceToHost, m.stream));
    }
    HX_HIP(hipStreamSynchronize(m.stream));
    bool twice = false;  // tagged puts count satisfied up (hx_dag.h kTagged): 2 = put twice
    for (size_t p = 0; p < sat.size(); ++p) {
        if (satisfied_out) satisfied_out[p] = sat[p] ? 1 : 0;
        twice = twice || sat[p] > 1;
    }
    if (twice && !err) err = kErrDoublePut;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, m.ev0, m.ev1);
#if HX_DAG_TRACE
    if (v.trace) {
        HX_HIP(hipStreamSynchronize(m.stream));
        std::vector<unsigned long long> tr((size_t)g_dag.ntasks * kDagTraceWords);
        HX_HIP(hipMemcpy(tr.data(), v.trace, tr.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = fopen(getenv("HCLIB_HIP_DAG_TRACE"), "wb")) {
            fwrite(tr.data(), 8, tr.size(), f);
            fclose(f);
        }
    }
#endif
#if defined(HX_STAMPS) && HX_STAMPS
    if (st[0] && (st[3] | st[4] | st[5]))
        fprintf(stderr, "dag group phases (cycles per task, wave 0): take %.0f body %.0f put %.0f\n",
                (double)st[3] / st[0], (double)st[4] / st[0], (double)st[5] / st[0]);
#endif
    if (stats) {
        stats->tasks = st[0];
        stats->puts = st[1];
        stats->releases = st[2];
        stats->kernel_ms = ms;
    }
    const char *w = who ? who : "hclib_hip_dag";
    if (err == kErrDoublePut) {
        set_error("%s: violated single assignment property for promises (device put on a satisfied promise)", w);
        return HCLIB_HIP_EDEVICE;
    }
    if (err == kErrSpinTimeout) {
        set_error("%s: %llu of %u task(s) ran; the rest wait on promises that nothing puts (deadlock)", w,
                  (unsigned long long)st[0], g_dag.ntasks);
        return HCLIB_HIP_EDEVICE;
    }
    if (err) {
        set_error("%s: device error %u", w, err);
        return HCLIB_HIP_EDEVICE;
    }
    if (st[0] != g_dag.ntasks) {
        set_error("%s: %llu of %u tasks ran", w, (unsigned long long)st[0], g_dag.ntasks);
        return HCLIB_HIP_EDEVICE;
    }
    return HCLIB_HIP_OK;
}

// ------------------------------------------------ dynamic device dataflow
// (include/hclib_hip/hx_dyn.h) — the host half: pools, the roots, the
// launch's end. Promise heads start kDynOpen (0xff bytes), the ready list
// kDynEmpty; the roots take ready slots 0 .. nroots - 1 with no pending
// futures, and `live` starts at nroots.
#include "../../include/hclib_hip/hx_dyn.h"

namespace hx {
namespace {
struct DynState {
    bool active = false;
    DynView view{};
    void *arena = nullptr;
    size_t arena_bytes = 0;
};
DynState g_dyn;
}  // namespace
}  // namespace hx

extern "C" int hclib_hip_dyn_begin(uint32_t payload_words, const uint32_t *root_payload, uint32_t nroots,
                                   uint32_t task_cap, uint32_t promise_cap, uint32_t node_cap, int waves_per_cu,
                                   uint32_t spin_limit_ms, hclib_hip_dyn_launch_t *out) {
    if (!out || payload_words > (uint32_t)kDynMaxPayload || nroots == 0 || nroots > task_cap ||
        (payload_words && !root_payload) || task_cap >= kDynPut || promise_cap >= kDynPut || node_cap >= kDynPut ||
        waves_per_cu < 1 || waves_per_cu > 8) {
        set_error("hclib_hip_dyn_begin: invalid arguments (1 <= nroots <= task_cap, payload_words <= %d, "
                  "1..8 waves per CU)", kDynMaxPayload);
        return HCLIB_HIP_EINVAL;
    }
    if (g_dyn.active) {
        set_error("hclib_hip_dyn_begin: a dynamic launch is already open (call hclib_hip_dyn_end)");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = mod();
    const int64_t grid = (int64_t)m.num_cus * waves_per_cu;
    const uint32_t rcap = task_cap + (uint32_t)grid + 64;
    const uint32_t pcap = promise_cap ? promise_cap : 1, wcap = node_cap ? node_cap : 1;
    const size_t o_ctl = 0, o_stats = 2048, o_datum = 2304;
    const size_t o_phead = o_datum + up256((size_t)pcap * 8);
    const size_t o_wtask = o_phead + up256((size_t)pcap * 4);
    const size_t o_wnext = o_wtask + up256((size_t)wcap * 4);
    const size_t o_tdeps = o_wnext + up256((size_t)wcap * 4);
    const size_t o_tpay = o_tdeps + up256((size_t)task_cap * 4);
    const size_t o_ready = o_tpay + up256((size_t)task_cap * payload_words * 4 + 4);
    const size_t bytes = o_ready + up256((size_t)rcap * 4);
    if (bytes > g_dyn.arena_bytes) {
        if (g_dyn.arena) (void)hipFree(g_dyn.arena);
        g_dyn.arena = nullptr;
        g_dyn.arena_bytes = 0;
        if (hipMalloc(&g_dyn.arena, bytes) != hipSuccess) {
            set_error("hclib_hip_dyn_begin: hipMalloc(%zu) failed", bytes);
            return HCLIB_HIP_ENOMEM;
        }
        g_dyn.arena_bytes = bytes;
    }
    char *d = (char *)g_dyn.arena;
    // control + stats zeroed, heads and ready slots 0xff, then the roots
    HX_HIP(hipMemsetAsync(d, 0, o_datum, m.stream));
    HX_HIP(hipMemsetAsync(d + o_phead, 0xff, (size_t)pcap * 4, m.stream));
    HX_HIP(hipMemsetAsync(d + o_tdeps, 0, (size_t)task_cap * 4, m.stream));
    HX_HIP(hipMemsetAsync(d + o_ready, 0xff, (size_t)rcap * 4, m.stream));
    std::vector<uint32_t> ctl(2048 / 4, 0), ready(nroots);
    ctl[64] = nroots;   // tail
    ctl[128] = nroots;  // live
    ctl[256] = nroots;  // next task id
    for (uint32_t r = 0; r < nroots; ++r) ready[r] = r;
    HX_TRY(upload_async(d + o_ctl, ctl.data(), 2048, m.stream));
    HX_TRY(upload_async(d + o_ready, ready.data(), (size_t)nroots * 4, m.stream));
    if (payload_words) HX_TRY(upload_async(d + o_tpay, root_payload, (size_t)nroots * payload_words * 4, m.stream));
    DynView &v = g_dyn.view;
    v.ctl = (uint32_t *)(d + o_ctl);
    v.stats = (unsigned long long *)(d + o_stats);
    v.datum = (unsigned long long *)(d + o_datum);
    v.phead = (uint32_t *)(d + o_phead);
    v.wtask = (uint32_t *)(d + o_wtask);
    v.wnext = (uint32_t *)(d + o_wnext);
    v.tdeps = (uint32_t *)(d + o_tdeps);
    v.tpay = (uint32_t *)(d + o_tpay);
    v.ready = (uint32_t *)(d + o_ready);
    v.tcap = task_cap;
    v.pcap = promise_cap;
    v.wcap = node_cap;
    v.rcap = rcap;
    v.payload_words = payload_words;
    v.spin_ms = spin_limit_ms ? spin_limit_ms : (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    g_dyn.active = true;
    HX_HIP(hipEventRecord(m.ev0, m.stream));
    out->view = &g_dyn.view;
    out->stream = m.stream;
    out->grid = (int)grid;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_dyn_end(const char *who, hclib_hip_dyn_stats_t *stats) {
    if (!g_dyn.active) {
        set_error("hclib_hip_dyn_end: no open dynamic launch");
        return HCLIB_HIP_EINVAL;
    }
    g_dyn.active = false;
    Module &m = mod();
    const DynView &v = g_dyn.view;
    HX_HIP(hipGetLastError());
    HX_HIP(hipEventRecord(m.ev1, m.stream));
    uint32_t ctl[512];
    unsigned long long st[5] = {0, 0, 0, 0, 0};
    HX_HIP(hipMemcpyAsync(ctl, v.ctl, sizeof(ctl), hipMemcpyDeviceToHost, m.stream));
    HX_HIP(hipMemcpyAsync(st, v.stats, sizeof(st), hipMemcpyDeviceToHost, m.stream));
    HX_HIP(hipStreamSynchronize(m.stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, m.ev0, m.ev1);
    if (stats) {
        stats->tasks = st[0];
        stats->puts = st[1];
        stats->created = st[2];
        stats->releases = st[3];
        stats->promises = st[4];
        stats->kernel_ms = ms;
    }
    const char *w = who ? who : "hclib_hip_dyn";
    const uint32_t err = ctl[192], live = ctl[128];
    if (err == kErrDynDoublePut) {
        set_error("%s: violated single assignment property for promises (device put on a satisfied promise)", w);
        return HCLIB_HIP_EDEVICE;
    }
    if (err == kErrDynPool) {
        set_error("%s: a device pool ran out (tasks %u/%u, promises %u/%u, wait nodes %u/%u)", w, ctl[256], v.tcap,
                  ctl[320], v.pcap, ctl[384], v.wcap);
        return HCLIB_HIP_EDEVICE;
    }
    if (err == kErrSpinTimeout || (!err && live)) {
        set_error("%s: %llu task(s) ran, %u still wait on promises that nothing puts (deadlock)", w,
                  (unsigned long long)st[0], live);
        return HCLIB_HIP_EDEVICE;
    }
    if (err) {
        set_error("%s: device error %u", w, err);
        return HCLIB_HIP_EDEVICE;
    }
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_dyn_datum(uint32_t first, uint32_t n, uint64_t *datum, uint8_t *put) {
    const DynView &v = g_dyn.view;
    if (g_dyn.active || !g_dyn.arena || (uint64_t)first + n > v.pcap) {
        set_error("hclib_hip_dyn_datum: no finished launch or promises [%u, %u) outside the pool", first, first + n);
        return HCLIB_HIP_EINVAL;
    }
    if (!n) return HCLIB_HIP_OK;
    if (datum) HX_HIP(hipMemcpy(datum, v.datum + first, (size_t)n * 8, hipMemcpyDeviceToHost));
    if (put) {
        std::vector<uint32_t> h(n);
        HX_HIP(hipMemcpy(h.data(), v.phead + first, (size_t)n * 4, hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < n; ++k) put[k] = h[k] == kDynPut ? 1 : 0;
    }
    return HCLIB_HIP_OK;
}
