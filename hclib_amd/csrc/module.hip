// module.hip — `modules/hip` lifecycle, error reporting and the shared
// chunk-deque arena (the HBM side of the per-wave deques, sched.h).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hx_module.h"

namespace hx {

static Module g_mod;
static thread_local char g_err[512] = "";

Module &mod() { return g_mod; }

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_resident(const void *kern, int blocks, int threads, size_t lds, const char *what) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess) return HCLIB_HIP_OK;
    const long long cap = (long long)per_cu * mod().num_cus;
    if (blocks > cap) {
        set_error("%s: %d workgroups of %d threads cannot all be resident (%d per CU x %d CUs: LDS / registers); "
                  "the persistent workers would wait on waves that never start (lower HCLIB_HIP_WAVES_PER_CU)",
                  what, blocks, threads, per_cu, mod().num_cus);
        return HCLIB_HIP_EINVAL;
    }
    return HCLIB_HIP_OK;
}

int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return HCLIB_HIP_OK;
    set_error("%s failed: %s", what, hipGetErrorString(e));
    return HCLIB_HIP_EHIP;
}

int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

int ensure_device() {
    if (g_mod.inited) return HCLIB_HIP_OK;
    return hclib_hip_init(env_int("HCLIB_HIP_DEVICE", 0)) == HCLIB_HIP_OK ? HCLIB_HIP_OK
                                                                           : HCLIB_HIP_ENODEV;
}

// slot control pairs {seq, cnt}: slot i is free for ticket i (mod cap)
__global__ void k_reset_pool(uint32_t *seq, uint32_t cap, uint32_t total) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) {
        seq[2 * i] = i & (cap - 1);
        seq[2 * i + 1] = 0;
    }
}

int make_pool(uint32_t nq, uint32_t cap, uint32_t chunk, uint32_t words, PoolView *out) {
    if (nq < 8 || nq % 8 || cap < 2 || (cap & (cap - 1)) || chunk < 1 || chunk > 64) {
        set_error("chunk deques: need 8k deques, power-of-two capacity, 1..64 items per chunk");
        return HCLIB_HIP_EINVAL;
    }
    // capacity is counted in ITEMS: `cap` slots hold cap * 64 items at the
    // full chunk, so a smaller chunk gets proportionally more slots (a
    // smaller HCLIB_HIP_CHUNK must not shrink what the frontier can spill to)
    for (uint32_t c = chunk; c * 2 <= 64; c *= 2) cap *= 2;
    const size_t hdr = sizeof(QueueHdr) * nq;
    const size_t slots = (size_t)nq * cap;
    const size_t need = hdr + slots * 4 * 2 + slots * chunk * words * 4 + 4096;
    Module &m = g_mod;
    if (need > m.pool_bytes) {
        if (m.pool_mem) (void)hipFree(m.pool_mem);
        m.pool_mem = nullptr;
        m.pool_bytes = 0;
        if (hipMalloc(&m.pool_mem, need) != hipSuccess) {
            set_error("hipMalloc(%zu) for the chunk deques failed", need);
            return HCLIB_HIP_ENOMEM;
        }
        m.pool_bytes = need;
    }
    char *p = (char *)m.pool_mem;
    out->hdr = (QueueHdr *)p;
    p += hdr;
    // {seq, cnt} pairs, 8-B aligned (hx_sched.h slot_ctl); cnt = seq + 1
    out->seq = (uint32_t *)p;
    out->cnt = out->seq + 1;
    p += slots * 8;
    p = (char *)(((uintptr_t)p + 255) & ~(uintptr_t)255);
    out->data = (uint32_t *)p;
    out->nq = nq;
    out->cap = cap;
    out->chunk = chunk;
    return HCLIB_HIP_OK;
}

// Host -> device copies of temporaries travel through pinned staging
// buffers: an asynchronous copy from pageable memory may read its source
// after the call returns (observed: a forasync sweep reading a stale run
// table from stream-ordered memory), so the source must live until the
// copy is done. Each buffer is freed once the event recorded
// after its copy has completed (checked on every upload).
struct Staged {
    void *host;
    hipEvent_t done;
};
std::vector<Staged> &staged() {
    static std::vector<Staged> v;
    return v;
}
void reap_staged() {
    std::vector<Staged> &v = staged();
    for (size_t i = 0; i < v.size();) {
        if (hipEventQuery(v[i].done) == hipSuccess) {
            (void)hipHostFree(v[i].host);
            (void)hipEventDestroy(v[i].done);
            v[i] = v.back();
            v.pop_back();
        } else {
            ++i;
        }
    }
}
// copy `bytes` of `src` to device `dst` in `st` order; src may be freed on return
int upload_async(void *dst, const void *src, size_t bytes, hipStream_t st) {
    reap_staged();
    void *pin = nullptr;
    HX_HIP(hipHostMalloc(&pin, bytes, hipHostMallocDefault));
    memcpy(pin, src, bytes);
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipHostFree(pin);
        set_error("upload: hipEventCreate failed");
        return HCLIB_HIP_EHIP;
    }
    if (hipMemcpyAsync(dst, pin, bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(ev, st) != hipSuccess) {
        (void)hipStreamSynchronize(st);
        (void)hipHostFree(pin);
        (void)hipEventDestroy(ev);
        set_error("upload: host-to-device copy failed");
        return HCLIB_HIP_EHIP;
    }
    staged().push_back(Staged{pin, ev});
    return HCLIB_HIP_OK;
}

int reset_sched(const PoolView &pool, uint32_t outstanding_init, bool global, uint32_t workers,
                const SeedCfg *seed) {
    Module &m = g_mod;
    HX_HIP(hipMemsetAsync(pool.hdr, 0, sizeof(QueueHdr) * pool.nq, m.stream));
    const uint32_t total = pool.nq * pool.cap;
    hipLaunchKernelGGL(k_reset_pool, dim3((total + 255) / 256), dim3(256), 0, m.stream, pool.seq,
                       pool.cap, total);
    HX_HIP(hipGetLastError());
    SchedGlobals init;
    memset(&init, 0, sizeof(init));
    init.outstanding = outstanding_init;
    init.wave_stats = m.wave_stats;
    init.wave_stats_cap = m.wave_stats_cap;
    m.rec_workers = workers < m.wave_stats_cap ? workers : m.wave_stats_cap;
    init.wave_ctr = m.rec_workers ? m.wave_ctr : nullptr;
    init.wave_ctr_cap = m.rec_workers;
    if (seed && seed->target && workers) {
        // level buffers: a level stops growing at `target` slots, the next one
        // is at most ~100x a node's... in practice b x target: 8 x target + slack
        const uint32_t cap = 8u * seed->target + 65536u;
        const size_t ctl = (size_t)kSeedCtlLines * 256;
        const size_t need = ctl + 2ull * cap * seed->words * 4;
        if (need > m.seed_bytes) {
            if (m.seed_mem) (void)hipFree(m.seed_mem);
            m.seed_mem = nullptr;
            m.seed_bytes = 0;
            HX_HIP(hipMalloc(&m.seed_mem, need));
            m.seed_bytes = need;
        }
        HX_HIP(hipMemsetAsync(m.seed_mem, 0, ctl, m.stream));
        init.seed.ctl = (uint32_t *)m.seed_mem;
        init.seed.buf = (uint32_t *)((char *)m.seed_mem + ctl);
        init.seed.cap = cap;
        init.seed.target = seed->target;
        init.seed.max_levels = seed->max_levels;
        init.seed.min_levels = seed->min_levels;
        init.seed.solo_cap = seed->solo_cap;
        init.outstanding = workers;  // every wave holds a unit until it has its share
    }
    if (global) init.gview = m.gview;
    // diagnostic timelines: only a HX_TIMELINE build writes them
    const int tl_cap = env_int("HCLIB_HIP_TIMELINE", 0);
    if (tl_cap > 0) {
        if (!m.timeline || (uint32_t)tl_cap != m.timeline_cap) {
            if (m.timeline) (void)hipFree(m.timeline);
            m.timeline = nullptr;
            HX_HIP(hipMalloc((void **)&m.timeline, (size_t)m.wave_stats_cap * tl_cap * 8));
            m.timeline_cap = (uint32_t)tl_cap;
        }
        HX_HIP(hipMemsetAsync(m.timeline, 0, (size_t)m.wave_stats_cap * tl_cap * 8, m.stream));
        init.timeline = m.timeline;
        init.timeline_cap = m.timeline_cap;
    }
    // a pinned staging copy of its own, reused: every launch ends with the
    // stream synchronised (hclib_hip_sched_end), so the last copy is done
    static SchedGlobals *stage = nullptr;
    if (!stage && hipHostMalloc((void **)&stage, sizeof(SchedGlobals), hipHostMallocDefault) != hipSuccess)
        return upload_async(m.globals, &init, sizeof(init), m.stream);
    *stage = init;
    HX_HIP(hipMemcpyAsync(m.globals, stage, sizeof(init), hipMemcpyHostToDevice, m.stream));
    return HCLIB_HIP_OK;
}

static const char *err_name(uint32_t e) {
    switch (e) {
    case kErrQueueFull: return "chunk deque full and LDS ring near capacity";
    case kErrStackOverflow: return "LDS ring overflow";
    case kErrSpinTimeout: return "idle spin timed out (no termination)";
    case kErrDepthTable: return "tree deeper than the device depth-rule table";
    case kErrArena: return "device arena exhausted";
    case kErrBadTask: return "malformed task";
    default: return "unknown device error";
    }
}

int finish_sched(SchedGlobals *host_copy, const char *who) {
    Module &m = g_mod;
    HX_HIP(hipMemcpyAsync(host_copy, m.globals, sizeof(SchedGlobals), hipMemcpyDeviceToHost,
                          m.stream));
    const uint32_t nw_cap = m.wave_stats_cap;
    // the workers' exit records (every worker of the grid writes its own)
    static std::vector<unsigned long long> rec;
    const uint32_t nrec = m.rec_workers;
    for (int i = 0; i < 8; ++i) m.last_phase[i] = 0;
    m.rec_workers = 0;
    if (nrec) {
        rec.resize((size_t)nrec * kWaveCtrWords);
        HX_HIP(hipMemcpyAsync(rec.data(), m.wave_ctr, rec.size() * 8, hipMemcpyDeviceToHost, m.stream));
    }
    HX_HIP(hipStreamSynchronize(m.stream));
    for (uint32_t w = 0; w < nrec; ++w) {
        const unsigned long long *r = &rec[(size_t)w * kWaveCtrWords];
        for (int i = 0; i < 16; ++i)
            if (i >= 8 || i < 4) host_copy->counters[i] += r[i];
        for (int i = 4; i < 8; ++i) host_copy->counters[i] += r[24 + i - 4];
        for (int i = 0; i < 4; ++i)
            if (r[16 + i] > host_copy->maxes[i]) host_copy->maxes[i] = r[16 + i];
        for (int i = 0; i < 3; ++i) host_copy->narrow[i] += r[20 + i];
        m.last_phase[0] += r[23];
        for (int i = 0; i < 4; ++i) m.last_phase[1 + i] += r[28 + i];
        m.last_phase[5] += r[24];  // HX_PHASES builds only (else the stamps' push cycles)
        m.last_phase[6] += r[27];
    }
    memcpy(m.last_counters, host_copy->counters, sizeof(m.last_counters));
    memcpy(m.last_narrow, host_copy->narrow, sizeof(m.last_narrow));
    // every wave of the grid leaves exactly once: counters[kCtrWaves] records
    uint64_t nw = host_copy->counters[kCtrWaves];
    if (nw > nw_cap) nw = nw_cap;
    m.last_waves.resize(nw);
    if (nw) HX_HIP(hipMemcpy(m.last_waves.data(), m.wave_stats, nw * sizeof(WaveStat), hipMemcpyDeviceToHost));
    if (host_copy->timeline) {
        m.last_timeline.resize((size_t)nw * m.timeline_cap);
        if (nw)
            HX_HIP(hipMemcpy(m.last_timeline.data(), m.timeline, (size_t)nw * m.timeline_cap * 8,
                             hipMemcpyDeviceToHost));
    } else {
        m.last_timeline.clear();
    }
    if (host_copy->err) {
        set_error("%s: device error %u (%s)", who, host_copy->err, err_name(host_copy->err));
        return HCLIB_HIP_EDEVICE;
    }
    return HCLIB_HIP_OK;
}

}  // namespace hx

using namespace hx;

extern "C" {

const char *hclib_hip_version(void) { return "hclib-mi355x 0.1 (gfx950 megakernel scheduler)"; }

const char *hclib_hip_last_error(void) { return g_err; }

int hclib_hip_init(int device) {
    Module &m = g_mod;
    if (m.inited) return HCLIB_HIP_OK;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_error("hclib_hip_init: no HIP device visible");
        return HCLIB_HIP_ENODEV;
    }
    if (device < 0 || device >= n) {
        set_error("hclib_hip_init: device %d out of range (%d devices)", device, n);
        return HCLIB_HIP_EINVAL;
    }
    HX_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    HX_HIP(hipGetDeviceProperties(&prop, device));
    m.arch = prop.gcnArchName;
    if (m.arch.rfind("gfx950", 0) != 0) {
        set_error("hclib_hip_init: device %d is %s, this module is built for gfx950 only", device,
                  prop.gcnArchName);
        return HCLIB_HIP_ENODEV;
    }
    m.device = device;
    m.num_cus = prop.multiProcessorCount;
    HX_HIP(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
    HX_HIP(hipEventCreate(&m.ev0));
    HX_HIP(hipEventCreate(&m.ev1));
    HX_HIP(hipMalloc((void **)&m.globals, sizeof(SchedGlobals)));
    m.wave_stats_cap = (uint32_t)m.num_cus * 32;  // 32 waves per CU at most
    HX_HIP(hipMalloc((void **)&m.wave_stats, sizeof(WaveStat) * m.wave_stats_cap));
    HX_HIP(hipMalloc((void **)&m.wave_ctr, 8ull * kWaveCtrWords * m.wave_stats_cap));
    m.inited = true;
    return HCLIB_HIP_OK;
}

void hclib_hip_finalize(void) {
    Module &m = g_mod;
    if (!m.inited) return;
    (void)hipStreamSynchronize(m.stream);
    if (m.pool_mem) (void)hipFree(m.pool_mem);
    (void)hipFree(m.globals);
    (void)hipFree(m.wave_stats);
    (void)hipFree(m.wave_ctr);
    if (m.seed_mem) (void)hipFree(m.seed_mem);
    if (m.timeline) (void)hipFree(m.timeline);
    (void)hipEventDestroy(m.ev0);
    (void)hipEventDestroy(m.ev1);
    (void)hipStreamDestroy(m.stream);
    m = Module();
}

int hclib_hip_num_cus(void) { return g_mod.inited ? g_mod.num_cus : 0; }

int hclib_hip_device(void) { return g_mod.inited ? g_mod.device : -1; }

void *hclib_hip_stream(void) { return g_mod.inited ? (void *)g_mod.stream : nullptr; }

void hclib_hip_last_sched_counters(uint64_t out[16]) {
    for (int i = 0; i < 16; ++i) out[i] = g_mod.last_counters[i];
}

// HX_PHASES builds: [0] main-loop single batches, [1..4] s_memtime cycles
// summed over them: loop top -> pop issued -> pop landed -> body -> batch end
extern "C" void hclib_hip_last_phase_counters(uint64_t out[8]) {
    for (int i = 0; i < 8; ++i) out[i] = g_mod.last_phase[i];
}

void hclib_hip_last_narrow_counters(uint64_t out[4]) {
    for (int i = 0; i < 4; ++i) out[i] = g_mod.last_narrow[i];
}

int hclib_hip_last_wave_stats(hclib_hip_wave_stats_t *out, int max) {
    static_assert(sizeof(hclib_hip_wave_stats_t) == sizeof(WaveStat), "layout");
    const int n = (int)g_mod.last_waves.size();
    for (int i = 0; out && i < n && i < max; ++i) memcpy(&out[i], &g_mod.last_waves[(size_t)i], sizeof(WaveStat));
    return n;
}

int hclib_hip_last_timeline(uint64_t *out, uint64_t max_words, uint32_t *events_per_worker) {
    Module &m = g_mod;
    if (events_per_worker) *events_per_worker = m.last_timeline.empty() ? 0u : m.timeline_cap;
    const uint64_t n = m.last_timeline.size();
    for (uint64_t i = 0; out && i < n && i < max_words; ++i) out[i] = m.last_timeline[i];
    return m.timeline_cap ? (int)(n / m.timeline_cap) : 0;
}

int hclib_hip_sched_begin(uint32_t entry_words, uint32_t chunk, int waves_per_cu,
                          hclib_hip_sched_launch_t *out) {
    if (!out || entry_words < 4 || entry_words > 64 || waves_per_cu < 1 || waves_per_cu > 8) {
        set_error("hclib_hip_sched_begin: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = g_mod;
    PoolView pool;
    HX_TRY(make_pool((uint32_t)env_int("HCLIB_HIP_DEQUES", 64), (uint32_t)env_int("HCLIB_HIP_DEQUE_CAP", 4096),
                     chunk, entry_words, &pool));
    HX_TRY(reset_sched(pool, 1, false, (uint32_t)(m.num_cus * waves_per_cu)));
    HX_HIP(hipEventRecord(m.ev0, m.stream));
    out->hdr = pool.hdr;
    out->seq = pool.seq;
    out->cnt = pool.cnt;
    out->data = pool.data;
    out->nq = pool.nq;
    out->cap = pool.cap;
    out->chunk = pool.chunk;
    out->globals = m.globals;
    out->stream = m.stream;
    out->grid = m.num_cus * waves_per_cu;
    out->num_cus = m.num_cus;
    return HCLIB_HIP_OK;
}

int hclib_hip_sched_end(const char *who, uint64_t counters[16], uint64_t maxes[4], double *kernel_ms) {
    Module &m = g_mod;
    if (!m.inited) {
        set_error("hclib_hip_sched_end: no device");
        return HCLIB_HIP_ENODEV;
    }
    HX_HIP(hipGetLastError());
    HX_HIP(hipEventRecord(m.ev1, m.stream));
    SchedGlobals gl;
    const int rc = finish_sched(&gl, who ? who : "hclib_hip_sched_end");
    float ms = 0;
    (void)hipEventElapsedTime(&ms, m.ev0, m.ev1);
    if (kernel_ms) *kernel_ms = ms;
    for (int i = 0; counters && i < 16; ++i) counters[i] = gl.counters[i];
    for (int i = 0; maxes && i < 4; ++i) maxes[i] = gl.maxes[i];
    return rc;
}

int hclib_hip_num_workers(void) {
    if (!g_mod.inited) return 0;
    return g_mod.num_cus * env_int("HCLIB_HIP_WAVES_PER_CU", 4);
}

}  // extern "C"

// ------------------------------------------------- cross-GPU work sharing
// One region (GlobalHdr + cap {seq, cnt} pairs + cap chunk payloads) in one
// rank's HBM, mapped into every other rank's process over IPC
// (hclib_hip_ipc_export / _import); every sharded UTS launch of a rank that
// attached it shares work through it (hx_sched.h GlobalView).
static size_t global_layout(uint32_t cap, size_t *ctl_off, size_t *data_off) {
    const size_t words = 64 * 8;  // a chunk: up to 64 entries of 8 words (UTS, fib)
    const size_t hdr = (sizeof(GlobalHdr) + 255) & ~(size_t)255;
    const size_t ctl = ((size_t)cap * 8 + 255) & ~(size_t)255;
    *ctl_off = hdr;
    *data_off = hdr + ctl;
    return hdr + ctl + (size_t)cap * words * 4;
}

extern "C" size_t hclib_hip_global_bytes(uint32_t cap) {
    size_t a, b;
    if (cap < 2 || (cap & (cap - 1))) return 0;
    return global_layout(cap, &a, &b);
}

__global__ void k_reset_global(uint32_t *ctl, uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap) {
        ctl[2 * i] = i;
        ctl[2 * i + 1] = 0;
    }
}

extern "C" int hclib_hip_global_init(void *region, uint32_t cap, int nranks) {
    if (!region || cap < 2 || (cap & (cap - 1)) || nranks < 1 || nranks > kGlobalMaxRanks) {
        set_error("hclib_hip_global_init: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = g_mod;
    size_t co, dof;
    global_layout(cap, &co, &dof);
    HX_HIP(hipMemsetAsync(region, 0, co, m.stream));
    hipLaunchKernelGGL(k_reset_global, dim3((cap + 255) / 256), dim3(256), 0, m.stream,
                       (uint32_t *)((char *)region + co), cap);
    HX_HIP(hipGetLastError());
    // every rank starts holding its shard's top levels: active = ranks, and
    // each rank's handshake word says it holds its unit
    const uint32_t active = (uint32_t)nranks;
    uint32_t held[kGlobalMaxRanks];
    for (int r = 0; r < kGlobalMaxRanks; ++r) held[r] = r < nranks ? 1u : 0u;
    HX_HIP(hipMemcpyAsync(region, &active, 4, hipMemcpyHostToDevice, m.stream));
    HX_HIP(hipMemcpyAsync((char *)region + offsetof(GlobalHdr, held), held, sizeof(held), hipMemcpyHostToDevice,
                          m.stream));
    HX_HIP(hipStreamSynchronize(m.stream));
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_global_attach(void *region, uint32_t cap, int rank) {
    HX_TRY(ensure_device());
    Module &m = g_mod;
    if (!region) {
        m.gview = GlobalView{nullptr, nullptr, nullptr, 0, 0};
        return HCLIB_HIP_OK;
    }
    if (cap < 2 || (cap & (cap - 1)) || rank < 0 || rank >= kGlobalMaxRanks) {
        set_error("hclib_hip_global_attach: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    size_t co, dof;
    global_layout(cap, &co, &dof);
    m.gview.hdr = (GlobalHdr *)region;
    m.gview.ctl = (uint32_t *)((char *)region + co);
    m.gview.data = (uint32_t *)((char *)region + dof);
    m.gview.cap = cap;
    m.gview.rank = (uint32_t)rank;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_global_read(const void *region, uint64_t out[3 + 2 * kGlobalMaxRanks]) {
    if (!region || !out) {
        set_error("hclib_hip_global_read: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    GlobalHdr h;
    HX_HIP(hipMemcpy(&h, region, sizeof(h), hipMemcpyDeviceToHost));
    out[0] = h.active;
    out[1] = h.idle;
    out[2] = h.tail - h.head;
    for (int i = 0; i < 2 * kGlobalMaxRanks; ++i) out[3 + i] = h.moved[i];
    return HCLIB_HIP_OK;
}

// The region's memory: uncached device memory (kind 0: every access, local
// or over xGMI, goes to the owner's HBM, the coherence a region that several
// GPUs update inside their kernels needs), fine-grained (kind 1) or plain
// coarse-grained hipMalloc (kind 2, coherent at system scope on one GPU).
// Allocated here rather than through a caching allocator so the IPC handle
// names exactly this allocation (no sub-allocation offset).
extern "C" int hclib_hip_global_alloc(uint32_t cap, int kind, void **region_out) {
    size_t co, dof;
    if (!region_out || cap < 2 || (cap & (cap - 1)) || kind < 0 || kind > 2) {
        set_error("hclib_hip_global_alloc: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    *region_out = nullptr;
    HX_TRY(ensure_device());
    const size_t bytes = global_layout(cap, &co, &dof);
    if (kind == 2) {
        HX_HIP(hipMalloc(region_out, bytes));
    } else {
        HX_HIP(hipExtMallocWithFlags(region_out, bytes,
                                     kind == 0 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    }
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_global_free(void *region) {
    if (!region) return HCLIB_HIP_OK;
    HX_TRY(ensure_device());
    HX_HIP(hipFree(region));
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_ipc_export(void *dev_ptr, void *handle_out) {
    if (!dev_ptr || !handle_out) {
        set_error("hclib_hip_ipc_export: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    hipIpcMemHandle_t h;
    HX_HIP(hipIpcGetMemHandle(&h, dev_ptr));
    memcpy(handle_out, &h, sizeof(h));
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_ipc_import(const void *handle, void **dev_ptr_out) {
    if (!handle || !dev_ptr_out) {
        set_error("hclib_hip_ipc_import: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    HX_HIP(hipIpcOpenMemHandle(dev_ptr_out, h, hipIpcMemLazyEnablePeerAccess));
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_ipc_close(void *dev_ptr) {
    HX_TRY(ensure_device());
    HX_HIP(hipIpcCloseMemHandle(dev_ptr));
    return HCLIB_HIP_OK;
}
