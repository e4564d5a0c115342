// hx_module.h — host-side state of the MI355X `modules/hip` plug-in.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/hclib_hip.h"
#include "../../include/hclib_hip/hx_sched.h"

namespace hx {

// Per-process module state (one bound device per process, like one rank
// per GPU in the multi-GPU launch).
struct Module {
    bool inited = false;
    int device = -1;
    int num_cus = 0;
    std::string arch;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // chunk-deque arena, sized for the largest entry type, reused by launches
    void *pool_mem = nullptr;
    size_t pool_bytes = 0;
    SchedGlobals *globals = nullptr;
    unsigned long long last_counters[16] = {};  // counters of the last megakernel launch
    unsigned long long last_narrow[4] = {};     // SchedGlobals::narrow of the last launch
    unsigned long long last_phase[8] = {};      // HX_PHASES builds (hclib_hip_last_phase_counters)
    // per-wave records of megakernel launches (WaveStat, hx_sched.h)
    WaveStat *wave_stats = nullptr;
    uint32_t wave_stats_cap = 0;
    std::vector<WaveStat> last_waves;  // the last launch's, copied back by finish_sched
    // per-worker exit records (hx_sched.h kWaveCtrWords), summed by finish_sched
    unsigned long long *wave_ctr = nullptr;
    // breadth-first seeding arena (two level buffers + control lines)
    void *seed_mem = nullptr;
    size_t seed_bytes = 0;
    uint32_t rec_workers = 0;  // records the running launch writes
    // cross-GPU work sharing (hclib_hip_global_attach): the shared region's
    // view for sharded launches, hdr null while detached
    GlobalView gview = {nullptr, nullptr, nullptr, 0, 0};
    // diagnostic worker timelines (HX_TIMELINE builds, HCLIB_HIP_TIMELINE=<events per worker>)
    unsigned long long *timeline = nullptr;
    uint32_t timeline_cap = 0;
    std::vector<unsigned long long> last_timeline;  // the last launch's, workers * timeline_cap
};

Module &mod();
void set_error(const char *fmt, ...);
int ensure_device();  // HCLIB_HIP_OK or HCLIB_HIP_ENODEV
int hip_check(hipError_t e, const char *what);
// A persistent launch (every worker waits for every other one to end) must
// fit the chip at once: HCLIB_HIP_EINVAL, with the numbers, when `blocks`
// workgroups of `threads` (and `lds` dynamic bytes) cannot all be resident
int check_resident(const void *kern, int blocks, int threads, size_t lds, const char *what);
// host -> device copy of `bytes` at `src` in `stream` order through a pinned
// staging buffer: `src` may be freed as soon as the call returns
int upload_async(void *dst, const void *src, size_t bytes, hipStream_t stream);

// Carve a PoolView for `words` u32 per entry out of the arena (grows it).
int make_pool(uint32_t nq, uint32_t cap, uint32_t chunk, uint32_t words, PoolView *out);
// Reset the deques and the globals on the module stream before a launch.
// `workers`: the launch's worker count (its exit records are summed by
// finish_sched); 0 = exit counts as atomics only
// `seed` (optional): breadth-first seeding of the launch (hx_sched.h
// seed_levels) with this many slots per level before the share-out, entries
// of `seed_words` u32; outstanding then starts at `workers`
struct SeedCfg {
    uint32_t target, max_levels, words, min_levels;
    uint32_t solo_cap = 0;  // hx_sched.h Seed::solo_cap
};
int reset_sched(const PoolView &pool, uint32_t outstanding_init, bool global = false, uint32_t workers = 0,
                const SeedCfg *seed = nullptr);
// Read back globals and translate the device error word.
int finish_sched(SchedGlobals *host_copy, const char *who);

// Environment knobs (HCLIB_HIP_WAVES_PER_CU, ...) with defaults.
int env_int(const char *name, int dflt);

}  // namespace hx

#define HX_TRY(expr)                         \
    do {                                     \
        int _rc = (expr);                    \
        if (_rc != HCLIB_HIP_OK) return _rc; \
    } while (0)
#define HX_HIP(call) HX_TRY(::hx::hip_check((call), #call))
