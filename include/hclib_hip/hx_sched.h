// hx_sched.h — the persistent work-stealing megakernel (device side).
//
// Replaces HClib's pthread worker loop and deques (src/hclib-runtime.c:646-729
// core_work_loop/find_and_run_task, src/hclib-deque.c:50-139) with a
// wavefront-granular scheduler:
//
//   worker        = one 64-lane wave (one workgroup of 64 threads), resident
//                   for the whole launch; a few per SIMD.
//   local deque   = a ring of task items in the wave's LDS (the "LDS-cached
//                   hot end"); the owner pushes/pops at the top (LIFO,
//                   work-first like ss_get_work, test/uts/UTS.cpp:383-402).
//   spill/steal   = the oldest items of a ring (the shallowest, largest
//                   subtrees) move as one chunk into an HBM chunk deque
//                   (bounded MPMC ring, eight per XCD); idle waves take
//                   chunks from their own XCD's deques first, then the last
//                   deque pushed to, then anywhere — the reference's
//                   intra-socket-first victim order
//                   (src/hclib-locality-graph.c:864-884) mapped to XCDs.
//   a "task"      = one ring item = one lane of a batch. An item is a range
//                   [k, kend) of the children of a task template (the
//                   parent); running it spawns child k. A task with c
//                   children is pushed as min(c, kPieces) range items, so a
//                   batch is simply the top min(size, 64) items. A lane
//                   whose item still holds children k+1.. re-pushes that
//                   residual range split in two (wide nodes such as the
//                   2000-child T3L root fan out by doubling).
//   ring layout   = two LDS planes: an 8-byte descriptor per item {k, kend,
//                   delta} and the task template, stored ONCE per group of
//                   pieces at the group's first position (delta = distance
//                   back to it). One wave's LDS write instructions cost
//                   ~100 cycles each whatever their lane count, so the push
//                   is one scattered template store plus lane-contiguous
//                   descriptor stores (one per 64 pushed items), the lane ->
//                   group mapping coming from a tagged mark + DPP max-scan.
//   termination   = `outstanding` = chunks in deques + waves holding work;
//                   the launch ends when it reads 0 (the finish counter of
//                   src/hclib-runtime.c:431-446 for the whole launch).
//   hunger        = waves - outstanding = waves with neither work nor a
//                   queued chunk to take; a wave gives away its oldest
//                   items only while that is > 0 (no chunk floods).
//
// All cross-wave words use agent-scope atomics; chunk payloads are written
// with sc1 stores and published behind s_waitcnt, consumed with sc1 loads
// (hx_common.h). Every spin is bounded.
#pragma once

#include <type_traits>

#include "hx_common.h"

namespace hx {

constexpr int kWaveSize = 64;

// One HBM chunk deque header, head and tail on separate 128-B lines. `done`
// shares the head's 8 bytes: the wave that ends the launch (its decrement
// takes `outstanding` to 0) sets it in every header, so an idle wave learns
// of termination from the head load of its next probe instead of polling the
// one `outstanding` line that every busy wave's spills and hunger reads use.
struct alignas(256) QueueHdr {
    uint32_t head;
    uint32_t done;
    uint32_t pad0[30];
    uint32_t tail;
    uint32_t pad1[31];
};

// One wave's scheduler statistics, written by the wave itself when it
// leaves the megakernel (the HCLIB_STATS per-worker record of
// src/hclib-runtime.c:83-104 with the device's vocabulary): items executed
// (one lane of a batch = one task run), tasks spawned (children created),
// batches, chunks it pushed to / took from the HBM deques, the items in the
// chunks it took, and which XCD's deques those chunks came from.
struct WaveStat {
    unsigned long long executed, spawned, batches, chunks_pushed, chunks_stolen, items_stolen;
    unsigned long long xcd;                 // XCD the wave ran on
    unsigned long long reserved;
    unsigned long long stolen_from[8];      // chunks taken from each XCD's deques
};
static_assert(sizeof(WaveStat) == 128, "WaveStat is 16 words");

// Cross-GPU work sharing (one process per GPU; SURVEY §8e items 2-3, the
// reference's distributed UTS moves work between ranks, test/performance-
// regression/full-apps/uts/uts_hclib_shmem_opt.cpp:98-140). One region in one
// rank's HBM, mapped by every rank (IPC), every word system-scope:
//   active  = ranks holding work + chunks queued in the global ring; the
//             launch of EVERY rank ends when it reads 0 (the termination
//             count the reference's ranks reach by messages)
//   idle    = ranks with no local work: the global hunger signal
//   a bounded MPMC ring of chunks (the local deques' slot format).
// A rank counts as holding work while its local `outstanding` is non-zero:
// the wave that takes it to 0 releases the rank's unit of `active`, a wave
// that takes it from 0 (only a global steal can) re-acquires it before it
// gives back the stolen chunk's unit, so `active` never reads 0 early.
struct alignas(256) GlobalHdr {
    uint32_t active;
    uint32_t pad0[63];
    uint32_t idle;
    uint32_t pad1[63];
    uint32_t head;
    uint32_t pad2[63];
    uint32_t tail;
    uint32_t pad3[63];
    uint32_t err;  // first DevError any rank hit in the shared protocol: every rank stops
    uint32_t pad4[63];
    unsigned long long moved[32];  // [2r] chunks rank r exported, [2r+1] chunks it imported
    // per rank: 1 while the rank holds its unit of `active`, 0 once a release
    // (idle += 1 included) has landed; the import that takes the unit back
    // waits for 0, so its idle -= 1 never runs ahead of the release's
    // idle += 1 (`idle` cannot underflow; tests/model/global_sharing_model.c)
    uint32_t held[16];
};
constexpr int kGlobalMaxRanks = 16;

struct GlobalView {
    GlobalHdr *hdr;  // null: this launch shares nothing
    uint32_t *ctl;   // cap {seq, cnt} pairs (slot_ctl layout)
    uint32_t *data;  // cap * chunk * words
    uint32_t cap;    // slots (power of two)
    uint32_t rank;
};

// Global scheduler state shared by all waves of one launch (device memory).
struct alignas(256) SchedGlobals {
    uint32_t outstanding;  // chunks queued + waves holding work
    uint32_t pad0[63];
    uint32_t hint;  // (unused; per-XCD hints below)
    uint32_t pad1[63];
    // per XCD x, hints[64 x]: the deque most recently pushed to in x's slice
    // (eight lines, so idle waves' hint reads do not all hit one line)
    uint32_t hints[8 * 64];
    uint32_t err;  // DevError
    uint32_t pad2[63];
    unsigned long long counters[16];  // [0..7] kind-specific, [8..15] scheduler
    unsigned long long maxes[4];      // kind-specific reductions (atomic max)
    WaveStat *wave_stats;             // per-wave records (indexed by blockIdx.x), or null
    uint32_t wave_stats_cap;          // records available
    unsigned long long narrow[4];     // narrow-frontier loop: [0] batches, [1] s_memtime cycles, [2] entries
    GlobalView gview;                 // cross-GPU work sharing (gview.hdr null: off)
    // diagnostic timeline (HX_TIMELINE builds, HCLIB_HIP_TIMELINE=1): per
    // worker `timeline_cap` events of lane 0 (see Timeline), or null
    unsigned long long *timeline;
    uint32_t timeline_cap;
    // per-worker exit records (kWaveCtrWords u64 each, plain stores; the
    // host sums them into counters / maxes / narrow, finish_sched), or null:
    // then the exit counts are agent atomics on the lines above. Thousands
    // of workers adding ~15 counts each to two lines serialised 100-250 us
    // of every launch's exit (worker timelines, profiles/r04)
    unsigned long long *wave_ctr;
    uint32_t wave_ctr_cap;
    // breadth-first seeding of the launch (see seed_levels), or buf null
    struct Seed {
        uint32_t *buf;         // two level buffers of `cap` entries, kWords u32 each
        uint32_t *ctl;         // kSeedCtlLines lines of 64 words (see seed_levels)
        uint32_t cap;          // entries per level buffer
        uint32_t target;       // distribute once a level holds at least this many entries
        uint32_t max_levels;   // ... or after this many levels
        uint32_t min_levels;   // ... but not before this many (a sharded search: past its split)
        uint32_t solo_cap;     // wave 0 runs levels of at most this many slots alone (0: the ring's room)
    } seed;
};
constexpr int kSeedMaxLevels = 24;
constexpr int kSeedGoLines = 64;  // "level d is complete" broadcast lines (a wave polls line gid % 64)
constexpr int kSeedCtlLines = 2 * kSeedMaxLevels + 2 + kSeedGoLines;
// a worker's exit record: [0..7] the kind's counters, [8..15] the
// scheduler's counters (SchedGlobals::counters [8..15]; [4..7] of the
// diagnostic stamps go to [24..27]), [16..19] the kind's maxima, [20..22]
// the narrow-loop counts
constexpr int kWaveCtrWords = 32;

// Diagnostic build (-DHX_TIMELINE=1, `python -m hclib_amd.build --variant
// timeline`): every worker logs its transitions — start, busy (work taken),
// idle, chunk given away, termination seen, exit — as
// s_memrealtime (100 MHz) << 24 | type << 20 | value (20 bits), so the host
// can draw the active-worker count against time (scripts/uts_timeline.py).
// Transitions are rare (never per batch), so the log costs the search
// little; the product build compiles it out.
#ifndef HX_TIMELINE
#define HX_TIMELINE 0
#endif
enum : uint32_t {
    kTlStart = 1,  // value: 0
    kTlBusy = 2,   // value: items taken | source << 16 (0 roots, 1 home deque, 2 other deque, 3 inbox, 4 global)
    kTlIdle = 3,   // value: 0
    kTlSpill = 4,  // value: items given away (a chunk or an inbox)
    kTlTerm = 5,   // value: 0 — this worker saw the launch's termination
    kTlEnd = 6,    // value: 0 — after the exit reductions
    kTlProbe = 7,  // value: probe statistics at exit, (kind << 16) | count / 16 (saturating):
                   // kind 0 probes, 1 empty deques seen, 2 lost head CASes, 3 publish waits (x1 us)
    kTlSeed = 8,   // value: the seeding level this worker has just seen complete
};
struct Timeline {
    unsigned long long *p;
    uint32_t n, cap;
    __device__ __forceinline__ void init(SchedGlobals *g, uint32_t worker) {
#if HX_TIMELINE
        cap = g->timeline_cap;
        p = g->timeline ? g->timeline + (size_t)worker * cap : nullptr;
        n = 0;
#endif
    }
    __device__ __forceinline__ void log(uint32_t type, uint32_t value) {
#if HX_TIMELINE
        if (p && n < cap && lane_id() == 0)
            p[n] = ((unsigned long long)__builtin_amdgcn_s_memrealtime() << 24) | ((unsigned long long)type << 20) |
                   (value & 0xfffffu);
        ++n;
#endif
    }
};

// Diagnostic build (-DHX_STAMPS=1): per-phase s_memtime stamps, enabled at run
// time by HCLIB_HIP_STAMPS=1. Each stamp waits for the batch's LDS traffic,
// so the product build compiles them out of the hot loop.
#ifndef HX_STAMPS
#define HX_STAMPS 0
#endif

// scheduler counters (SchedGlobals::counters)
enum : int {
    kCtrPushCycles = 4,   // diagnostic stamps: pushing the batch's outputs
    kCtrClockTicks = 5,   // s_memtime ticks over each wave's lifetime (clock calibration)
    kCtrRealTicks = 6,    // s_memrealtime (100 MHz) ticks over the same span
    kCtrFormCycles = 7,   // diagnostic stamps: batch formation (scans, LDS map)
    kCtrProcCycles = 8,   // diagnostic stamps: Kind::process over the batch
    kCtrBusyCycles = 9,   // s_memtime cycles inside batches (all waves)
    kCtrIdleCycles = 10,  // s_memtime cycles idle / stealing
    kCtrSpillCycles = 11, // cycles inside enqueue
    kCtrWaves = 12,
    kCtrBatches = 13,
    kCtrPushed = 14,
    kCtrStolen = 15,
};

struct PoolView {
    QueueHdr *hdr;    // nq headers
    uint32_t *seq;    // nq * cap sequence words
    uint32_t *cnt;    // nq * cap entry counts
    uint32_t *data;   // nq * cap * chunk * words
    uint32_t nq;      // number of deques (multiple of 8)
    uint32_t cap;     // slots per deque (power of two)
    uint32_t chunk;   // entries per chunk (<= 64)
};

struct SchedConfig {
    uint32_t spill_hi;   // always spill above this many entries (ring capacity valve)
    uint32_t spill_lo;   // give away entries to hungry waves when holding >= this many
    uint32_t spin_limit; // ms a wave may stay idle before declaring a timeout
    uint32_t nwaves;     // waves in the launch (hunger = nwaves - outstanding)
    uint32_t stamps;     // diagnostic: accumulate per-phase s_memtime cycles
    uint32_t hunger;     // batches between reads of the hunger signal (0: never give work
                         // away unless the ring is full)
    uint32_t backoff = 16;  // longest idle s_sleep (1, 4 or 16 units of 64 clocks)
    uint32_t carry = 2;  // keep a uniform batch's outputs in registers as the next batch
                         // (no ring push / pop) while they fit one batch and no hungry
                         // wave could take them (see run_worker); 2 also runs narrow
                         // frontiers in a tight carry-to-carry loop, 1 does not
    uint32_t defer = 1;  // a hunger spill's chunk is published after the next batch body
                         // (PendingChunk) instead of behind a store round trip
    uint32_t dual = 1;   // kinds with process2 (KindDual): a wave holding more than 64
                         // items runs TWO per lane per batch, their bodies interleaved
    uint32_t spills = 0; // hunger spills per batch at most (0: until the ring is below
                         // spill_lo or no wave is hungry)
    // a seeded launch's first batches run before any hunger read has landed:
    // 0 = they see every wave hungry (an early rebalancing of the seeded
    // shares, from spill_lo items), 1 = they see none hungry (every wave holds
    // its share)
    uint32_t hunger_init_full = 0;
};

// Kind concept:
//   static constexpr int kTmplWords;  // 2 or 6 u32 words of task template
//   static constexpr int kWords;      // kTmplWords + 2: an item as a chunk
//                                     // payload {template, k, kend}
//   struct Ctx;                       // per-launch read-only parameters
//   struct Acc { ...; __device__ void flush(SchedGlobals*); };  // per-lane stats
//        (optional, in place of flush: __device__ void totals(unsigned long long
//        (&c)[8], unsigned long long (&m)[4]) — the wave's sums / maxima,
//        wave-uniform, which the scheduler stores in the worker's exit record
//        instead of adding them to SchedGlobals::counters / maxes atomically)
//   __device__ static int process(const Ctx&, Acc&, const uint32_t *tmpl, uint32_t k,
//                                 uint32_t *child_tmpl, uint32_t *err);
//        run child k of `tmpl`; return the number of children of the new
//        task (0: nothing to push), whose template it wrote to child_tmpl
//   __device__ static int roots(const Ctx&, Acc&, uint32_t *tmpl);  // wave 0 only
//   static constexpr bool kPure;      // process() touches nothing but Acc: the
//                                     // batch runs branch-free on all 64 lanes
//                                     // (process gets `valid`; invalid lanes'
//                                     // results are dropped)
//   static constexpr bool kBoundedChildren;  // process() never returns >= kMaxChildren
//   optional, pure kinds only:
//   __device__ static void process2(const Ctx&, Acc&, const uint32_t *tmplA, uint32_t kA,
//                                   uint32_t *childA, int &ncA, const uint32_t *tmplB,
//                                   uint32_t kB, uint32_t *childB, int &ncB, uint32_t *err,
//                                   bool validB);
//        two items in one lane, their bodies interleaved (independent
//        dependency chains fill each other's issue slots: a dependent chain of
//        one wave issues a VALU op only every ~4-5 cycles of the 2 it needs)

// Range items one task's children are pushed as (Kind::kPieces, default 8):
// a task with c children becomes min(c, pieces) items. Fewer pieces need a
// smaller ring (one batch pushes at most 64 * (pieces + 2) items), so a
// kind with wide nodes can trade residual splitting for LDS, i.e. for more
// resident waves per CU.
// A popped range item's residual (children k+1..kend-1) goes back as two
// halves, a wide node's children spread over more batches sooner (as one
// whole item: T1XL 37.4 -> 39.2 ms, profiles/r02/residual_ab.log); a residual
// of one child stays whole (keeping 3-4 whole was even, 8 slower:
// residual_split_ab.log)
constexpr uint32_t kResidualSplitMin = 2;

// a Kind's seeding slots run Kind::seed_process when it has one (UTS: the
// shard filter at the split depth, which the seeding passes), else process
template <class K, class = void>
struct KindHasSeedProcess {
    static constexpr bool value = false;
};
template <class K>
struct KindHasSeedProcess<K, decltype((void)&K::seed_process)> {
    static constexpr bool value = true;
};
template <class K>
__device__ __forceinline__ int kind_seed_process(const typename K::Ctx &c, typename K::Acc &acc, const uint32_t *t,
                                                 uint32_t k, uint32_t *child, uint32_t *err, bool valid) {
    if constexpr (KindHasSeedProcess<K>::value) return K::seed_process(c, acc, t, k, child, err, valid);
    else return K::process(c, acc, t, k, child, err, valid);
}

template <class K, class = void>
struct KindPieces {
    static constexpr int value = 8;
};
template <class K>
struct KindPieces<K, decltype((void)K::kPieces)> {
    static constexpr int value = K::kPieces;
};
template <class K>
constexpr int pieces_of() { return KindPieces<K>::value; }
template <class K, class = void>
struct KindHasDual {
    static constexpr bool value = false;
};
template <class K>
struct KindHasDual<K, decltype((void)&K::process2)> {
    static constexpr bool value = K::kPure;
};
template <class K>
constexpr int group_max_of() { return KindPieces<K>::value + 2; }  // items one lane pushes per batch
// Optional: static uint32_t fixed_children(const Ctx&) — every task has either
// no children or exactly this many (<= the Kind's pieces; UTS BIN trees: m):
// the narrow loop then skips its uniformity test and reads no group size
// (declared with static constexpr bool kFixedChildren = true; a return of 0
// or more than the pieces falls back to the general test)
template <class K, class = void>
struct KindFixedChildren {
    static constexpr bool value = false;
};
// Optional with kFixedChildren: static constexpr bool kBulkCount = true, a
// process_bulk (process without the per-lane task and leaf counts, returning
// whether the task spawns its fixed_children() children; called only while
// that count is > 0) and
// count_bulk(acc, tasks, leaves) — the fixed-size narrow loop then keeps
// those counts as wave-uniform sums and hands them over once at its exit
template <class K, class = void>
struct KindBulkCount {
    static constexpr bool value = false;
};
template <class K>
struct KindBulkCount<K, decltype((void)K::kBulkCount)> {
    static constexpr bool value = K::kBulkCount;
};
template <class K>
struct KindFixedChildren<K, decltype((void)K::kFixedChildren)> {
    static constexpr bool value = K::kFixedChildren;
};
constexpr uint32_t kMaxChildren = 1u << 24;  // kend shares its descriptor word with delta

// register carry through LDS (carry_lds) where the ring's stack has room,
// carry_permute elsewhere (through LDS: T3L 31.29 -> 30.59 ms,
// profiles/r04/carry_ab_t3l.log)
template <class Kind, int CAP>
struct WaveStack {
    static constexpr int TW = Kind::kTmplWords;
    static_assert(TW == 2 || TW == 6, "templates are 2 or 6 words");
    static_assert((CAP & (CAP - 1)) == 0, "CAP must be a power of two");
    uint2 d[CAP];                  // item descriptor {k, kend | delta << 24}
    uint4 t0[TW == 6 ? CAP : 1];   // template words 0..3 (6-word templates)
    uint2 t1[CAP];                 // template words 4..5 (or 0..1)
    uint32_t mark[64];             // tagged group-start marks of the transposed push
    uint32_t stolen_from[8];       // chunks this wave took from each XCD's deques
    // rarely-updated 64-bit sums kept out of the batch loop's SGPRs:
    // [0] busy cycles, [1] idle cycles, [2] spill cycles, [3] narrow-loop
    // cycles, [4] s_memtime at start, [5] s_memrealtime at start
    unsigned long long cyc[6];
    // register carry's template slots (carry_lds: 2 x 16 B per spawning
    // rank), on the 1,024-item rings only: the 512-item rings of the wide GEO
    // trees run 8 waves per CU, whose stacks then just fit the 160 KiB
    static constexpr bool kCarryLds = CAP >= 1024;
    uint4 cscr[kCarryLds ? 128 : 1];
};

// lane 0 adds to a per-wave LDS sum (no return value, no wait)
template <class WS>
__device__ __forceinline__ void lds_sum(WS &st, int i, unsigned long long v) {
    if (lane_id() == 0) __hip_atomic_fetch_add(&st.cyc[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

template <class Kind, int CAP>
__device__ __forceinline__ void load_tmpl(const WaveStack<Kind, CAP> &st, uint32_t slot, uint32_t *t) {
    if constexpr (Kind::kTmplWords == 6) {
        const uint4 a = st.t0[slot];
        const uint2 b = st.t1[slot];
        t[0] = a.x;
        t[1] = a.y;
        t[2] = a.z;
        t[3] = a.w;
        t[4] = b.x;
        t[5] = b.y;
    } else {
        const uint2 b = st.t1[slot];
        t[0] = b.x;
        t[1] = b.y;
    }
}
template <class Kind, int CAP>
__device__ __forceinline__ void store_tmpl(WaveStack<Kind, CAP> &st, uint32_t slot, const uint32_t *t) {
    if constexpr (Kind::kTmplWords == 6) {
        st.t0[slot] = make_uint4(t[0], t[1], t[2], t[3]);
        st.t1[slot] = make_uint2(t[4], t[5]);
    } else {
        st.t1[slot] = make_uint2(t[0], t[1]);
    }
}

// ------------------------------------------------------- DPP wave scans
// Inclusive scans over the 64 lanes with DPP row shifts and row broadcasts
// (GFX9 row_bcast:15/31), ~12 VALU ops, no LDS round trips.
__device__ __forceinline__ int wave_scan_add(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int wave_scan_max(int x) {  // identity -1 (x >= -1)
    x = imax(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xf, 0xf, false));
    x = imax(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xf, 0xf, false));
    x = imax(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xf, 0xf, false));
    x = imax(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xf, 0xf, false));
    x = imax(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xa, 0xf, false));
    x = imax(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xc, 0xf, false));
    return x;
}
__device__ __forceinline__ int lane63(int x) { return __builtin_amdgcn_readlane(x, 63); }

// Chunk hand-off. Every payload word is stored with an agent-scope (sc1,
// write-through) store and loaded with an agent-scope (sc1) load, so the
// form of MI355X_MICROARCH.md "Valid forms" applies: the producer drains
// its stores (s_waitcnt vmcnt(0)) before the sequence word, the consumer
// needs no L1 invalidate. HX_STRICT_HANDOFF=1 restores the release/acquire
// fences (diagnostic build).
#ifndef HX_STRICT_HANDOFF
#define HX_STRICT_HANDOFF 0
#endif
__device__ __forceinline__ void handoff_publish() {
#if HX_STRICT_HANDOFF
    release_agent();
#else
    vm_drain();
#endif
}
__device__ __forceinline__ void handoff_consume() {
#if HX_STRICT_HANDOFF
    acquire_agent();
#else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
#endif
}
__device__ __forceinline__ uint32_t lane0(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// Chunk slot control word pair {seq, cnt} (8 B, one atomic 64-bit load reads
// both): seq = pos when the slot is free for ticket pos, pos + 1 once that
// ticket's chunk is published (cnt = its item count, stored before the
// publish drain, so a load that sees the new seq sees the new cnt).
__device__ __forceinline__ uint32_t *slot_ctl(const PoolView &pool, uint32_t slot) { return pool.seq + 2u * slot; }

// A chunk whose payload is written but whose seq word is not yet stored: the
// producer publishes it after its next batch's body, when the payload stores
// have long landed (the drain is free there) instead of waiting a round trip
// for them while it holds the rest of its items.
struct PendingChunk {
    uint32_t slot, pos, q;
    bool live;
};

// Where a compiler barrier behind a batch body's results would go (so that
// the deferred publish and its drain stay after the body's arithmetic). It
// is empty: from round 5 until round 6 its guard macro was defined only
// after this function, so every measured build compiled it out, and the
// active barrier measured no better (profiles/r06/ab_afterbody.log)
template <int TW>
__device__ __forceinline__ void after_body(const uint32_t *child) {
    (void)child;
}

template <class Kind, int CAP>
__device__ __forceinline__ void publish_pending(const PoolView &pool, SchedGlobals *g, PendingChunk &pc) {
    if (!pc.live) return;
    handoff_publish();  // the payload + cnt stores are complete
    if (lane_id() == 0) {
        st_sc1_u32(slot_ctl(pool, pc.slot), pc.pos + 1);
        st_sc1_u32(&g->hints[64u * ((pc.q / (pool.nq / 8u)) & 7u)], pc.q);
    }
    pc.live = false;
}

// Optional Kind hook: static void export_item(const Ctx&, uint32_t *w, bool valid, uint32_t *err)
// — called by the whole wave for the items it is about to hand to another
// wave (a chunk, an inbox, the global ring; `w` = {template, k, kend},
// `valid` = the lane packs an item). A Kind whose templates name wave-local
// state (fib's LDS finish scopes, hx_finish.h LocalScopes) rewrites them to
// names every wave can use.
template <class K, class = void>
struct kind_has_export : std::false_type {};
template <class K>
struct kind_has_export<K, decltype((void)&K::export_item)> : std::true_type {};
template <class Kind>
__device__ __forceinline__ void kind_export(const typename Kind::Ctx &ctx, uint32_t *w, bool valid, uint32_t *err) {
    if constexpr (kind_has_export<Kind>::value) Kind::export_item(ctx, w, valid, err);
}

// Optional Kind hook (diagnostic traces): static void trace_item(const Ctx&,
// const uint32_t *w, bool valid, uint32_t ev) — called by the whole wave for
// items {template, k, kend} that change hands: ev 2 = given away (a chunk
// or an inbox; `via_inbox`), 3 = taken by the receiving wave
template <class K, class = void>
struct kind_has_trace_item : std::false_type {};
template <class K>
struct kind_has_trace_item<K, decltype((void)&K::trace_item)> : std::true_type {};
template <class Kind>
__device__ __forceinline__ void kind_trace_item(const typename Kind::Ctx &ctx, const uint32_t *w, bool valid,
                                                uint32_t ev, bool via_inbox) {
    if constexpr (kind_has_trace_item<Kind>::value) Kind::trace_item(ctx, w, valid, ev, via_inbox);
}

// Optional Kind hooks: static bool seeding(const Ctx&) and
// template <class WS> static uint32_t seed(const Ctx&, Acc&, WS &stack,
// uint32_t worker, uint32_t workers, uint32_t spin_ms, uint32_t *err) — the
// Kind expands its roots itself and leaves each worker's share in its ring
// (slots 0..n-1, each its own template, child 0); run by every wave of the
// launch in place of roots() when seeding() holds
template <class K, class = void>
struct kind_has_seed : std::false_type {};
template <class K>
struct kind_has_seed<K, decltype((void)&K::seeding)> : std::true_type {};

// Optional Kind hook: static void drain(const Ctx&, Acc&, uint32_t *err),
// called by the whole wave when its ring runs empty, before the wave counts
// itself idle: work the Kind left in flight across batches (fib's HBM
// check-outs, hx_finish.h finish_issue) must end before termination can.
template <class K, class = void>
struct kind_has_drain : std::false_type {};
template <class K>
struct kind_has_drain<K, decltype((void)&K::drain)> : std::true_type {};
template <class Kind>
__device__ __forceinline__ void kind_drain(const typename Kind::Ctx &ctx, typename Kind::Acc &acc, uint32_t *err) {
    if constexpr (kind_has_drain<Kind>::value) Kind::drain(ctx, acc, err);
}

// Try to publish `n` entries (ring positions bot..bot+n-1) as one chunk into
// deque q. Called by the whole wave; returns true if the chunk is placed.
// `occ`: the deque occupancy this wave saw at its last enqueue. While that
// is low, the ticket is taken at once (one fetch-add, the head read beside
// it refreshes `occ`); once it was high, the occupancy is read first and a
// ring at least half full is refused, so a ticket never waits behind a
// consumer that cannot come. With `defer`, the publish is deferred into `pc`
// (see PendingChunk); the caller must publish a live one before the next
// enqueue. (`pc` is a reference, never a pointer that may be null: a
// select between a local's address and null keeps the local in scratch
// memory, and every batch then read its `live` flag behind a vmcnt(0) wait.)
template <class Kind, int CAP>
__device__ bool enqueue_chunk(const typename Kind::Ctx &ctx, const PoolView &pool, SchedGlobals *g, uint32_t q,
                              WaveStack<Kind, CAP> &st, uint32_t bot, uint32_t n, uint32_t &occ, PendingChunk &pc,
                              bool defer, bool relief = false) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    QueueHdr *h = &pool.hdr[q];
    // lane i packs item bot+i as {template, k, kend} (n <= 64): its LDS reads
    // go out before the ticket's round trip, which then hides them
    const bool valid = (uint32_t)lane < n;
    uint32_t w[W];
    {
        const uint32_t p = bot + (valid ? (uint32_t)lane : 0u);
        const uint2 dd = st.d[p & (CAP - 1)];
        load_tmpl<Kind, CAP>(st, (p - (dd.y >> 24)) & (CAP - 1), w);
        w[W - 2] = dd.x;
        w[W - 1] = dd.y & (kMaxChildren - 1);
    }
    uint32_t pos = 0, seen = 0;
    int ok = 0;
    const bool fast = occ < pool.cap / 4;
    if (lane == 0) {
        if (fast) {
            add_agent(&g->outstanding, 1u);  // counts before it becomes visible
            pos = add_agent(&h->tail, 1u);
            seen = pos - ld_agent(&h->head);
            ok = 1;
        } else {
            const uint32_t hd = ld_agent(&h->head), tl = ld_agent(&h->tail);
            seen = tl - hd;
            // a ring-full relief may fill the deque to its last slot: a ticket
            // below head + cap waits only for a consumer that already claimed
            // the previous lap's ticket (no deadlock, a short bounded wait).
            // The ticket is taken by CAS on the tail it checked, so concurrent
            // producers cannot together push it past that bound
            if ((int)(tl - hd) < (int)(relief ? pool.cap - 1 : pool.cap / 2) && cas_agent(&h->tail, tl, tl + 1u)) {
                add_agent(&g->outstanding, 1u);  // before the chunk is published
                pos = tl;
                ok = 1;
            }
        }
    }
    occ = lane0(seen);
    if (!lane0((uint32_t)ok)) return false;
    pos = lane0(pos);
    const uint32_t slot = q * pool.cap + (pos & (pool.cap - 1));
    if (lane == 0) {
        // the slot is free once its previous lap was consumed (normally at once)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_agent(slot_ctl(pool, slot)) != pos) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                dev_error(&g->err, kErrQueueFull);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    uint32_t *dst = pool.data + (size_t)slot * pool.chunk * W;
    {
        kind_export<Kind>(ctx, w, valid, &g->err);
        kind_trace_item<Kind>(ctx, w, valid, 2u, false);
        if (valid) {
            if constexpr (W % 4 == 0) {
                // 16-byte sc1 stores (a dword sc1 store costs ~6x the bytes of
                // a dwordx4 one), written as inline asm, which the compiler's
                // waitcnt pass does not see: it would otherwise wait for them
                // (vmcnt(0), and so for every load issued since) before the
                // next batch reuses their data registers
#pragma unroll
                for (int i = 0; i < W; i += 4)
                    st_sc1_x4(&dst[(uint32_t)lane * W + i], make_uint4(w[i], w[i + 1], w[i + 2], w[i + 3]));
            } else {
#pragma unroll
                for (int i = 0; i < W; ++i) st_agent(&dst[(uint32_t)lane * W + i], w[i]);
            }
        }
    }
    if (lane == 0) st_sc1_u32(slot_ctl(pool, slot) + 1, n);
    if (defer) {
        pc.slot = slot;
        pc.pos = pos;
        pc.q = q;
        pc.live = true;
        return true;
    }
    handoff_publish();
    if (lane == 0) {
        st_sc1_u32(slot_ctl(pool, slot), pos + 1);
        st_sc1_u32(&g->hints[64u * ((q / (pool.nq / 8u)) & 7u)], q);
    }
    // nothing stays in flight past a spill (see vm_drain)
    vm_drain();
    return true;
}

// Try to take one chunk from deque q into the (empty) stack. Returns the
// number of entries taken (0 if the deque looked empty). Round trips: the
// head/tail read, the head CAS beside the {seq, cnt} pair's read, the
// payload; the slot is handed back with a store nobody waits for
// (profiles/r06/ab_seqcas.log: the pair after the CAS cost T3L 0.13 ms).
// `done` (wave-uniform) receives the header's termination flag.
// Probe statistics of an idle wave (HX_TIMELINE builds: logged at exit)
struct ProbeStats {
    uint32_t probes = 0, empty = 0, lost = 0, wait_us = 0;
};

template <class Kind, int CAP>
__device__ uint32_t dequeue_chunk(const typename Kind::Ctx &ctx, const PoolView &pool, uint32_t q, WaveStack<Kind, CAP> &st,
                                  SchedGlobals *g, uint32_t &done, ProbeStats &ps) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    QueueHdr *h = &pool.hdr[q];
    uint32_t pos = 0, fin = 0;
    int ok = 0, nonempty = 0;
    unsigned long long sc0 = 0;  // the claimed slot's {seq, cnt}, read beside the claim
    if (lane == 0) {
        // one claim attempt: a ticket below the tail, taken by CAS on the head
        const unsigned long long hd2 = ld_agent((const unsigned long long *)&h->head);
        const uint32_t hd = (uint32_t)hd2, tl = ld_agent(&h->tail);
        fin = (uint32_t)(hd2 >> 32);
        nonempty = (int)(tl - hd) > 0;
        if (nonempty) {
            // the slot's pair is read in the same round trip as the CAS: a
            // value that shows the ticket published was stored after its
            // payload had landed, whoever wins the claim
            sc0 = ld_agent((const unsigned long long *)slot_ctl(pool, q * pool.cap + (hd & (pool.cap - 1))));
            if (cas_agent(&h->head, hd, hd + 1)) {
                pos = hd;
                ok = 1;
            }
        }
    }
    done = lane0(fin);
    if (HX_TIMELINE) {
        ps.probes++;
        if (!lane0((uint32_t)nonempty)) ps.empty++;
        else if (!lane0((uint32_t)ok)) ps.lost++;
    }
    if (!lane0((uint32_t)ok)) return 0;
    pos = lane0(pos);
    const uint32_t slot = q * pool.cap + (pos & (pool.cap - 1));
    uint32_t cnt = 0;
    uint32_t waited = 0;
    if (lane == 0) {
        // the producer holds this ticket and is publishing it (bounded wait)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (bool first = true;; first = false) {
            const unsigned long long sc = first ? sc0 : ld_agent((const unsigned long long *)slot_ctl(pool, slot));
            if ((uint32_t)sc == pos + 1) {
                cnt = (uint32_t)(sc >> 32);
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                dev_error(&g->err, kErrSpinTimeout);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (HX_TIMELINE) waited = (uint32_t)((__builtin_amdgcn_s_memrealtime() - t0) / 100u);
    }
    if (HX_TIMELINE) ps.wait_us += lane0(waited);
    handoff_consume();
    // uniform (readfirstlane): the ring bounds derived from it stay in SGPRs,
    // so every scheduler branch and loop of the batch is scalar
    const uint32_t n = lane0(cnt);
    // lane i unpacks item i: its own template slot (delta 0)
    const uint32_t *src = pool.data + (size_t)slot * pool.chunk * W;
    if ((uint32_t)lane < n) {
        uint32_t w[W];
        if constexpr (W == 8) {
            uint4 a, b;
            ld_sc1_x4x2(&src[(uint32_t)lane * W], a, b);
            w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w, w[4] = b.x, w[5] = b.y, w[6] = b.z, w[7] = b.w;
        } else {
#pragma unroll
            for (int i = 0; i < W; ++i) w[i] = ld_agent(&src[(uint32_t)lane * W + i]);
        }
        store_tmpl<Kind, CAP>(st, (uint32_t)lane, w);
        st.d[lane] = make_uint2(w[W - 2], w[W - 1]);
        kind_trace_item<Kind>(ctx, w, true, 3u, false);
    }
    // all reads of the slot have landed before it is handed back
    vm_drain();
    if (lane == 0) st_sc1_u32(slot_ctl(pool, slot), pos + pool.cap);
    // one wave per workgroup: its LDS ops complete in issue order
    return n;
}

// Export `n` entries (ring positions bot..) as one chunk into the global
// ring (whole wave; false if the ring is half full). The chunk's unit of
// `active` is taken before it becomes visible.
// Only items the Kind calls movable leave the rank (UTS: nodes below the
// shard split depth; the replicated top levels stay where they are counted).
template <class Kind, int CAP>
__device__ bool global_enqueue(const typename Kind::Ctx &ctx, const GlobalView &gv, uint32_t words_per_chunk,
                               WaveStack<Kind, CAP> &st, uint32_t bot, uint32_t n, uint32_t *err) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    GlobalHdr *h = gv.hdr;
    // lane i packs item bot+i as {template, k, kend} (n <= 64)
    uint32_t w[W];
    bool mv = true;
    if ((uint32_t)lane < n) {
        const uint32_t p = bot + (uint32_t)lane;
        const uint2 dd = st.d[p & (CAP - 1)];
        load_tmpl<Kind, CAP>(st, (p - (dd.y >> 24)) & (CAP - 1), w);
        w[W - 2] = dd.x;
        w[W - 1] = dd.y & (kMaxChildren - 1);
        mv = Kind::movable(ctx, w);
    }
    if (__ballot(!mv) != 0) return false;
    uint32_t pos = 0;
    int ok = 0;
    if (lane == 0) {
        const uint32_t hd = ld_sys(&h->head), tl = ld_sys(&h->tail);
        if ((int)(tl - hd) < (int)(gv.cap / 2)) {
            add_sys(&h->active, 1u);
            pos = add_sys(&h->tail, 1u);
            ok = 1;
        }
    }
    if (!lane0((uint32_t)ok)) return false;
    kind_export<Kind>(ctx, w, (uint32_t)lane < n, err);
    pos = lane0(pos);
    const uint32_t slot = pos & (gv.cap - 1);
    uint32_t *ctl = gv.ctl + 2u * slot;
    uint32_t timed_out = 0;
    if (lane == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_sys(ctl) != pos) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                // the slot's previous lap was never consumed: write nothing
                // (its chunk is still unread) and stop every rank through the
                // shared error word (the ticket taken here is never published)
                dev_error(err, kErrQueueFull);
                dev_error_sys(&h->err, kErrQueueFull);
                timed_out = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (lane0(timed_out)) return false;
    uint32_t *dst = gv.data + (size_t)slot * words_per_chunk;
    if ((uint32_t)lane < n) {
#pragma unroll
        for (int i = 0; i < W; ++i) st_sys(&dst[(uint32_t)lane * W + i], w[i]);
    }
    if (lane == 0) st_sys(ctl + 1, n);
    vm_drain();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: visible to the other GPUs
    if (lane == 0) {
        st_sys(ctl, pos + 1);
        if (gv.rank < (uint32_t)kGlobalMaxRanks) add_sys(&h->moved[2 * gv.rank], 1ull);
    }
    vm_drain();
    return true;
}

// Take one chunk from the global ring into the (empty) stack; returns the
// entries taken (0: none). The caller converts the chunk's unit of `active`
// into its rank's (see GlobalHdr).
template <class Kind, int CAP>
__device__ uint32_t global_dequeue(const GlobalView &gv, uint32_t words_per_chunk, WaveStack<Kind, CAP> &st,
                                   uint32_t *err) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    GlobalHdr *h = gv.hdr;
    uint32_t pos = 0;
    int ok = 0;
    if (lane == 0) {
        const uint32_t hd = ld_sys(&h->head), tl = ld_sys(&h->tail);
        if ((int)(tl - hd) > 0 && cas_sys(&h->head, hd, hd + 1)) {
            pos = hd;
            ok = 1;
        }
    }
    if (!lane0((uint32_t)ok)) return 0;
    pos = lane0(pos);
    const uint32_t slot = pos & (gv.cap - 1);
    uint32_t *ctl = gv.ctl + 2u * slot;
    uint32_t cnt = 0;
    if (lane == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (true) {
            const unsigned long long sc = ld_sys((const unsigned long long *)ctl);
            if ((uint32_t)sc == pos + 1) {
                cnt = (uint32_t)(sc >> 32);
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                dev_error(err, kErrSpinTimeout);
                dev_error_sys(&h->err, kErrSpinTimeout);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint32_t n = lane0(cnt);
    const uint32_t *src = gv.data + (size_t)slot * words_per_chunk;
    if ((uint32_t)lane < n) {
        uint32_t w[W];
#pragma unroll
        for (int i = 0; i < W; ++i) w[i] = ld_sys(&src[(uint32_t)lane * W + i]);
        store_tmpl<Kind, CAP>(st, (uint32_t)lane, w);
        st.d[lane] = make_uint2(w[W - 2], w[W - 1]);
    }
    vm_drain();
    if (lane == 0) {
        st_sys(ctl, pos + gv.cap);
        if (gv.rank < (uint32_t)kGlobalMaxRanks) add_sys(&h->moved[2 * gv.rank + 1], 1ull);
    }
    vm_drain();
    return n;
}

__device__ __forceinline__ uint32_t xorshift(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

// ceil(2^16 / mu) for 1 <= mu <= 8 as a scalar select chain (a division
// would cost a float reciprocal round trip through a VGPR on the batch's
// critical path); (o * rcp16(mu)) >> 16 == o / mu for o < 1024
__device__ __forceinline__ uint32_t rcp16(uint32_t mu) {
    return mu <= 4 ? (mu <= 2 ? (mu == 1 ? 65536u : 32768u) : (mu == 3 ? 21846u : 16384u))
                   : (mu <= 6 ? (mu == 5 ? 13108u : 10923u) : (mu == 7 ? 9363u : 8192u));
}

// Register carry: output o of a uniform batch (every spawning lane spawned
// mu children) is child o % mu of the spawning lane of rank o / mu. One
// ds_permute tells rank r its source lane, two ds_bpermute hops bring the
// template to lane o.
template <int TW>
__device__ __forceinline__ void carry_permute(unsigned long long spawn, uint32_t mu, uint32_t nch,
                                              const uint32_t *child, uint32_t *ctmpl, uint32_t &ck,
                                              uint32_t rcp = 0) {
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t nsp = (uint32_t)__builtin_popcountll(spawn);
    const uint32_t rk = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(spawn >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)spawn, 0u));
    const uint32_t dst = nch != 0 ? rk : nsp + (lane - rk);
    const int src_of_rank = __builtin_amdgcn_ds_permute((int)(dst * 4u), (int)lane);
    // lane / mu (lane < 64, mu <= 8); 24-bit multiplies issue at full rate
    const uint32_t r = __umul24(lane, rcp ? rcp : rcp16(mu)) >> 16;
    const int src = __builtin_amdgcn_ds_bpermute((int)(r * 4u), src_of_rank);
#pragma unroll
    for (int i = 0; i < TW; ++i) ctmpl[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(src * 4, (int)child[i]);
    ck = lane - __umul24(r, mu);
}

// Register carry through LDS (WaveStack::kCarryLds; otherwise
// carry_permute): every spawning lane stores its new task's template in slot
// rank (its rank among the spawning lanes), output o reads slot o / mu and
// is child o % mu of it. One LDS round trip where carry_permute takes three
// dependent ones (ds_permute -> ds_bpermute -> 6 x ds_bpermute): the wave's
// LDS operations complete in issue order, so the reads see the stores.
// The store side, and the read of slot r (this lane's source rank).
// (`mine`: this lane's bit of `spawn`, when the caller has it as a lane mask
// already — testing the bit again is three VALU instructions per carry)
template <int TW>
__device__ __forceinline__ void carry_lds_slot(uint4 *scr, unsigned long long spawn, bool mine, const uint32_t *child,
                                               uint32_t *ctmpl, uint32_t r) {
    const uint32_t rk = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(spawn >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)spawn, 0u));
    if (mine) {
        if constexpr (TW == 6) {
            scr[2 * rk] = make_uint4(child[0], child[1], child[2], child[3]);
            *(uint2 *)&scr[2 * rk + 1] = make_uint2(child[4], child[5]);
        } else {
            *(uint2 *)&scr[2 * rk] = make_uint2(child[0], child[1]);
        }
    }
    if constexpr (TW == 6) {
        const uint4 a = scr[2 * r];
        const uint2 b = *(const uint2 *)&scr[2 * r + 1];
        ctmpl[0] = a.x;
        ctmpl[1] = a.y;
        ctmpl[2] = a.z;
        ctmpl[3] = a.w;
        ctmpl[4] = b.x;
        ctmpl[5] = b.y;
    } else {
        const uint2 a = *(const uint2 *)&scr[2 * r];
        ctmpl[0] = a.x;
        ctmpl[1] = a.y;
    }
}

template <int TW>
__device__ __forceinline__ void carry_lds(uint4 *scr, unsigned long long spawn, uint32_t mu, const uint32_t *child,
                                          uint32_t *ctmpl, uint32_t &ck, uint32_t rcp = 0) {
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t r = __umul24(lane, rcp ? rcp : rcp16(mu)) >> 16;  // lane / mu
    carry_lds_slot<TW>(scr, spawn, ((spawn >> lane) & 1ull) != 0, child, ctmpl, r);
    ck = lane - __umul24(r, mu);
}

// Uniform push: no lane has a residual range and every lane that spawned a
// task spawned exactly `mu` (<= kPieces) children — every BIN-tree batch
// after the root fan-out, every fib batch. Group starts are then
// mu * (rank among spawning lanes): a ballot + mbcnt, no scan, no marks.
// Output o is child o % mu of its group, whose template sits o % mu slots
// back (the descriptor's delta). o / mu uses a 16-bit reciprocal, exact for
// o < 1024 and mu <= 8.
template <class Kind, int CAP>
__device__ __forceinline__ void push_uniform(WaveStack<Kind, CAP> &st, uint32_t base, uint32_t excl,
                                             uint32_t tout, uint32_t mu, bool spawned,
                                             const uint32_t *child) {
    constexpr uint32_t M = CAP - 1;
    if (spawned) store_tmpl<Kind, CAP>(st, (base + excl) & M, child);
    const uint32_t rcp = rcp16(mu);  // wave-uniform (scalar)
    for (uint32_t r0 = 0; r0 < tout; r0 += kWaveSize) {
        const uint32_t o = r0 + (uint32_t)lane_id();
        if (o < tout) {
            const uint32_t kk = o - ((o * rcp) >> 16) * mu;
            st.d[(base + o) & M] = make_uint2(kk, (kk + 1) | (kk << 24));
        }
    }
}

// Push one batch's outputs at ring positions [base, base + tout). Lane L's
// items are contiguous at base + excl: the residual of its item (children
// k+1..kend-1 of `tmpl`, <= 2 pieces) then the new task's children (`child`,
// ucnt children, nch = min(ucnt, kPieces) pieces). Fast path (no residuals,
// no split): every group is children 0..nch-1 unsplit, so an item's k equals
// its distance to the group start; the group starts are marked in LDS with a
// per-round tag and a DPP max-scan gives every output lane its group start.
template <class Kind, int CAP>
__device__ __forceinline__ void push_outputs(WaveStack<Kind, CAP> &st, uint32_t base, uint32_t excl,
                                             uint32_t tout, uint32_t nres, uint32_t ucnt,
                                             uint32_t nch, const uint32_t *tmpl,
                                             const uint32_t *child, uint32_t k, uint32_t kend,
                                             uint32_t tag) {
    constexpr uint32_t M = CAP - 1;
    constexpr int kPieces = pieces_of<Kind>();
    const int lane = lane_id();
    if (__ballot(nres != 0 || ucnt > (uint32_t)kPieces) == 0) {
        if (nch) store_tmpl<Kind, CAP>(st, (base + excl) & M, child);
        uint32_t carry = 0;
        for (uint32_t r0 = 0; r0 < tout; r0 += kWaveSize, ++tag) {
            if (nch && excl >= r0 && excl < r0 + kWaveSize) st.mark[excl - r0] = tag;
            const int s = wave_scan_max(st.mark[lane] == tag ? lane : -1);
            const uint32_t start = s >= 0 ? r0 + (uint32_t)s : carry;
            carry = (uint32_t)lane63((int)start);
            const uint32_t o = r0 + (uint32_t)lane;
            if (o < tout) {
                const uint32_t kk = o - start;
                st.d[(base + o) & M] = make_uint2(kk, (kk + 1) | (kk << 24));
            }
        }
        return;
    }
    // general path: residual ranges and wide (split) child ranges
    uint32_t pos = base + excl;
    if (nres) {
        store_tmpl<Kind, CAP>(st, pos & M, tmpl);  // the residual's own copy of its template
        const uint32_t mid = k + 1 + ((kend - k - 1) >> 1);
        st.d[pos & M] = make_uint2(k + 1, nres == 1 ? kend : mid);
        if (nres == 2) st.d[(pos + 1) & M] = make_uint2(mid, kend | (1u << 24));
        pos += nres;
    }
    if (nch) store_tmpl<Kind, CAP>(st, pos & M, child);
    for (uint32_t j = 0; __ballot(j < nch); ++j) {
        if (j < nch) {
            uint32_t lo = j, hi = j + 1;
            if (ucnt > (uint32_t)kPieces) {
                lo = (j * ucnt) / (uint32_t)kPieces;
                hi = ((j + 1) * ucnt) / (uint32_t)kPieces;
            }
            st.d[(pos + j) & M] = make_uint2(lo, hi | (j << 24));
        }
    }
}

// One lane's outputs of one item at ring positions pos..: the residual of
// the item (children k+1..kend-1 of `tmpl`, nres <= 2 pieces), then the new
// task's children (`child`, ucnt children as nch pieces) — the general path
// of push_outputs for a lane that pushes two items' outputs (dual batches).
template <class Kind, int CAP>
__device__ __forceinline__ void push_group(WaveStack<Kind, CAP> &st, uint32_t pos, uint32_t nres, uint32_t ucnt,
                                           uint32_t nch, const uint32_t *tmpl, const uint32_t *child, uint32_t k,
                                           uint32_t kend) {
    constexpr uint32_t M = CAP - 1;
    constexpr int kPieces = pieces_of<Kind>();
    if (nres) {
        store_tmpl<Kind, CAP>(st, pos & M, tmpl);
        const uint32_t mid = k + 1 + ((kend - k - 1) >> 1);
        st.d[pos & M] = make_uint2(k + 1, nres == 1 ? kend : mid);
        if (nres == 2) st.d[(pos + 1) & M] = make_uint2(mid, kend | (1u << 24));
        pos += nres;
    }
    if (nch) store_tmpl<Kind, CAP>(st, pos & M, child);
#pragma unroll
    for (uint32_t j = 0; j < (uint32_t)kPieces; ++j) {
        if (j < nch) {
            uint32_t lo = j, hi = j + 1;
            if (ucnt > (uint32_t)kPieces) {
                lo = (j * ucnt) / (uint32_t)kPieces;
                hi = ((j + 1) * ucnt) / (uint32_t)kPieces;
            }
            st.d[(pos + j) & M] = make_uint2(lo, hi | (j << 24));
        }
    }
}

// Narrow frontier (span-bound trees): the ring is empty and no hunger can
// stop a carry of at most one batch (spill_lo above it), so the chain runs in
// a loop of its own: process the carried items, carry their children,
// nothing else — no ring, no hunger reads, no spill checks. It returns when a
// batch has no children (the wave goes idle) or outputs that do not carry
// (non-uniform, or more than one batch): those go onto the empty ring and
// the main loop takes over. A separate (not inlined) function so the
// compiler keeps its own copy of the task body instead of sharing the main
// loop's, whose scheduler state would otherwise ride along every iteration.
template <int TW>
struct NarrowState {
    uint32_t ctmpl[TW];
    uint32_t ck, carry, top, tag, n_exec, n_spawn, batches;
};

#ifndef HX_PHASES
#define HX_PHASES 0  // diagnostic: main-loop batch phase stamps (run_worker)
#endif
// Optional diagnostic: a Kind's Acc with a `mode` field learns whether its
// tasks run in the narrow loop (1) or the main loop (0).
template <class A, class = void>
struct acc_has_mode : std::false_type {};
template <class A>
struct acc_has_mode<A, decltype((void)A::mode)> : std::true_type {};
template <class A>
__device__ __forceinline__ void acc_set_mode(A &a, uint32_t m) {
    if constexpr (acc_has_mode<A>::value) a.mode = m;
}
// ... and a `wid` field the running worker's id (diagnostic traces)
template <class A, class = void>
struct acc_has_totals : std::false_type {};
template <class A>
struct acc_has_totals<A, decltype((void)&A::totals)> : std::true_type {};

template <class A, class = void>
struct acc_has_wid : std::false_type {};
template <class A>
struct acc_has_wid<A, decltype((void)A::wid)> : std::true_type {};
template <class A>
__device__ __forceinline__ void acc_set_wid(A &a, uint32_t w) {
    if constexpr (acc_has_wid<A>::value) a.wid = w;
}

// The narrow loop of a fixed-size family (KindFixedChildren, pure, bounded,
// LDS carry; BIN trees): every spawning lane has exactly mu children, so a
// level is process -> ballot -> carry, with the wave's task and child counts
// kept as two scalar sums (the carry and t2) instead of per-lane adds, and no
// uniformity branches. The general loop below compiled this case to ~70
// instructions around the SHA-1 with five taken branches per level.
template <class Kind, int CAP>
__device__ __forceinline__ NarrowState<Kind::kTmplWords> narrow_loop_fixed(
    const typename Kind::Ctx &ctx_ref, typename Kind::Acc &acc_ref, uint32_t *err, WaveStack<Kind, CAP> &st,
    NarrowState<Kind::kTmplWords> ns, uint32_t mu, uint32_t r_fix, uint32_t ck_fix) {
    constexpr int TW = Kind::kTmplWords;
    const typename Kind::Ctx ctx = ctx_ref;
    typename Kind::Acc acc = acc_ref;
    acc_set_mode(acc, 1u);
    const uint32_t lane = (uint32_t)lane_id();
    constexpr bool kBulk = KindBulkCount<Kind>::value;
    // per level: the tasks run (the carry) and the spawning lanes, as scalar
    // sums; spawned = m x spawners, leaves = tasks - spawners
    uint32_t carry = lane0(ns.carry), batches = 0, s_exec = 0, s_nsp = 0, t2;
    // the task index: at entry the main loop's carry_lds left ck = lane % mu
    // for the same mu (a fixed family's uniform batch), which is ck_fix, so
    // every level passes ck_fix (no per-level copy of a loop-carried ck)
    const uint32_t k = ck_fix;
    uint32_t ch2[TW];
    bool sp;
    unsigned long long sp2;
    // one exit test per level (t2 = 0: nothing spawned; t2 > one batch: onto
    // the ring below): a chain level spawns and carries and falls through
    // to the back-edge
    do {
        const bool h = lane < carry;
        if constexpr (kBulk) sp = Kind::process_bulk(ctx, acc, ns.ctmpl, k, ch2, err, h);
        else sp = Kind::process(ctx, acc, ns.ctmpl, k, ch2, err, h) > 0;
        ++batches;
        s_exec += carry;
        // (the builtin on the lane mask itself: __ballot takes an int and
        // re-tests it, a select and a compare per level)
        sp2 = __builtin_amdgcn_ballot_w64(sp);
        const uint32_t nsp = (uint32_t)__builtin_popcountll(sp2);
        s_nsp += nsp;
        t2 = mu * nsp;
        // the carry runs on every level, also one that does not carry (its
        // templates are then unused; with no spawner nothing is written):
        // the LDS reads land straight in the loop's template registers
        carry_lds_slot<TW>(st.cscr, sp2, sp, ch2, ns.ctmpl, r_fix);
        carry = t2;
    } while (t2 - 1u < (uint32_t)kWaveSize);
    ns.ck = ck_fix;
    if (t2 != 0) {
        // more than one batch: onto the empty ring
        const uint32_t rk2 = (uint32_t)__builtin_amdgcn_mbcnt_hi(
            (uint32_t)(sp2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sp2, 0u));
        push_uniform<Kind, CAP>(st, ns.top, mu * rk2, t2, mu, sp, ch2);
        ns.top += t2;
        carry = 0;
    }
    if constexpr (kBulk) Kind::count_bulk(acc, s_exec, s_exec - s_nsp);
    if (lane == 0) {
        ns.n_exec += s_exec;
        ns.n_spawn += mu * s_nsp;
    }
    ns.carry = carry;
    ns.batches = batches;
    acc_set_mode(acc, 0u);
    acc_ref = acc;
    return ns;
}

template <class Kind, int CAP>
__device__ __forceinline__ NarrowState<Kind::kTmplWords> narrow_loop(
    const typename Kind::Ctx &ctx_ref, typename Kind::Acc &acc_ref, uint32_t *err, WaveStack<Kind, CAP> &st,
    NarrowState<Kind::kTmplWords> ns) {
    constexpr int TW = Kind::kTmplWords;
    constexpr int kPieces = pieces_of<Kind>();
    // private copies: through the references every iteration would reload
    // the parameters and store the counters (flat memory, waited on mid-task)
    const typename Kind::Ctx ctx = ctx_ref;
    typename Kind::Acc acc = acc_ref;
    acc_set_mode(acc, 1u);
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t carry = lane0(ns.carry), batches = 0;
    // fixed-size families (KindFixedChildren): the group size and its
    // reciprocal are loop invariants
    uint32_t mu_fix = 0, rcp_fix = 0;
    if constexpr (KindFixedChildren<Kind>::value) {
        mu_fix = lane0(Kind::fixed_children(ctx));
        if (mu_fix > (uint32_t)kPieces) mu_fix = 0;
        rcp_fix = mu_fix ? rcp16(mu_fix) : 0u;
    }
    // ... and so are each lane's carry source slot and child index
    const bool hoist = mu_fix != 0;  // (wave-uniform)
    const uint32_t r_fix = hoist ? __umul24(lane, rcp_fix) >> 16 : 0u;
    const uint32_t ck_fix = hoist ? lane - __umul24(r_fix, mu_fix) : 0u;
    if constexpr (KindFixedChildren<Kind>::value && Kind::kPure && Kind::kBoundedChildren &&
                  WaveStack<Kind, CAP>::kCarryLds) {
        if (hoist) return narrow_loop_fixed<Kind, CAP>(ctx_ref, acc_ref, err, st, ns, mu_fix, r_fix, ck_fix);
    }
    while (true) {
        const bool h = lane < carry;
        uint32_t ch2[TW];
        int c2 = 0;
        if constexpr (Kind::kPure) {
            c2 = Kind::process(ctx, acc, ns.ctmpl, ns.ck, ch2, err, h);
        } else {
            if (h) c2 = Kind::process(ctx, acc, ns.ctmpl, ns.ck, ch2, err, true);
        }
        ++batches;
        uint32_t u2 = c2 > 0 ? (uint32_t)c2 : 0u;
        if (!Kind::kBoundedChildren && u2 >= kMaxChildren) {
            dev_error(err, kErrBadTask);
            u2 = 0;
        }
        ns.n_exec += h ? 1u : 0u;
        ns.n_spawn += h ? u2 : 0u;
        const uint32_t n2 = u2 > (uint32_t)kPieces ? (uint32_t)kPieces : u2;
        const unsigned long long sp2 = __ballot(n2 != 0);
        if (!sp2) {
            carry = 0;
            break;
        }
        uint32_t mu2;
        bool uni2;
        if (KindFixedChildren<Kind>::value && mu_fix) {
            mu2 = mu_fix;
            uni2 = true;
        } else {
            mu2 = (uint32_t)__builtin_amdgcn_readlane((int)n2, __builtin_ctzll(sp2));
            uni2 = __ballot(u2 > (uint32_t)kPieces || (n2 != 0 && n2 != mu2)) == 0;
        }
        if (uni2) {
            const uint32_t t2 = mu2 * (uint32_t)__builtin_popcountll(sp2);
            if (t2 <= (uint32_t)kWaveSize) {
                // (a scalar walk over the spawn mask instead of the permute pair
                // measured slower: T3L 31.8 -> 32.6 ms, profiles/r04/walk_ab.log)
                if constexpr (WaveStack<Kind, CAP>::kCarryLds) {
                    if (hoist) {
                        carry_lds_slot<TW>(st.cscr, sp2, ((sp2 >> lane) & 1ull) != 0, ch2, ns.ctmpl, r_fix);
                        ns.ck = ck_fix;
                    } else {
                        carry_lds<TW>(st.cscr, sp2, mu2, ch2, ns.ctmpl, ns.ck, rcp_fix);
                    }
                }
                else carry_permute<TW>(sp2, mu2, n2, ch2, ns.ctmpl, ns.ck, rcp_fix);
                carry = t2;
                continue;
            }
            // more than one batch: onto the empty ring
            const uint32_t rk2 = (uint32_t)__builtin_amdgcn_mbcnt_hi(
                (uint32_t)(sp2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sp2, 0u));
            push_uniform<Kind, CAP>(st, ns.top, mu2 * rk2, t2, mu2, n2 != 0, ch2);
            ns.top += t2;
        } else {
            const int P2 = wave_scan_add((int)n2);
            const uint32_t t2 = (uint32_t)lane63(P2);
            push_outputs<Kind, CAP>(st, ns.top, (uint32_t)(P2 - (int)n2), t2, 0u, u2, n2, ns.ctmpl, ch2, ns.ck,
                                    ns.ck + 1, ns.tag);
            ns.tag += 16;
            ns.top += t2;
        }
        carry = 0;
        break;
    }
    ns.carry = carry;
    ns.batches = batches;
    acc_set_mode(acc, 0u);
    acc_ref = acc;
    return ns;
}

// Sibling hand-off in LDS (workgroups of WPG > 1 worker waves). Every wave
// of the workgroup has an inbox; a wave about to spill to the HBM deques
// first offers the chunk to an idle sibling: it claims the sibling's empty
// inbox (LDS CAS 0 -> 2), writes the items and sets it full (1) — LDS
// operations of one wave land in issue order, so the items are there before
// the flag. The idle sibling polls its own inbox before the deques. An inbox
// chunk holds one unit of `outstanding` like an HBM chunk: the putter (which
// holds its own unit, so the count cannot read 0 meanwhile) adds it before
// the chunk becomes visible, and the taker inherits it, so no wave can see
// 0 while a chunk waits in an inbox. A wave that leaves the megakernel closes
// its inbox (state 3) so nothing is put there afterwards.
template <class Kind>
struct Inbox {
    uint32_t state;  // 0 empty, 2 being filled, 1 full, 3 closed (owner left)
    uint32_t n;
    uint32_t idle;   // the owner wave holds no work
    uint32_t pad;
    uint32_t w[64 * Kind::kWords];
};

template <class Kind, int CAP>
__device__ bool inbox_put(const typename Kind::Ctx &ctx, Inbox<Kind> &ib, WaveStack<Kind, CAP> &st, uint32_t bot,
                          uint32_t n, SchedGlobals *g) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    // the items' reads go out beside the claim (they depend on nothing it
    // decides: one wait instead of three round trips in a row)
    const bool valid = (uint32_t)lane < n;
    const uint32_t p = bot + (valid ? (uint32_t)lane : 0u);
    const uint2 dd = st.d[p & (CAP - 1)];
    uint32_t ok = 0;
    if (lane == 0) ok = lds_cas(&ib.state, 0u, 2u) ? 1u : 0u;
    uint32_t w[W];
    load_tmpl<Kind, CAP>(st, (p - (dd.y >> 24)) & (CAP - 1), w);
    if (!lane0(ok)) return false;
    {
        w[W - 2] = dd.x;
        w[W - 1] = dd.y & (kMaxChildren - 1);
        kind_export<Kind>(ctx, w, valid, &g->err);
        kind_trace_item<Kind>(ctx, w, valid, 2u, true);
        if (valid) {
#pragma unroll
            for (int i = 0; i < W; ++i) ib.w[(uint32_t)lane * W + i] = w[i];
        }
    }
    asm volatile("" ::: "memory");
    if (lane == 0) {
        add_agent(&g->outstanding, 1u);  // the chunk's unit, before it becomes visible
        lds_store(&ib.n, n);
        lds_store(&ib.idle, 0u);
        lds_store(&ib.state, 1u);  // after the items (one wave's DS operations land in order)
    }
    return true;
}

// take a full inbox into the (empty) ring; returns the items (0: empty)
template <class Kind, int CAP>
__device__ uint32_t inbox_take(const typename Kind::Ctx &ctx, Inbox<Kind> &ib, WaveStack<Kind, CAP> &st) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    if (lane0(lds_load(&ib.state)) != 1u) return 0;
    const uint32_t n = lane0(lds_load(&ib.n));
    if ((uint32_t)lane < n) {
        uint32_t w[W];
#pragma unroll
        for (int i = 0; i < W; ++i) w[i] = ib.w[(uint32_t)lane * W + i];
        store_tmpl<Kind, CAP>(st, (uint32_t)lane, w);
        st.d[lane] = make_uint2(w[W - 2], w[W - 1]);
        kind_trace_item<Kind>(ctx, w, true, 3u, true);
    }
    if (lane == 0) lds_store(&ib.state, 0u);
    return n;
}

// a wave stops holding work: local `outstanding` -1; the wave that takes it
// to 0 releases its rank's unit of the global `active` (GLOBAL launches)
template <bool GLOBAL>
__device__ __forceinline__ void wave_goes_idle(SchedGlobals *g, const GlobalView &gv, const PoolView &pool) {
    if (lane_id() != 0) return;
    if constexpr (GLOBAL) {
        const uint32_t prev = __hip_atomic_fetch_add(&g->outstanding, (uint32_t)-1, __ATOMIC_RELEASE, HX_AGENT);
        if (prev == 1u) {
            // release the rank's unit: idle += 1, then the handshake word (a
            // release store: the idle add has been performed before it)
            add_sys(&gv.hdr->idle, 1u);
            __hip_atomic_store(&gv.hdr->held[gv.rank], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            add_sys(&gv.hdr->active, (uint32_t)-1);
        }
    } else {
        const uint32_t prev = __hip_atomic_fetch_add(&g->outstanding, (uint32_t)-1, __ATOMIC_RELEASE, HX_AGENT);
        if (prev == 1u) {
            // no wave holds work and no chunk is queued: that is final (only
            // holders create work), so tell every deque's pollers
            for (uint32_t q = 0; q < pool.nq; ++q) st_agent(&pool.hdr[q].done, 1u);
        }
    }
}

// Breadth-first seeding (SchedGlobals::seed): a tree grown from one root on
// thousands of waves spends most of a small search handing work out — every
// generation of hand-offs (batches to fill a ring, a spill, a probe that
// finds it) only doubles the waves that hold work (worker timelines,
// profiles/r04). Instead the whole grid first expands the top of the tree
// level by level: level d is a list of child slots {template, k, k + 1} in
// HBM; the waves split it into 64-slot blocks, run each slot (Kind::process:
// counting, sharding and all), and append the children of every node as the
// slots of level d + 1 (one bump per wave). A level ends when every wave
// that had a block has counted itself done (ctl line 2d + 1) — only the
// participants touch the counters; everyone polls one line for a few
// microseconds. The narrow top levels (at most kSoloCap slots) wave 0 runs
// alone in its LDS ring, before any other wave is needed. Once a level holds
// at least `target` slots (or after `max_levels`) every wave takes an equal
// share of it straight into its ring and the work-stealing loop starts with
// every wave busy. ctl lines: [2d + 1] one 64-bit word per grid-wide level d
// {slots appended to level d + 1 (low half), participants done (high)},
// then kSeedGoLines broadcast lines: word d < L the size + 1 of level d + 1,
// words L / L + 1 the solo levels' result (size + 1, depth; wave 0). The host sets `outstanding` to the wave
// count: every wave holds a unit until its share is taken.
// Pure kinds only (the slots of a block run branch-free, as in a batch).
// Ordering of the seeding's level hand-offs. Every word another wave reads
// travels as an sc1 (device-coherent, write-through) store or load: the
// slots (st_sc1_x4 / ld_sc1_x4x2), the counters and go lines (agent-scope
// atomics). A producer drains its stores (s_waitcnt vmcnt(0)) before the
// atomic or store that publishes them; the done add is acq_rel and the solo
// result a release store. Full agent release / acquire fences around each
// hand-off (L2 write-back and invalidate on every wave, every level:
// HX_SEED_FENCES=1) cost T1 0.240-0.250 -> 0.256-0.267 ms and T1L 2.43 ->
// 2.53 ms same-box (profiles/r05/ab_seedfence.log), so they are a build
// option, not the default.
#ifndef HX_SEED_FENCES
#define HX_SEED_FENCES 0
#endif
template <class Kind, int CAP>
__device__ uint32_t seed_levels(const typename Kind::Ctx &ctx, typename Kind::Acc &acc, SchedGlobals *g,
                                WaveStack<Kind, CAP> &st, uint32_t gid, uint32_t nw, uint32_t spin_limit_ms,
                                uint32_t &n_exec, uint32_t &n_spawn, uint32_t &nbatch, Timeline &tl) {
    static_assert(Kind::kPure, "breadth-first seeding runs slots branch-free");
    constexpr int TW = Kind::kTmplWords, W = Kind::kWords;
    static_assert(TW == 6 && W == 8, "seeding moves 32-byte slots {6-word template, k, k + 1}");
    const int lane = lane_id();
    const auto &sd = g->seed;
    uint32_t *ctl = sd.ctl;
    auto line = [&](int i) { return ctl + 64 * i; };
    // go[d]: level d + 1 is complete (written by the level's last participant
    // into every broadcast line; a wave polls its own)
    uint32_t *go = line(2 * kSeedMaxLevels + 2 + (int)(gid % kSeedGoLines));
    uint32_t *err = &g->err;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    auto wait_ge = [&](uint32_t *p, uint32_t want) -> bool {
        uint32_t v = 0;
        for (uint32_t n = 0;; ++n) {
            if (lane == 0) v = ld_agent(p);
            if (lane0(v) >= want) return true;
            if ((n & 63) == 63) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * spin_limit_ms) {
                    if (lane == 0) dev_error(err, kErrSpinTimeout);
                    return false;
                }
                uint32_t e = 0;
                if (lane == 0) e = ld_agent(err);
                if (lane0(e)) return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // the lane -> node map of a block lives in ring entries [kScr, kScr + 64)
    // (the ring is still empty; wave 0's solo levels use [0, 2 kSoloCap))
    constexpr uint32_t kSoloCap = (uint32_t)(CAP - 64) / 2;
    constexpr uint32_t kScr = 2 * kSoloCap;
    static_assert(kSoloCap >= 64, "the solo levels need ring room");
    // one block of 64 slots (template `tmpl`, child k, valid) -> the children
    // of every node as slots of the next level, written flat to dst from
    // slot `base` (output o by lane o % 64, so every store instruction writes
    // consecutive slots) and, for outputs below kSoloCap, to the LDS level
    // buffer at ring entry `lds_out` (~0u: none). Slots are 32 B {template,
    // k, k + 1}, stored as 16-B sc1 accesses; base / count come from `alloc`
    uint32_t mtag = 1u << 20;  // run_slots' window marks (above any main-loop tag; cleared below)
    auto run_slots = [&](const uint32_t (&tmpl)[TW], uint32_t k, bool valid, uint32_t *dst, uint32_t lds_out,
                         auto &&alloc) -> bool {
        uint32_t child[TW];
        const int nc = kind_seed_process<Kind>(ctx, acc, tmpl, k, child, err, valid);
        ++nbatch;
        const uint32_t u = valid && nc > 0 ? (uint32_t)nc : 0u;
        n_exec += valid ? 1u : 0u;
        n_spawn += u;
        const int S = wave_scan_add((int)u);
        const uint32_t tot = (uint32_t)lane63(S), excl = (uint32_t)S - u;
        const uint32_t base = alloc(tot);
        st.t0[kScr + lane] = make_uint4(child[0], child[1], child[2], child[3]);
        st.t1[kScr + lane] = make_uint2(child[4], child[5]);
        st.d[kScr + lane] = make_uint2(excl, u);
        asm volatile("" ::: "memory");
        if (base + tot > sd.cap) {  // the level buffer is sized by the host; never expected
            if (lane == 0) dev_error(err, kErrStackOverflow);
            return false;
        }
        // the node of output o: the last lane whose first output is <= o —
        // each spawning lane marks its first output's place in the 64-output
        // window, a max-scan spreads the marks (one LDS round trip a window,
        // where a binary search over the lanes took six)
        int owner = 0;
        for (uint32_t r0 = 0; r0 < tot; r0 += 64) {
            ++mtag;
            if (u && excl >= r0 && excl < r0 + 64u) st.mark[excl - r0] = (mtag << 6) | (uint32_t)lane;
            const uint32_t mk = st.mark[lane];
            const int sc = wave_scan_max((mk >> 6) == mtag ? (int)(mk & 63u) : -1);
            const int prev = owner;
            owner = (int)lane63(sc >= 0 ? sc : prev);
            const uint32_t o = r0 + (uint32_t)lane;
            if (o < tot) {
                const int lo = sc >= 0 ? sc : prev;
                const uint32_t j = o - st.d[kScr + lo].x;
                const uint4 t0 = st.t0[kScr + lo];
                const uint2 t1 = st.t1[kScr + lo];
                uint32_t *q = dst + (size_t)(base + o) * W;
                st_sc1_x4(q, t0);
                st_sc1_x4(q + 4, make_uint4(t1.x, t1.y, j, j + 1));
                if (lds_out != ~0u && base + o < kSoloCap) {
                    st.t0[lds_out + base + o] = t0;
                    st.t1[lds_out + base + o] = t1;
                    st.d[lds_out + base + o] = make_uint2(j, j + 1);
                }
            }
        }
        asm volatile("" ::: "memory");
        return true;
    };
    auto buf = [&](int d) { return sd.buf + (size_t)(d & 1) * sd.cap * W; };
    auto stop = [&](uint32_t E, int d) {
        return E == 0 || d >= (int)sd.max_levels || d + 1 >= kSeedMaxLevels ||
               (E >= sd.target && d >= (int)sd.min_levels);
    };
    // wave 0: the root's slots (level 0), and the narrow top levels on its
    // own, entirely in its ring (LDS) and registers: no round trip per
    // block or level, the slots of every level also stored to HBM (stores
    // only) for the grid-wide levels to read, drained once at the end
    uint32_t E = 0;
    int d = 0;
    if (gid == 0) {
        uint32_t tmpl[TW];
        const int rn = Kind::roots(ctx, acc, tmpl);
        E = rn > 0 ? ((uint32_t)rn < sd.cap ? (uint32_t)rn : sd.cap) : 0u;
        for (uint32_t e = (uint32_t)lane; e < E; e += 64) {
            uint32_t *q = buf(0) + (size_t)e * W;
            st_sc1_x4(q, make_uint4(tmpl[0], tmpl[1], tmpl[2], tmpl[3]));
            st_sc1_x4(q + 4, make_uint4(tmpl[4], tmpl[5], e, e + 1));
            if (e < kSoloCap) {
                st.t0[e] = make_uint4(tmpl[0], tmpl[1], tmpl[2], tmpl[3]);
                st.t1[e] = make_uint2(tmpl[4], tmpl[5]);
                st.d[e] = make_uint2(e, e + 1);
            }
        }
        asm volatile("" ::: "memory");
        uint32_t in = 0, out = kSoloCap;
        bool ok = true;
        const uint32_t solo = sd.solo_cap && sd.solo_cap < kSoloCap ? sd.solo_cap : kSoloCap;
        while (ok && !stop(E, d) && E <= solo) {
            uint32_t cnt = 0;
            auto alloc = [&](uint32_t tot) {
                const uint32_t b0 = cnt;
                cnt += tot;
                return b0;
            };
            for (uint32_t b = 0; b * 64 < E && ok; ++b) {
                const uint32_t e = b * 64 + (uint32_t)lane;
                const bool valid = e < E;
                const uint32_t src = in + (valid ? e : 0u);
                const uint4 a = st.t0[src];
                const uint2 c = st.t1[src];
                const uint32_t t[TW] = {a.x, a.y, a.z, a.w, c.x, c.y};
                ok = run_slots(t, st.d[src].x, valid, buf(d + 1), out, alloc);
            }
            E = cnt;
            ++d;
            const uint32_t x = in;
            in = out;
            out = x;
            tl.log(kTlSeed, (uint32_t)d);
        }
        // every level's slots land before the result is published, on every
        // broadcast line (1,023 waves polling one line made it a hot spot:
        // the first grid-wide level took 20 us, timeline tl_t1_a). The slot
        // stores are inline-asm sc1 stores the waitcnt pass cannot see, so
        // they are drained here, before the publish, unconditionally
        vm_drain();
        if (HX_SEED_FENCES) release_agent();
        for (uint32_t i = (uint32_t)lane; i < (uint32_t)kSeedGoLines; i += 64) {
            // one 8-byte store {size + 1, depth}: a reader that sees the size sees the depth
            unsigned long long *gl = (unsigned long long *)(line(2 * kSeedMaxLevels + 2 + (int)i) + kSeedMaxLevels);
            st_agent(gl, (unsigned long long)(E + 1) | ((unsigned long long)(uint32_t)d << 32));
        }
        vm_drain();
        if (!ok) return 0;
    }
    if (!wait_ge(go + kSeedMaxLevels, 1u)) return 0;
    if (HX_SEED_FENCES) acquire_agent();
    if (lane == 0) {
        const unsigned long long r = ld_agent((const unsigned long long *)(go + kSeedMaxLevels));
        E = (uint32_t)r - 1u;
        d = (int)(r >> 32);
    }
    E = lane0(E);
    d = (int)lane0((uint32_t)d);
    // the wide levels: the grid's waves, 64 slots a block. Per level one
    // 64-bit word (ctl line 2d + 1): low half the slots appended to level
    // d + 1, high half the participants done; the participant whose done
    // add completes the count reads the level's size from its own atomic
    for (; !stop(E, d); ++d) {
        const uint32_t nblk = (E + 63) / 64;
        unsigned long long *word = (unsigned long long *)line(2 * d + 1);
        auto alloc = [&](uint32_t tot) {
            unsigned long long b0 = 0;
            if (lane == 0 && tot) b0 = add_agent(word, (unsigned long long)tot);
            return (uint32_t)lane0((uint32_t)b0);
        };
        bool ok = true;
        for (uint32_t b = gid; b < nblk && ok; b += nw) {
            const uint32_t e = b * 64 + (uint32_t)lane;
            const bool valid = e < E;
            uint4 s0, s1;
            ld_sc1_x4x2(buf(d) + (size_t)(valid ? e : 0u) * W, s0, s1);
            const uint32_t t[TW] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y};
            ok = run_slots(t, s1.z, valid, buf(d + 1), ~0u, alloc);
        }
        if (!ok) return 0;
        // participants count themselves done once their slots are drained; the
        // last one publishes the next level's size (+ 1) on every broadcast line
        const uint32_t P = nblk < nw ? nblk : nw;
        if (gid < P) {
            vm_drain();
            unsigned long long prev = 0;
            if (lane == 0) prev = __hip_atomic_fetch_add(word, 1ull << 32, __ATOMIC_ACQ_REL, HX_AGENT);
            const uint32_t done = lane0((uint32_t)(prev >> 32)) + 1u;
            const uint32_t e1 = lane0((uint32_t)prev) + 1u;  // (biased: 0 = not yet)
            if (done == P) {
                // go line i holds, per level, the next level's size + 1 at word d
                if (HX_SEED_FENCES) release_agent();
                for (uint32_t i = (uint32_t)lane; i < (uint32_t)kSeedGoLines; i += 64)
                    st_agent(line(2 * kSeedMaxLevels + 2 + (int)i) + d, e1);
            }
        }
        if (!wait_ge(go + d, 1u)) return 0;
        if (HX_SEED_FENCES) acquire_agent();
        uint32_t e2 = 0;
        if (lane == 0) e2 = ld_agent(go + d);
        E = lane0(e2) - 1u;
        tl.log(kTlSeed, (uint32_t)d + 1u);
    }
    // this wave's share of level d's slots, as ring items
    if (E > sd.cap) E = sd.cap;
    const uint32_t lo = (uint32_t)(((unsigned long long)E * gid) / nw),
                   hi = (uint32_t)(((unsigned long long)E * (gid + 1)) / nw);
    const uint32_t n = hi - lo;
    constexpr uint32_t kMax = CAP / 2;
    if (n > kMax) {  // (never with the host's target: a share far below a ring)
        if (lane == 0) dev_error(err, kErrStackOverflow);
        return 0;
    }
    const uint32_t *src = buf(d);
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane;
        uint4 a, c;
        ld_sc1_x4x2(src + (size_t)(lo + (i < n ? i : 0u)) * W, a, c);
        if (i < n) {
            const uint32_t w[W] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
            store_tmpl<Kind, CAP>(st, i, w);
            st.d[i] = make_uint2(w[W - 2], w[W - 1]);
        }
    }
    return n;
}

// GLOBAL: the launch shares work with the other ranks through g->gview
// (idle waves take chunks from the global ring, a wave holding spill_lo+
// items exports a chunk while some rank is idle and none of its own waves
// is hungry; termination waits for the global `active` count)
// WPG > 1: the workgroup's WPG worker waves hand work to each other through
// LDS inboxes (`ib`: WPG of them, this wave's is ib[wave]; see Inbox)
template <class Kind, int CAP, bool GLOBAL = false, int WPG = 1>
__device__ void run_worker(const typename Kind::Ctx &ctx, const PoolView &pool, SchedGlobals *g,
                           const SchedConfig &cfg, WaveStack<Kind, CAP> &st, bool seed_roots,
                           Inbox<Kind> *ib = nullptr, uint32_t wave = 0, uint32_t worker = 0xffffffffu) {
    constexpr int TW = Kind::kTmplWords;
    constexpr uint32_t M = CAP - 1;
    constexpr int kPieces = pieces_of<Kind>();
    constexpr int kGroupMax = group_max_of<Kind>();
    // a push never comes within kGroupMax of the ring bottom: a spill may
    // leave the bottom item's template up to kGroupMax-1 slots below `bot`
    constexpr uint32_t kRoom = CAP - kGroupMax;
    static_assert(CAP >= kWaveSize * kGroupMax + kGroupMax, "ring must hold one batch's pushes");
    const int lane = lane_id();
    const uint32_t gid = worker != 0xffffffffu ? worker : blockIdx.x;
    GlobalView gv;
    if constexpr (GLOBAL) gv = g->gview;
    uint32_t gidle_pf = 0, gidle = 0;  // GLOBAL: idle ranks, read with the hunger signal
    const uint32_t qpx = pool.nq / 8;
    const uint32_t xcc = xcc_id() & 7u;
    const uint32_t home = xcc * qpx + (gid / 8) % qpx;
    uint32_t rng = 0x9e3779b9u ^ (gid * 0x85ebca6bu + 1u);

    typename Kind::Acc acc;
    acc_set_wid(acc, gid);
    Timeline tl;
    tl.init(g, gid);
    tl.log(kTlStart, 0);
    ProbeStats pstat;
    uint32_t bot = 0, top = 0;
    bool active = false;
    uint32_t spins = 0;
    unsigned long long idle_since = 0;
    // event counts fit 32 bits per wave (a wave runs < 2^32 batches); the
    // 64-bit cycle sums and stamps stay 64-bit. Fewer live SGPR pairs: the
    // batch loop's scalar state then spills less (v_writelane/readlane)
    uint32_t nbatch = 0, npush = 0, nsteal = 0;
    unsigned long long cyc_form = 0, cyc_proc = 0, cyc_push = 0;  // HX_STAMPS builds only
    // HX_PHASES builds: main-loop single batches split at four s_memtime
    // stamps: loop top -> pop issued -> pop landed -> body done -> batch end
    unsigned long long ph_sum[6] = {0, 0, 0, 0, 0, 0}, ph_n = 0, ph_a = 0, ph_b = 0, ph_c = 0, ph_d = 0, ph_m = 0,
                       ph_p = 0;
    bool ph_single = false;
    uint32_t tag = 1;  // mark tags: 16 per batch
    for (int i = lane; i < kWaveSize; i += kWaveSize) st.mark[i] = 0;
    if (lane < 8) st.stolen_from[lane] = 0;
    uint32_t n_exec = 0, n_spawn = 0;          // per lane: tasks run, children created
    uint32_t items_stolen = 0;
    uint32_t n_narrow = 0, n_narrow_in = 0;
    // register carry: the previous batch's `carry` outputs, lane o holding
    // item o (template ctmpl, child index ck); they form the front of the
    // next batch instead of round-tripping through the LDS ring
    uint32_t carry = 0, ck = 0;
    uint32_t ctmpl[TW];
    PendingChunk pend;  // a spilled chunk waiting for its publish (see PendingChunk)
    pend.live = false;
    uint32_t occ = 0;   // deque occupancy seen at the last enqueue
#pragma unroll
    for (int i = 0; i < TW; ++i) ctmpl[i] = 0;

    bool seeded = false;
    if constexpr (Kind::kPure && Kind::kTmplWords == 6 && Kind::kWords == 8 && CAP >= 128) {
        if (g->seed.buf) {
            // breadth-first seeding: every wave starts with its share of the
            // tree's top levels (the host set outstanding = every wave)
            seeded = true;
            top = seed_levels<Kind, CAP>(ctx, acc, g, st, gid, cfg.nwaves, cfg.spin_limit, n_exec, n_spawn, nbatch, tl);
            st.mark[lane] = 0;  // (the seeding's window marks)
            active = true;
            tl.log(kTlBusy, top);
            if (top == 0) {
                active = false;
                wave_goes_idle<GLOBAL>(g, gv, pool);
            }
        }
    }
    if constexpr (kind_has_seed<Kind>::value) {
        // a Kind's own seeding (fib: the call tree's top levels, HBM scopes):
        // every wave starts with its share; the host set outstanding = every wave
        if (!seeded && Kind::seeding(ctx)) {
            seeded = true;
            top = lane0(Kind::seed(ctx, acc, st, gid, cfg.nwaves, cfg.spin_limit, &g->err));
            active = true;
            tl.log(kTlBusy, top);
            if (top == 0) {
                active = false;
                wave_goes_idle<GLOBAL>(g, gv, pool);
            }
        }
    }
    if (seed_roots && !seeded) {
        uint32_t tmpl[TW];
        const int n = Kind::roots(ctx, acc, tmpl);  // uniform across the wave
        uint32_t ucnt = lane == 0 && n > 0 ? (uint32_t)n : 0u;
        if (ucnt >= kMaxChildren) {
            dev_error(&g->err, kErrBadTask);
            ucnt = 0;
        }
        const uint32_t nch = ucnt > (uint32_t)kPieces ? (uint32_t)kPieces : ucnt;
        const uint32_t tout = lane0(nch);
        push_outputs<Kind, CAP>(st, 0, 0, tout, 0, ucnt, nch, tmpl, tmpl, 0, 0, tag);
        tag += 16;
        top = tout;
        active = true;  // the host initialised outstanding = 1 for this wave
        tl.log(kTlBusy, tout);
        if (top == 0) {
            active = false;
            wave_goes_idle<GLOBAL>(g, gv, pool);
        }
    }

    // busy/idle time is stamped only at busy<->idle transitions (a per-batch
    // s_memtime would wait for every LDS write of the batch); the per-phase
    // stamps of cfg.stamps are a diagnostic build that pays that wait
    unsigned long long t_mark = __builtin_amdgcn_s_memtime();
    if (lane < 6) st.cyc[lane] = 0;
    if (lane == 0) {
        st.cyc[4] = t_mark;
        st.cyc[5] = __builtin_amdgcn_s_memrealtime();
    }
    unsigned long long t_batch = t_mark;  // cfg.stamps only
    bool busy_phase = true;
    // lane 0: `outstanding` as loaded one batch ago. Until the first load
    // lands it reads 0, "every wave hungry": true for an unseeded launch (one
    // busy wave), and for a seeded one (every wave busy) an early rebalancing
    // of the seeded shares, which measured faster on the GEO trees (T1 0.20 vs
    // 0.22-0.23 ms, T1XL 30.8 vs 31.5) and slower on fib (0.40 vs 0.39 ms):
    // cfg.hunger_init_full picks (profiles/r06/ab_outstpf.log)
    uint32_t outst_pf = seeded && cfg.hunger_init_full ? cfg.nwaves : 0u;
    uint32_t outst_cur = 0, hunger_in = 0;
    // nothing from the set-up stays in flight into the loop: a load whose
    // register the loop's first batch body overwrites would make the
    // compiler wait (vmcnt(0)) there in every batch, and so for the
    // one-batch-late hunger read
    vm_drain();
    while (true) {
        // the ring bounds are wave-uniform: pin them to SGPRs (the uniformity
        // analysis cannot see through the loop's exits) so the batch's
        // bookkeeping is scalar and its branches are s_cbranch_scc
        top = lane0(top);
        bot = lane0(bot);
        carry = lane0(carry);
        const uint32_t size = top - bot;
        if (size == 0 && carry == 0) {
            publish_pending<Kind, CAP>(pool, g, pend);
            if (busy_phase) {
                const unsigned long long now = __builtin_amdgcn_s_memtime();
                lds_sum(st, 0, now - t_mark);
                t_mark = now;
                busy_phase = false;
            }
            if (active) {
                kind_drain<Kind>(ctx, acc, &g->err);
                active = false;
                wave_goes_idle<GLOBAL>(g, gv, pool);
                tl.log(kTlIdle, 0);
                if constexpr (WPG > 1) {
                    if (lane == 0) lds_store(&ib[wave].idle, 1u);
                }
            }
            // a sibling's inbox first (LDS, no round trip), then the deques.
            // Probe order: home, a hint (the last deque pushed in an XCD's
            // slice: this wave's own XCD first, then the others in turn), then
            // random (3/4 same XCD, 1/4 anywhere)
            uint32_t n = 0, src = 0;
            uint32_t q = home;
            if constexpr (WPG > 1) {
                n = inbox_take<Kind, CAP>(ctx, ib[wave], st);  // inherits the chunk's unit
                if (n) src = 3;
            }
            uint32_t fin = 0;
            if (n == 0) {
                const uint32_t phase = spins % 3;
                if (phase == 1) {
                    uint32_t hq = 0;
                    if (lane == 0) hq = ld_agent(&g->hints[64u * ((xcc + spins / 3u) & 7u)]);
                    q = lane0(hq) % pool.nq;
                } else if (phase == 2) {
                    uint32_t r = lane0(xorshift(rng));
                    q = ((r & 3) != 0) ? xcc * qpx + (r >> 2) % qpx : (r >> 2) % pool.nq;
                }
                n = dequeue_chunk<Kind, CAP>(ctx, pool, q, st, g, fin, pstat);
                src = q == home ? 1 : 2;
            }
            if constexpr (!GLOBAL) {
                // the launch's last holder flagged every deque (wave_goes_idle)
                if (fin) {
                    tl.log(kTlTerm, 0);
                    break;
                }
            }
            if constexpr (WPG > 1) {
                if (n && lane == 0) lds_store(&ib[wave].idle, 0u);
            }
            if constexpr (GLOBAL) {
                // every 4th probe that found nothing local: the global ring
                if (n == 0 && (spins & 3) == 3) {
                    n = global_dequeue<Kind, CAP>(gv, pool.chunk * (uint32_t)Kind::kWords, st, &g->err);
                    if (n && lane == 0) {
                        // this wave now holds work; a rank that had none takes
                        // its unit of `active` back before the chunk's is
                        // returned, once the release that gave it up has landed
                        // (handshake: held 0 -> 1; see GlobalHdr::held)
                        const uint32_t prev = add_agent(&g->outstanding, 1u);
                        if (prev == 0u) {
                            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                            while (true) {
                                uint32_t z = 0u;
                                if (__hip_atomic_compare_exchange_strong(&gv.hdr->held[gv.rank], &z, 1u,
                                                                         __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_SYSTEM))
                                    break;
                                if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                                    dev_error(&g->err, kErrSpinTimeout);
                                    dev_error_sys(&gv.hdr->err, kErrSpinTimeout);
                                    break;
                                }
                                __builtin_amdgcn_s_sleep(1);
                            }
                            add_sys(&gv.hdr->active, 1u);
                            add_sys(&gv.hdr->idle, (uint32_t)-1);
                        }
                        add_sys(&gv.hdr->active, (uint32_t)-1);
                    }
                    if (n) {
                        q = home;  // (not counted as a local steal)
                        src = 4;
                    }
                }
            }
            if (n) {
                tl.log(kTlBusy, n | src << 16);
                if (q != home) {
                    ++nsteal;
                    items_stolen += n;
                    if (lane == 0) st.stolen_from[(q / qpx) & 7u] += 1;
                }
                bot = 0;
                top = n;
                active = true;
                spins = 0;
                const unsigned long long now = __builtin_amdgcn_s_memtime();
                lds_sum(st, 1, now - t_mark);
                t_mark = now;
                t_batch = now;
                busy_phase = true;
                continue;
            }
            // termination / error check: `outstanding` is one line that every
            // idle wave would otherwise poll, and the busy waves' spills and
            // hunger reads queue behind those polls. A local launch learns of
            // its end from the deque headers (above) and reads the two words
            // only every 64th probe (the error word, and a backstop); a
            // sharing launch (GLOBAL) every 8th, its end being another count
            if ((spins & (GLOBAL ? 7u : 63u)) == (GLOBAL ? 7u : 63u)) {
                uint32_t outst = 0, e = 0;
                if (lane == 0) {
                    outst = ld_agent(&g->outstanding);
                    e = ld_agent(&g->err);
                }
                vm_drain();  // both loads land on every path (no phantom waits in the batch loop)
                if (lane0(e)) break;
                if (lane0(outst) == 0) {
                    if constexpr (!GLOBAL) {
                        tl.log(kTlTerm, 0);
                        break;
                    } else {
                        // no local work: the launch ends when no rank holds any
                        uint32_t ga = 0;
                        if (lane == 0) ga = ld_sys(&gv.hdr->active);
                        vm_drain();
                        if (lane0(ga) == 0) {
                            tl.log(kTlTerm, 0);
                            break;
                        }
                    }
                }
                if constexpr (GLOBAL) {
                    // another rank hit a protocol error: stop promptly
                    uint32_t ge = 0;
                    if (lane == 0) ge = ld_sys(&gv.hdr->err);
                    vm_drain();
                    if (lane0(ge)) {
                        if (lane == 0) dev_error(&g->err, ge);
                        break;
                    }
                }
                outst_pf = outst;  // fresh hunger signal for the first batch after a steal
                hunger_in = 0;
            }
            // bounded idle: 100 MHz constant clock, cfg.spin_limit in ms
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (spins++ == 0) idle_since = now;
            else if (now - idle_since > 100000ull * cfg.spin_limit) {
                if (lane == 0) dev_error(&g->err, kErrSpinTimeout);
                break;
            }
            // back off so idle pollers do not saturate the deque heads
            // (cfg.backoff: the longest sleep, 16 = 1024 clocks). With
            // siblings the sleep is cut into 64-clock naps that watch this
            // wave's inbox (an LDS read): a sibling's hand-off is taken within
            // one nap instead of after the sleep and the next deque probe
            if constexpr (WPG > 1) {
                const uint32_t naps = (spins < 8 || cfg.backoff <= 1) ? 1u : (spins < 64 || cfg.backoff <= 4) ? 3u : 8u;
                for (uint32_t i = 0; i < naps; ++i) {
                    __builtin_amdgcn_s_sleep(1);
                    if (lane0(lds_load(&ib[wave].state)) == 1u) break;
                }
            } else {
                if (spins < 8 || cfg.backoff <= 1) __builtin_amdgcn_s_sleep(1);
                else if (spins < 64 || cfg.backoff <= 4) __builtin_amdgcn_s_sleep(4);
                else __builtin_amdgcn_s_sleep(16);
            }
            continue;
        }
        ++nbatch;
        if (HX_PHASES) {
            ph_a = __builtin_amdgcn_s_memtime();
            ph_single = false;
        }
        // hunger signal: use the value loaded one batch ago (its latency hid
        // behind that whole batch), then issue the load for the next batch
        // (loaded every cfg.hunger batches; consumed that many batches later).
        // Narrow frontier: a batch of carried items only, with an empty ring
        // and spill_lo above one batch, can neither spill nor be kept from
        // carrying by hunger, so it neither reads nor waits for the signal:
        // the span-bound chain of a narrow tree runs carry to carry.
        const bool narrow = carry > 0 && size == 0 && cfg.spill_lo > (uint32_t)kWaveSize;
        uint32_t outst = cfg.nwaves;
        if (cfg.hunger && !narrow) {
            if (hunger_in == 0) {
                outst_cur = lane0(outst_pf);
                if (lane == 0) outst_pf = ld_agent(&g->outstanding);
                if constexpr (GLOBAL) {
                    gidle = lane0(gidle_pf);
                    if (lane == 0) gidle_pf = ld_sys(&gv.hdr->idle);
                }
                // many hungry waves (ramp-up, a narrowing tree): read again
                // soon; otherwise every cfg.hunger batches
                const uint32_t hg = cfg.nwaves > outst_cur ? cfg.nwaves - outst_cur : 0u;
                hunger_in = hg * 8u > cfg.nwaves ? (cfg.hunger + 3u) / 4u : cfg.hunger;
            }
            --hunger_in;
            outst = outst_cur;
        }
        // a push that would come near live items first moves the oldest
        // items out as chunks (rare: only bursts of wide nodes)
        auto make_room = [&](uint32_t tout) -> bool {
            unsigned long long full_since = 0;
            while ((top - bot) + tout > kRoom) {
                uint32_t n = top - bot;
                if (n > pool.chunk) n = pool.chunk;
                bool ok = false;
                for (uint32_t a = 0; a < pool.nq && !ok; ++a)
                    ok = enqueue_chunk<Kind, CAP>(ctx, pool, g, (home + a) % pool.nq, st, bot, n, occ, pend, false);
                // every deque is at its half mark: fill one past it rather than wait
                for (uint32_t a = 0; a < pool.nq && !ok; ++a)
                    ok = enqueue_chunk<Kind, CAP>(ctx, pool, g, (home + a) % pool.nq, st, bot, n, occ, pend, false,
                                                  true);
                if (!ok) {
                    // every deque is full: other waves are draining them, so wait
                    // (bounded) rather than fail at once
                    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                    if (full_since == 0) full_since = now;
                    uint32_t e = 0;
                    if (lane == 0) e = ld_agent(&g->err);
                    if (lane0(e) || now - full_since > 100000ull * cfg.spin_limit) {
                        if (lane == 0) dev_error(&g->err, kErrStackOverflow);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                    continue;
                }
                ++npush;
                tl.log(kTlSpill, n);
                bot += n;
            }
            return (top - bot) + tout <= kRoom;
        };
        uint32_t tout = 0;
        bool dual = false;
        if constexpr (KindHasDual<Kind>::value && CAP >= 2 * kWaveSize * kGroupMax + kGroupMax) {
            // ---- dual batch: a wave holding more than one batch of ring items
            // (and nothing carried) runs two per lane, item A = top-1-lane,
            // item B = top-65-lane, their bodies interleaved (process2)
            dual = cfg.dual && carry == 0 && size > (uint32_t)kWaveSize;
            if (dual) {
                const uint32_t take2 = size < 2u * kWaveSize ? size : 2u * kWaveSize;
                const bool hasB = (uint32_t)lane + kWaveSize < take2;
                uint32_t tA[TW], tB[TW], cA[TW], cB[TW];
                const uint32_t pA = top - 1 - (uint32_t)lane, pB = pA - (uint32_t)kWaveSize;
                const uint2 dA = st.d[pA & M], dB = st.d[pB & M];
                const uint32_t kA = dA.x, kendA = dA.y & (kMaxChildren - 1);
                const uint32_t kB = dB.x, kendB = hasB ? dB.y & (kMaxChildren - 1) : kB + 1;
                load_tmpl<Kind, CAP>(st, (pA - (dA.y >> 24)) & M, tA);
                load_tmpl<Kind, CAP>(st, (pB - (dB.y >> 24)) & M, tB);
                int ncA = 0, ncB = 0;
                Kind::process2(ctx, acc, tA, kA, cA, ncA, tB, kB, cB, ncB, &g->err, hasB);
                after_body<TW>(cA);
                after_body<TW>(cB);
                publish_pending<Kind, CAP>(pool, g, pend);
                top -= take2;
                const uint32_t rA = kendA - kA - 1u, rB = hasB ? kendB - kB - 1u : 0u;
                const uint32_t nresA = rA == 0 ? 0u : (rA < kResidualSplitMin ? 1u : 2u);
                const uint32_t nresB = rB == 0 ? 0u : (rB < kResidualSplitMin ? 1u : 2u);
                const uint32_t uA = ncA > 0 ? (uint32_t)ncA : 0u, uB = (hasB && ncB > 0) ? (uint32_t)ncB : 0u;
                const uint32_t nchA = uA > (uint32_t)kPieces ? (uint32_t)kPieces : uA;
                const uint32_t nchB = uB > (uint32_t)kPieces ? (uint32_t)kPieces : uB;
                n_exec += hasB ? 2u : 1u;
                n_spawn += uA + uB;
                const int nout = (int)(nresA + nchA + nresB + nchB);
                const int P = wave_scan_add(nout);
                tout = (uint32_t)lane63(P);
                const uint32_t excl = (uint32_t)(P - nout);
                if (!make_room(tout)) break;  // error already recorded
                push_group<Kind, CAP>(st, top + excl, nresA, uA, nchA, tA, cA, kA, kendA);
                push_group<Kind, CAP>(st, top + excl + nresA + nchA, nresB, uB, nchB, tB, cB, kB, kendB);
                top += tout;
            }
        }
        if (!dual) {
        // ---- a batch = the carried items, then the top items of the ring,
        // min(carry + size, 64) in all, one per lane
        const uint32_t room = (uint32_t)kWaveSize - carry;
        const uint32_t take_ring = size < room ? size : room;
        const uint32_t take = carry + take_ring;
        const bool has = (uint32_t)lane < take;
        uint32_t tmpl[TW], child[TW];
        uint32_t k = 0, kend = 0;
        int cnt = 0;
        unsigned long long ts0 = 0;
        if (HX_STAMPS && cfg.stamps) ts0 = __builtin_amdgcn_s_memtime();
        if (HX_PHASES) {
            ph_b = __builtin_amdgcn_s_memtime();
            ph_single = true;
        }
        // a batch of carried items only (take_ring == 0) loads nothing from
        // the ring: its idle lanes run (pure kinds) on a carried template
        if ((uint32_t)lane < carry || take_ring == 0) {
#pragma unroll
            for (int i = 0; i < TW; ++i) tmpl[i] = ctmpl[i];
            k = ck;
            kend = ck + 1;
        } else if (Kind::kPure || has) {  // pure kinds: every lane loads (slots wrap inside the ring)
            const uint32_t p = top - 1 - ((uint32_t)lane - carry);
            const uint2 dd = st.d[p & M];
            k = dd.x;
            kend = has ? dd.y & (kMaxChildren - 1) : k + 1;
            load_tmpl<Kind, CAP>(st, (p - (dd.y >> 24)) & M, tmpl);
        }
        carry = 0;
        if (HX_PHASES) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            ph_c = __builtin_amdgcn_s_memtime();
        }
        unsigned long long tsl = 0;
        if (HX_STAMPS && cfg.stamps) {
            // diagnostic build only: form = loop top + pop (LDS loads landed)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            tsl = __builtin_amdgcn_s_memtime();
            cyc_form += tsl - t_batch;
            ts0 = tsl;
        }
        if constexpr (Kind::kPure) {
            cnt = Kind::process(ctx, acc, tmpl, k, child, &g->err, has);
        } else {
            if (has) cnt = Kind::process(ctx, acc, tmpl, k, child, &g->err, true);
        }
        // the previous batch's spilled chunk: its payload stores landed while
        // this batch ran (after_body: the body's register-only work would
        // otherwise be scheduled after the publish, whose drain then waited
        // for those stores' whole round trip before the body)
        after_body<TW>(child);
        if (HX_PHASES) {
#pragma unroll
            for (int i = 0; i < TW; ++i) asm volatile("" ::"v"(child[i]));
            ph_d = __builtin_amdgcn_s_memtime();
        }
        publish_pending<Kind, CAP>(pool, g, pend);
        if (HX_STAMPS && cfg.stamps) {
            const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
            cyc_proc += ts1 - tsl;
        }
        top -= take_ring;
        // ---- push: residual range of the item + the new task's children
        const uint32_t rlen = has ? kend - k - 1u : 0u;
        const uint32_t nres = rlen == 0 ? 0u : (rlen < kResidualSplitMin ? 1u : 2u);
        uint32_t ucnt = cnt > 0 ? (uint32_t)cnt : 0u;
        n_exec += has ? 1u : 0u;
        n_spawn += has ? ucnt : 0u;
        if (!Kind::kBoundedChildren && ucnt >= kMaxChildren) {
            dev_error(&g->err, kErrBadTask);
            ucnt = 0;
        }
        const uint32_t nch = ucnt > (uint32_t)kPieces ? (uint32_t)kPieces : ucnt;
        // uniform batch (see push_uniform): group size of the first spawning lane
        const unsigned long long spawn = __ballot(nch != 0);
        const uint32_t mu = spawn ? (uint32_t)__builtin_amdgcn_readlane((int)nch, __builtin_ctzll(spawn)) : 0u;
        const bool uniform = __ballot(nres != 0 || ucnt > (uint32_t)kPieces || (nch != 0 && nch != mu)) == 0;
        uint32_t excl;
        int nout = 0;
        if (uniform) {
            excl = mu * (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(spawn >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)spawn, 0u));
            tout = mu * (uint32_t)__builtin_popcountll(spawn);
        } else {
            nout = (int)(nres + nch);
            const int P = wave_scan_add(nout);
            tout = (uint32_t)lane63(P);
            excl = (uint32_t)(P - nout);
        }
        // register carry: a uniform batch whose outputs fit one batch keeps
        // them in registers as the front of the next batch — unless a hungry
        // wave could be given items from the ring (then they go through it).
        // Output o is child o % mu of the spawning lane of rank o / mu: one
        // ds_permute tells rank r its source lane, two ds_bpermute hops bring
        // the template to lane o.
        {
            const uint32_t hungry0 = cfg.nwaves > outst ? cfg.nwaves - outst : 0;
            if (cfg.carry && uniform && tout > 0 && tout <= (uint32_t)kWaveSize &&
                !(hungry0 > 0 && (top - bot) + tout >= cfg.spill_lo)) {
                if constexpr (WaveStack<Kind, CAP>::kCarryLds) carry_lds<TW>(st.cscr, spawn, mu, child, ctmpl, ck);
                else carry_permute<TW>(spawn, mu, nch, child, ctmpl, ck);
                carry = tout;
                if (HX_STAMPS && cfg.stamps) cyc_push += __builtin_amdgcn_s_memtime() - ts0;
                if (HX_STAMPS && cfg.stamps) t_batch = __builtin_amdgcn_s_memtime();
                // Narrow frontier (span-bound trees): the ring is empty and no
                // hunger can stop a carry of at most one batch (spill_lo above
                // it), so the chain runs in a tight loop of its own: process the
                // carried items, carry their children, nothing else — no ring,
                // no hunger reads, no spill checks. It leaves when the batch has
                // no children (the wave goes idle at the loop top) or outputs
                // that do not carry (non-uniform, or more than one batch): those
                // go onto the empty ring and the main loop takes over.
                if (cfg.carry > 1 && top == bot && cfg.spill_lo > (uint32_t)kWaveSize && !(HX_STAMPS && cfg.stamps)) {
                    const unsigned long long tn0 = __builtin_amdgcn_s_memtime();
                    NarrowState<TW> ns;
#pragma unroll
                    for (int i = 0; i < TW; ++i) ns.ctmpl[i] = ctmpl[i];
                    ns.ck = ck;
                    ns.carry = carry;
                    ns.top = top;
                    ns.tag = tag;
                    ns.n_exec = n_exec;
                    ns.n_spawn = n_spawn;
                    ns.batches = 0;
                    ns = narrow_loop<Kind, CAP>(ctx, acc, &g->err, st, ns);
#pragma unroll
                    for (int i = 0; i < TW; ++i) ctmpl[i] = ns.ctmpl[i];
                    ck = ns.ck;
                    carry = lane0(ns.carry);
                    top = lane0(ns.top);
                    tag = lane0(ns.tag);
                    n_exec = ns.n_exec;
                    n_spawn = ns.n_spawn;
                    nbatch += lane0(ns.batches);
                    n_narrow += lane0(ns.batches);
                    lds_sum(st, 3, __builtin_amdgcn_s_memtime() - tn0);
                    ++n_narrow_in;
                }
                continue;
            }
        }
        if (HX_PHASES) ph_m = __builtin_amdgcn_s_memtime();
        if (!make_room(tout)) break;  // error already recorded
        if (uniform) {
            push_uniform<Kind, CAP>(st, top, excl, tout, mu, nch != 0, child);
        } else {
            push_outputs<Kind, CAP>(st, top, excl, tout, nres, ucnt, nch, tmpl, child, k, kend, tag);
            tag += 16;
        }
        top += tout;
        if (HX_STAMPS && cfg.stamps) cyc_push += __builtin_amdgcn_s_memtime() - ts0;
        }  // single batch
        if (HX_PHASES) ph_p = __builtin_amdgcn_s_memtime();
        // ---- give the oldest items to hungry waves, or relieve a full ring
        uint32_t sz = top - bot;
        uint32_t hungry = cfg.nwaves > outst ? cfg.nwaves - outst : 0;
        const uint32_t lo = cfg.spill_lo;
        if (sz > cfg.spill_hi || (hungry > 0 && sz >= lo)) {
            const unsigned long long ts = __builtin_amdgcn_s_memtime();
            const uint32_t cmax = pool.chunk;
            uint32_t nsp = 0;
            while (sz > cfg.spill_hi || (hungry > 0 && sz >= lo)) {
                uint32_t n = (sz + 1) / 2;
                if (n > cmax) n = cmax;
                if (n == 0 || n == sz) break;
                // home deque first, then the other deques of this XCD slice
                bool ok = false;
                if constexpr (WPG > 1) {
                    // an idle sibling of this workgroup first (LDS, no HBM
                    // round trip); every sibling's flags read in one go
                    uint32_t sid[WPG], sst[WPG];
#pragma unroll
                    for (uint32_t a = 1; a < (uint32_t)WPG; ++a) {
                        sid[a] = lds_load(&ib[(wave + a) % (uint32_t)WPG].idle);
                        sst[a] = lds_load(&ib[(wave + a) % (uint32_t)WPG].state);
                    }
#pragma unroll
                    for (uint32_t a = 1; a < (uint32_t)WPG; ++a)
                        if (!ok && lane0(sid[a]) == 1u && lane0(sst[a]) == 0u)
                            ok = inbox_put<Kind, CAP>(ctx, ib[(wave + a) % (uint32_t)WPG], st, bot, n, g);
                }
                if (!ok) publish_pending<Kind, CAP>(pool, g, pend);  // one deferred chunk at a time
                // where the chunk goes: the home deque first, then the XCD's others
                for (uint32_t a = 0; a < qpx && !ok; ++a) {
                    const uint32_t q = xcc * qpx + (home - xcc * qpx + a) % qpx;
                    ok = enqueue_chunk<Kind, CAP>(ctx, pool, g, q, st, bot, n, occ, pend, cfg.defer != 0);
                }
                if (!ok) break;  // deques full: keep the items (the ring still has room)
                ++npush;
                tl.log(kTlSpill, n);
                bot += n;
                sz = top - bot;
                if (hungry) --hungry;
                if (cfg.spills && ++nsp >= cfg.spills && sz <= cfg.spill_hi) break;
            }
            lds_sum(st, 2, __builtin_amdgcn_s_memtime() - ts);
        }
        if constexpr (GLOBAL) {
            // another rank is idle and no wave of this one is hungry: export
            // the oldest items (one chunk per batch)
            if (hungry == 0 && (int)gidle > 0 && sz >= cfg.spill_lo) {
                uint32_t n = (sz + 1) / 2;
                if (n > pool.chunk) n = pool.chunk;
                publish_pending<Kind, CAP>(pool, g, pend);
                if (n > 0 && n < sz &&
                    global_enqueue<Kind, CAP>(ctx, gv, pool.chunk * (uint32_t)Kind::kWords, st, bot, n, &g->err)) {
                    bot += n;
                    sz = top - bot;
                    --gidle;
                }
            }
        }
        if (HX_STAMPS && cfg.stamps) t_batch = __builtin_amdgcn_s_memtime();
        if (HX_PHASES && ph_single) {
            const unsigned long long ph_e = __builtin_amdgcn_s_memtime();
            ph_sum[0] += ph_b - ph_a;
            ph_sum[1] += ph_c - ph_b;
            ph_sum[2] += ph_d - ph_c;
            ph_sum[3] += ph_e - ph_d;
            ph_sum[4] += ph_m - ph_d;  // body -> push begins (carry decision, publish)
            ph_sum[5] += ph_p - ph_m;  // the push
            ++ph_n;
        }
    }
    publish_pending<Kind, CAP>(pool, g, pend);  // (error exits)
    if constexpr (WPG > 1) {
        // close this wave's inbox: no sibling may hand it work any more
        if (lane == 0) {
            lds_store(&ib[wave].idle, 0u);
            (void)lds_cas(&ib[wave].state, 0u, 3u);
        }
    }
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
    lds_sum(st, busy_phase ? 0 : 1, t_end - t_mark);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the LDS sums have landed
    const unsigned long long cyc_busy = st.cyc[0], cyc_idle = st.cyc[1], cyc_spill = st.cyc[2],
                             cyc_narrow = st.cyc[3], t_begin = st.cyc[4], rt_begin = st.cyc[5];
    if (active) {
        // only reached on an error break: keep the protocol consistent
        wave_goes_idle<GLOBAL>(g, gv, pool);
    }
    const bool rec = g->wave_ctr && gid < g->wave_ctr_cap;
    unsigned long long kc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, km[4] = {0, 0, 0, 0};
    if constexpr (acc_has_totals<typename Kind::Acc>::value) {
        acc.totals(kc, km);
        if (!rec && lane == 0) {
            for (int i = 0; i < 8; ++i)
                if (kc[i]) add_agent(&g->counters[i], kc[i]);
            for (int i = 0; i < 4; ++i)
                if (km[i]) __hip_atomic_fetch_max(&g->maxes[i], km[i], __ATOMIC_RELAXED, HX_AGENT);
        }
    } else {
        acc.flush(g);
    }
    {
        // this wave's record (plain stores: the host reads it after the launch)
        const unsigned long long ex = wave_sum((unsigned long long)n_exec),
                                 sp = wave_sum((unsigned long long)n_spawn);
        if (g->wave_stats && gid < g->wave_stats_cap && lane < 16) {
            unsigned long long v = 0;
            switch (lane) {
            case 0: v = ex; break;
            case 1: v = sp; break;
            case 2: v = nbatch; break;
            case 3: v = npush; break;
            case 4: v = nsteal; break;
            case 5: v = items_stolen; break;
            case 6: v = xcc; break;
            case 7: v = 0; break;
            default: v = st.stolen_from[lane - 8]; break;
            }
            ((unsigned long long *)&g->wave_stats[gid])[lane] = v;
        }
    }
    const unsigned long long c_push = (HX_STAMPS && cfg.stamps) ? cyc_push - cyc_proc : 0,
                             c_form = (HX_STAMPS && cfg.stamps) ? cyc_form : 0,
                             c_proc = (HX_STAMPS && cfg.stamps) ? cyc_proc : 0;
    if (rec) {
        // one store instruction: lane i writes word i of the record
        unsigned long long v = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (lane == i) v = kc[i];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (lane == 16 + i) v = km[i];
        switch (lane) {
        case 8 + kCtrProcCycles - 8: v = c_proc; break;
        case 8 + kCtrBusyCycles - 8: v = cyc_busy; break;
        case 8 + kCtrIdleCycles - 8: v = cyc_idle; break;
        case 8 + kCtrSpillCycles - 8: v = cyc_spill; break;
        case 8 + kCtrWaves - 8: v = 1; break;
        case 8 + kCtrBatches - 8: v = nbatch; break;
        case 8 + kCtrPushed - 8: v = npush; break;
        case 8 + kCtrStolen - 8: v = nsteal; break;
        case 20: v = n_narrow_in ? (unsigned long long)n_narrow : 0; break;
        case 21: v = n_narrow_in ? cyc_narrow : 0; break;
        case 22: v = n_narrow_in; break;
        case 23: v = ph_n; break;
        case 28: v = ph_sum[0]; break;
        case 29: v = ph_sum[1]; break;
        case 30: v = ph_sum[2]; break;
        case 31: v = ph_sum[3]; break;
        case 24 + kCtrPushCycles - 4: v = HX_PHASES ? ph_sum[4] : c_push; break;
        case 24 + kCtrClockTicks - 4: v = t_end - t_begin; break;
        case 24 + kCtrRealTicks - 4: v = rt_end - rt_begin; break;
        case 24 + kCtrFormCycles - 4: v = HX_PHASES ? ph_sum[5] : c_form; break;
        default: break;
        }
        if (lane < kWaveCtrWords) g->wave_ctr[(size_t)gid * kWaveCtrWords + lane] = v;
    } else {
        if (lane == 0 && n_narrow_in) {
            add_agent(&g->narrow[0], (unsigned long long)n_narrow);
            add_agent(&g->narrow[1], cyc_narrow);
            add_agent(&g->narrow[2], (unsigned long long)n_narrow_in);
        }
        if (lane == 0) {
            add_agent(&g->counters[kCtrBusyCycles], cyc_busy);
            if (HX_STAMPS && cfg.stamps) {
                add_agent(&g->counters[kCtrFormCycles], c_form);
                add_agent(&g->counters[kCtrProcCycles], c_proc);
                add_agent(&g->counters[kCtrPushCycles], c_push);
            }
            add_agent(&g->counters[kCtrIdleCycles], cyc_idle);
            add_agent(&g->counters[kCtrSpillCycles], cyc_spill);
            add_agent(&g->counters[kCtrWaves], 1ull);
            add_agent(&g->counters[kCtrBatches], (unsigned long long)nbatch);
            add_agent(&g->counters[kCtrPushed], (unsigned long long)npush);
            add_agent(&g->counters[kCtrStolen], (unsigned long long)nsteal);
            add_agent(&g->counters[kCtrClockTicks], t_end - t_begin);
            add_agent(&g->counters[kCtrRealTicks], rt_end - rt_begin);
        }
    }
    tl.log(kTlEnd, 0);
    if (HX_TIMELINE) {
        auto sat = [](uint32_t v) { return v / 16u > 0xffffu ? 0xffffu : v / 16u; };
        tl.log(kTlProbe, 0u << 16 | sat(pstat.probes));
        tl.log(kTlProbe, 1u << 16 | sat(pstat.empty));
        tl.log(kTlProbe, 2u << 16 | sat(pstat.lost));
        tl.log(kTlProbe, 3u << 16 | sat(pstat.wait_us));
    }
}

}  // namespace hx
