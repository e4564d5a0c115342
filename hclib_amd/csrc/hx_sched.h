// hx_sched.h — the persistent work-stealing megakernel (device side).
//
// Replaces HClib's pthread worker loop and deques (src/hclib-runtime.c:646-729
// core_work_loop/find_and_run_task, src/hclib-deque.c:50-139) with a
// wavefront-granular scheduler:
//
//   worker        = one 64-lane wave (one workgroup of 64 threads), resident
//                   for the whole launch; a few per SIMD.
//   local deque   = a ring of task entries in the wave's LDS (the "LDS-cached
//                   hot end"); the owner pushes/pops at the top (LIFO,
//                   work-first like ss_get_work, test/uts/UTS.cpp:383-402).
//   spill/steal   = the oldest entries of a ring (the shallowest, largest
//                   subtrees) move as one chunk into an HBM chunk deque
//                   (bounded MPMC ring, two per XCD); idle waves take chunks
//                   from their own XCD's deques first, then the last deque
//                   pushed to, then anywhere — the reference's
//                   intra-socket-first victim order
//                   (src/hclib-locality-graph.c:864-884) mapped to XCDs.
//   a "task"      = one lane-item: an entry carries a count of items
//                   (children to spawn, or 1); the wave expands up to 64 items
//                   per batch (one per lane) by prefix sum (DPP wave scans).
//   termination   = `outstanding` = chunks in deques + waves holding work;
//                   the launch ends when it reads 0 (the finish counter of
//                   src/hclib-runtime.c:431-446 for the whole launch).
//   hunger        = waves - outstanding = waves with neither work nor a
//                   queued chunk to take; a wave gives away its oldest
//                   entries only while that is > 0 (no chunk floods).
//
// All cross-wave words use agent-scope atomics; chunk payloads are written
// with sc1 stores and published behind s_waitcnt + release, consumed after an
// acquire (hx_common.h). Every spin is bounded.
#pragma once

#include "hx_common.h"

namespace hx {

constexpr int kWaveSize = 64;

// One HBM chunk deque header, head and tail on separate 128-B lines.
struct alignas(256) QueueHdr {
    uint32_t head;
    uint32_t pad0[31];
    uint32_t tail;
    uint32_t pad1[31];
};

// Global scheduler state shared by all waves of one launch (device memory).
struct alignas(256) SchedGlobals {
    uint32_t outstanding;  // chunks queued + waves holding work
    uint32_t pad0[63];
    uint32_t hint;  // deque most recently pushed to
    uint32_t pad1[63];
    uint32_t err;  // DevError
    uint32_t pad2[63];
    unsigned long long counters[16];  // [0..7] kind-specific, [8..15] scheduler
    unsigned long long maxes[4];      // kind-specific reductions (atomic max)
};

// scheduler counters (SchedGlobals::counters)
enum : int {
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
};

// Kind concept:
//   static constexpr int kWords;      // u32 words per entry; word kWords-1 = start
//   static constexpr int kMaxOut;     // entries one item may push
//   struct Ctx;                       // per-launch read-only parameters
//   struct Acc { ...; __device__ void flush(SchedGlobals*); };  // per-lane stats
//   __device__ static uint32_t count(const uint32_t *e);        // items in entry
//   __device__ static int process(const Ctx&, Acc&, const uint32_t *e, uint32_t k,
//                                 uint32_t (*out)[kWords], uint32_t *err);
//   __device__ static int roots(const Ctx&, Acc&, uint32_t (*out)[kWords]);  // wave 0 only

template <class Kind, int CAP>
struct WaveStack {
    static constexpr int W = Kind::kWords;
    uint32_t e[CAP][W];
    int own[kWaveSize];
};

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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// Try to publish `n` entries (ring positions bot..bot+n-1) as one chunk into
// deque q. Called by the whole wave; returns true if published.
template <class Kind, int CAP>
__device__ bool enqueue_chunk(const PoolView &pool, SchedGlobals *g, uint32_t q,
                              WaveStack<Kind, CAP> &st, uint32_t bot, uint32_t n) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    QueueHdr *h = &pool.hdr[q];
    uint32_t pos = 0;
    int ok = 0;
    if (lane == 0) {
        // a producer takes a ticket with ONE fetch-add (no CAS retry storms);
        // it only does so while the ring is at most half full, so a ticket
        // never waits behind a consumer that cannot come
        const uint32_t hd = ld_agent(&h->head), tl = ld_agent(&h->tail);
        if ((int)(tl - hd) < (int)(pool.cap / 2)) {
            add_agent(&g->outstanding, 1u);  // counts before it becomes visible
            pos = add_agent(&h->tail, 1u);
            ok = 1;
        }
    }
    if (!lane0((uint32_t)ok)) return false;
    pos = lane0(pos);
    const uint32_t slot = q * pool.cap + (pos & (pool.cap - 1));
    if (lane == 0) {
        // the slot is free once its previous lap was consumed (normally at once)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_agent(&pool.seq[slot]) != pos) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                dev_error(&g->err, kErrQueueFull);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    uint32_t *dst = pool.data + (size_t)slot * pool.chunk * W;
    for (uint32_t i = lane; i < n * W; i += kWaveSize) {
        uint32_t ent = i / W, w = i % W;
        st_agent(&dst[i], st.e[(bot + ent) & (CAP - 1)][w]);
    }
    if (lane == 0) st_agent(&pool.cnt[slot], n);
    handoff_publish();
    if (lane == 0) {
        st_agent(&pool.seq[slot], pos + 1);
        st_agent(&g->hint, q);
    }
    return true;
}

// Try to take one chunk from deque q into the (empty) stack. Returns the
// number of entries taken (0 if the deque looked empty).
template <class Kind, int CAP>
__device__ uint32_t dequeue_chunk(const PoolView &pool, uint32_t q, WaveStack<Kind, CAP> &st,
                                  SchedGlobals *g) {
    constexpr int W = Kind::kWords;
    const int lane = lane_id();
    QueueHdr *h = &pool.hdr[q];
    uint32_t pos = 0;
    int ok = 0;
    if (lane == 0) {
        // one claim attempt: a ticket below the tail, taken by CAS on the head
        const uint32_t hd = ld_agent(&h->head), tl = ld_agent(&h->tail);
        if ((int)(tl - hd) > 0 && cas_agent(&h->head, hd, hd + 1)) {
            pos = hd;
            ok = 1;
        }
    }
    if (!lane0((uint32_t)ok)) return 0;
    pos = lane0(pos);
    const uint32_t slot = q * pool.cap + (pos & (pool.cap - 1));
    if (lane == 0) {
        // the producer holds this ticket and is publishing it (bounded wait)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_agent(&pool.seq[slot]) != pos + 1) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s
                dev_error(&g->err, kErrSpinTimeout);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    handoff_consume();
    const uint32_t n = ld_agent(&pool.cnt[slot]);
    const uint32_t *src = pool.data + (size_t)slot * pool.chunk * W;
    for (uint32_t i = lane; i < n * W; i += kWaveSize) {
        uint32_t ent = i / W, w = i % W;
        st.e[ent][w] = ld_agent(&src[i]);
    }
    // all reads of the slot have landed before it is handed back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) st_agent(&pool.seq[slot], pos + pool.cap);
    __syncthreads();  // one wave per workgroup: orders the LDS ring writes
    return n;
}

__device__ __forceinline__ uint32_t xorshift(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

template <class Kind, int CAP>
__device__ void run_worker(const typename Kind::Ctx &ctx, const PoolView &pool, SchedGlobals *g,
                           const SchedConfig &cfg, WaveStack<Kind, CAP> &st, bool seed_roots) {
    constexpr int W = Kind::kWords;
    constexpr int MO = Kind::kMaxOut;
    static_assert((CAP & (CAP - 1)) == 0, "CAP must be a power of two");
    const int lane = lane_id();
    const uint32_t gid = blockIdx.x;
    const uint32_t qpx = pool.nq / 8;
    const uint32_t xcc = xcc_id() & 7u;
    const uint32_t home = xcc * qpx + (gid / 8) % qpx;
    uint32_t rng = 0x9e3779b9u ^ (gid * 0x85ebca6bu + 1u);

    typename Kind::Acc acc;
    uint32_t bot = 0, top = 0;
    bool active = false;
    uint32_t spins = 0;
    unsigned long long idle_since = 0;
    unsigned long long nbatch = 0, npush = 0, nsteal = 0;
    unsigned long long cyc_busy = 0, cyc_idle = 0, cyc_spill = 0, cyc_form = 0, cyc_proc = 0;

    if (seed_roots) {
        uint32_t out[MO > 4 ? MO : 4][W];
        int n = Kind::roots(ctx, acc, out);
        // roots() is uniform across the wave; lane 0's view is authoritative
        if (lane == 0)
            for (int i = 0; i < n; ++i)
                for (int w = 0; w < W; ++w) st.e[i][w] = out[i][w];
        top = n;
        active = true;  // the host initialised outstanding = 1 for this wave
        if (n == 0) {
            active = false;
            if (lane == 0) __hip_atomic_fetch_add(&g->outstanding, (uint32_t)-1, __ATOMIC_RELEASE, HX_AGENT);
        }
        __syncthreads();
    }

    unsigned long long t_mark = __builtin_amdgcn_s_memtime();
    uint32_t outst_pf = 0;  // lane 0: `outstanding` as loaded one batch ago
    while (true) {
        const uint32_t size = top - bot;
        if (size == 0) {
            if (active) {
                active = false;
                if (lane == 0)
                    __hip_atomic_fetch_add(&g->outstanding, (uint32_t)-1, __ATOMIC_RELEASE, HX_AGENT);
            }
            // probe order: home, hint, then random (3/4 same XCD, 1/4 anywhere)
            uint32_t q = home;
            const uint32_t phase = spins % 3;
            if (phase == 1) {
                uint32_t hq = 0;
                if (lane == 0) hq = ld_agent(&g->hint);
                q = lane0(hq) % pool.nq;
            } else if (phase == 2) {
                uint32_t r = lane0(xorshift(rng));
                q = ((r & 3) != 0) ? xcc * qpx + (r >> 2) % qpx : (r >> 2) % pool.nq;
            }
            uint32_t n = dequeue_chunk<Kind, CAP>(pool, q, st, g);
            if (n) {
                if (q != home) ++nsteal;
                bot = 0;
                top = n;
                active = true;
                spins = 0;
                const unsigned long long now = __builtin_amdgcn_s_memtime();
                cyc_idle += now - t_mark;
                t_mark = now;
                continue;
            }
            uint32_t outst = 0, e = 0;
            if (lane == 0) {
                outst = ld_agent(&g->outstanding);
                e = ld_agent(&g->err);
            }
            if (lane0(outst) == 0 || lane0(e)) break;
            outst_pf = outst;  // fresh hunger signal for the first batch after a steal
            // bounded idle: 100 MHz constant clock, cfg.spin_limit in ms
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (spins++ == 0) idle_since = now;
            else if (now - idle_since > 100000ull * cfg.spin_limit) {
                if (lane == 0) dev_error(&g->err, kErrSpinTimeout);
                break;
            }
            // back off so idle pollers do not saturate the deque heads
            if (spins < 8) __builtin_amdgcn_s_sleep(1);
            else if (spins < 64) __builtin_amdgcn_s_sleep(4);
            else __builtin_amdgcn_s_sleep(16);
            continue;
        }
        ++nbatch;
        // hunger signal: use the value loaded one batch ago (its latency hid
        // behind that whole batch), then issue the load for the next batch
        const uint32_t outst = lane0(outst_pf);
        if (lane == 0) outst_pf = ld_agent(&g->outstanding);
        // ---- form a batch of up to 64 items from the top entries
        uint32_t cnt = 0, start = 0, eidx = 0;
        if ((uint32_t)lane < size) {
            eidx = (top - 1 - lane) & (CAP - 1);
            start = st.e[eidx][W - 1];
            cnt = Kind::count(st.e[eidx]) - start;
        }
        const int S = wave_scan_add((int)cnt);
        const int total = lane63(S);
        const int take = total < kWaveSize ? total : kWaveSize;
        const int excl = S - (int)cnt;
        st.own[lane] = -1;
        __syncthreads();
        if (cnt > 0 && excl < kWaveSize) st.own[excl] = lane;
        __syncthreads();
        // item `lane` belongs to the last entry whose first item is <= lane:
        // two DPP max-scans give that entry and where its items start
        const int mark = st.own[lane];
        const int owner = wave_scan_max(mark);
        const int owner_excl = wave_scan_max(mark >= 0 ? lane : -1);
        const uint32_t owner_e = (top - 1 - (uint32_t)(owner < 0 ? 0 : owner)) & (CAP - 1);
        uint32_t out[MO][W];
        int nout = 0;
        unsigned long long ts0 = 0;
        if (cfg.stamps) ts0 = __builtin_amdgcn_s_memtime();
        if (lane < take) {
            uint32_t ent[W];
#pragma unroll
            for (int w = 0; w < W; ++w) ent[w] = st.e[owner_e][w];
            const uint32_t k = ent[W - 1] + (uint32_t)(lane - owner_excl);
            nout = Kind::process(ctx, acc, ent, k, out, &g->err);
        }
        if (cfg.stamps) {
            // diagnostic build only: wait for the lanes' work, then stamp
            const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
            cyc_form += ts0 - t_mark;
            cyc_proc += ts1 - ts0;
        }
        __syncthreads();  // every lane has read its entry before the ring changes
        // ---- retire consumed entries (0-count entries retire too)
        const bool full = ((uint32_t)lane < size) && S <= take;
        const uint32_t nfull = __popcll(__ballot(full));
        // the entry just below the fully consumed ones may be partially consumed
        if ((uint32_t)lane == nfull && (uint32_t)lane < size && excl < take)
            st.e[eidx][W - 1] = start + (uint32_t)(take - excl);
        top -= nfull;
        // ---- push outputs
        const int P = wave_scan_add(nout);
        const int tout = lane63(P);
        if ((top - bot) + (uint32_t)tout > (uint32_t)CAP) {
            if (lane == 0) dev_error(&g->err, kErrStackOverflow);
            break;
        }
        {
            uint32_t p = top + (uint32_t)(P - nout);
            for (int o = 0; o < nout; ++o, ++p)
#pragma unroll
                for (int w = 0; w < W; ++w) st.e[p & (CAP - 1)][w] = out[o][w];
        }
        top += (uint32_t)tout;
        __syncthreads();
        // ---- give the oldest entries to hungry waves, or relieve a full ring
        uint32_t sz = top - bot;
        uint32_t hungry = cfg.nwaves > outst ? cfg.nwaves - outst : 0;
        if (sz > cfg.spill_hi || (hungry > 0 && sz >= cfg.spill_lo)) {
            const unsigned long long ts = __builtin_amdgcn_s_memtime();
            while (sz > cfg.spill_hi || (hungry > 0 && sz >= cfg.spill_lo)) {
                uint32_t n = (sz + 1) / 2;
                if (n > pool.chunk) n = pool.chunk;
                if (n == 0 || n == sz) break;
                // home deque first, then the other deques of this XCD slice
                bool ok = false;
                for (uint32_t a = 0; a < qpx && !ok; ++a) {
                    const uint32_t q = xcc * qpx + (home - xcc * qpx + a) % qpx;
                    ok = enqueue_chunk<Kind, CAP>(pool, g, q, st, bot, n);
                }
                if (!ok) {
                    if (sz > (uint32_t)(CAP - kWaveSize * MO)) {
                        if (lane == 0) dev_error(&g->err, kErrQueueFull);
                    }
                    break;
                }
                ++npush;
                bot += n;
                sz = top - bot;
                if (hungry) --hungry;
            }
            cyc_spill += __builtin_amdgcn_s_memtime() - ts;
        }
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        cyc_busy += now - t_mark;
        t_mark = now;
    }
    cyc_idle += __builtin_amdgcn_s_memtime() - t_mark;
    if (active && lane == 0) {
        // only reached on an error break: keep the protocol consistent
        __hip_atomic_fetch_add(&g->outstanding, (uint32_t)-1, __ATOMIC_RELEASE, HX_AGENT);
    }
    acc.flush(g);
    if (lane == 0) {
        add_agent(&g->counters[kCtrBusyCycles], cyc_busy);
        if (cfg.stamps) {
            add_agent(&g->counters[kCtrFormCycles], cyc_form);
            add_agent(&g->counters[kCtrProcCycles], cyc_proc);
        }
        add_agent(&g->counters[kCtrIdleCycles], cyc_idle);
        add_agent(&g->counters[kCtrSpillCycles], cyc_spill);
        add_agent(&g->counters[kCtrWaves], 1ull);
        add_agent(&g->counters[kCtrBatches], nbatch);
        add_agent(&g->counters[kCtrPushed], npush);
        add_agent(&g->counters[kCtrStolen], nsteal);
    }
}

}  // namespace hx
