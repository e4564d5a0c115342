// hx_dag.h — device promises, futures and dependency-counter task release.
//
// Replaces the reference's promise machinery for device tasks:
//   hclib_promise_put            src/hclib-promise.c:203-245 (walk the waiter
//                                list, re-register or schedule each waiter)
//   register_on_all_promise_dependencies / _register_if_promise_not_ready
//                                src/hclib-promise.c:132-195 (a task parks on
//                                its first unsatisfied future)
//   spawn_await / async_await    src/hclib-runtime.c:596-644,
//                                inc/hclib-async.h:247-355
// with one counter per task instead of a parking chain: the host sizes each
// task's counter to the number of its futures whose promises are not yet
// satisfied and builds, per promise, the list of tasks awaiting it (a CSR).
// A device put publishes the datum, marks the promise satisfied (a second put
// is the reference's "single assignment" HASSERT, here a device error), and
// decrements every waiter's counter — lanes in parallel; the decrement that
// reaches zero appends the waiter to a ticket-ordered ready list. Persistent
// waves take tickets in order (one agent atomic each) and run the task
// (Kind::run, a wave-wide body). The DAG is acyclic and every ticket below
// the task count is eventually filled, so waits end; a task whose promise
// nobody puts is reported as a bounded-spin timeout, the reference's
// end_finish deadlock.
//
// Memory protocol (hx_common.h, MI355X_MICROARCH.md "Valid forms"): a put
// releases at agent scope first (the body's plain stores become visible),
// stores the datum write-through and drains it before any decrement; a wave
// acquires at agent scope before running a task it took from the list.
#pragma once

#include <type_traits>

#include "hx_common.h"

namespace hx {

constexpr uint32_t kDagEmpty = 0xffffffffu;
constexpr uint32_t kDagSkip = 0xfffffffeu;  // a ready-list slot whose task its releaser ran

enum : uint32_t { kErrDoublePut = 7 };

// Device view of one DAG launch (hclib_hip_dag_launch_t, include/hclib_hip.h).
struct DagView {
    uint32_t *deps;              // [ntasks] unsatisfied futures per task
    const uint32_t *waiter_off;  // [npromises + 1] CSR offsets
    const uint32_t *waiters;     // tasks awaiting each promise (a task once per await)
    unsigned long long *datum;   // [npromises]
    uint32_t *satisfied;         // [npromises]
    const uint32_t *payload;     // [ntasks * payload_words]
    uint32_t *ready;             // [ntasks] ticket-ordered ready list
    uint32_t *head;              // next ticket
    uint32_t *tail;              // next free ready slot
    uint32_t *err;               // DevError
    unsigned long long *stats;   // [0] tasks run, [1] puts, [2] releases
    uint32_t ntasks, npromises, payload_words, spin_ms;
    uint32_t nslots;             // ready slots with reserved puts: initially ready + every waiter entry
    // diagnostic builds (HX_STAMPS, HX_TRACE) with HCLIB_HIP_DAG_TRACE set: per task
    // kDagTraceWords 100 MHz stamps (see run_dag_group); null otherwise
    unsigned long long *trace;
};
// trace record of task t: [0] released (its last counter decrement
// returned), [1] started (the workgroup has its id), [2] body done (every
// wave drained), [3] puts done, [4] 1 if its releaser kept it, [5] the
// workgroup, [6] the task that released it; [8..15] the Kind's own stamps
constexpr int kDagTraceWords = 16;
// the per-task trace is compiled into the stamps build and into the lighter
// trace build (HX_TRACE: these stamps only, none of the per-phase ones)
#if (defined(HX_STAMPS) && HX_STAMPS) || (defined(HX_TRACE) && HX_TRACE)
#define HX_DAG_TRACE 1
#else
#define HX_DAG_TRACE 0
#endif

// Per-wave state a task body receives: the view and the wave's counters.
struct DagWave {
    DagView v;
    unsigned long long puts, releases;
    uint32_t next;      // a task this wave's puts released and kept for itself
    uint32_t skip_pos;  // (lane skip_lane) the ready-list slot that task gave up
    int skip_lane;
};

// hclib_future_get on the device: the datum of a satisfied promise (one the
// running task awaited, or one put before the launch).
__device__ __forceinline__ unsigned long long dag_get(const DagWave &w, uint32_t p) {
    return ld_agent(&w.v.datum[p]);
}

__device__ __forceinline__ bool dag_is_satisfied(const DagWave &w, uint32_t p) {
    return ld_agent(&w.v.satisfied[p]) != 0;
}

// One promise of a put: publish the datum, mark it satisfied and release its
// waiters. The datum store, the satisfied exchange and the waiter-range loads
// are in flight together (one memory round trip before the decrements); a
// second put on a satisfied promise is reported as kErrDoublePut (its stray
// decrements only move counters already at zero, which never release).
__device__ __forceinline__ void dag_put_one(DagWave &w, uint32_t p, unsigned long long datum) {
    const DagView &v = w.v;
    const int lane = lane_id();
    const uint32_t b = v.waiter_off[p], e = v.waiter_off[p + 1];
    uint32_t was = 0;
    if (lane == 0) {
        st_agent(&v.datum[p], datum);
        was = __hip_atomic_exchange(&v.satisfied[p], 1u, __ATOMIC_RELAXED, HX_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the datum lands before any release
    was = (uint32_t)__shfl((int)was, 0, 64);
    if (was) {  // src/hclib-promise.c:206-207
        if (lane == 0) dev_error(v.err, kErrDoublePut);
        return;
    }
    uint32_t rel = 0;
    for (uint32_t k0 = b; k0 < e; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        uint32_t t = kDagEmpty;
        if (k < e) {
            const uint32_t c = v.waiters[k];
            if (add_agent(&v.deps[c], (uint32_t)-1) == 1u) t = c;
        }
        // the putter keeps one released task and runs it next, as the
        // reference's put pushes waiters onto the putting worker's own deque
        // and that worker pops it first (src/hclib-promise.c:224-240,
        // src/hclib-runtime.c:488-530); the others go to the ready list
        const unsigned long long m = __ballot(t != kDagEmpty);
        if (m && w.next == kDagEmpty) {
            const int leader = __builtin_ctzll(m);
            w.next = (uint32_t)__builtin_amdgcn_readlane((int)t, leader);
            w.skip_lane = leader;
            if (lane == leader) {
                // the task still owns one ready-list slot (the ticket count
                // stays exact); it is marked skipped once the kept task runs,
                // so this atomic's latency hides behind that task
                w.skip_pos = add_agent(v.tail, 1u);
                t = kDagEmpty;
                ++rel;
            }
        }
        if (t != kDagEmpty) {
            const uint32_t pos = add_agent(v.tail, 1u);
            st_agent(&v.ready[pos], t);
            ++rel;
        }
    }
    w.puts += 1;
    w.releases += (unsigned long long)wave_sum((int)rel);
}

// hclib_promise_put on the device. Wave-uniform: every lane calls it with the
// same (p, datum); lanes share the waiter decrements. The release makes the
// task's plain stores visible at agent scope before any waiter can run.
__device__ __forceinline__ void dag_put(DagWave &w, uint32_t p, unsigned long long datum) {
    release_agent();
    dag_put_one(w, p, datum);
}

// Several puts of one task behind a single release (a tile that satisfies
// its right-column, bottom-row and corner promises at once), in three
// memory round trips whatever N is: lane i < N publishes promise i (datum,
// satisfied exchange, waiter range), then the lanes decrement the waiters of
// all N promises together (each lane one waiter of the concatenated lists),
// then the released tasks take ready-list slots (one kept, as dag_put_one).
// Waiter lists longer than 64 in total fall back to one put at a time.
// SC1 = true: the task wrote everything its waiters read with agent-scope
// (sc1, write-through) stores, so draining them (vmcnt) is the release and
// the L2 write-back of a release fence is skipped (MI355X_MICROARCH.md, Valid
// forms: sc1 payload + drained counter, consumers read with sc1 loads).
template <int N, bool SC1 = false>
__device__ __forceinline__ void dag_put_n(DagWave &w, const uint32_t (&p)[N], const unsigned long long (&datum)[N]) {
    static_assert(N >= 1 && N <= 64, "dag_put_n: 1..64 promises");
    if (SC1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else release_agent();
    const DagView &v = w.v;
    const int lane = lane_id();
    uint32_t my_p = 0, b = 0, e = 0, was = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (lane == i) my_p = p[i];
    if (lane < N) {
        unsigned long long d = 0;
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (lane == i) d = datum[i];
        st_agent(&v.datum[my_p], d);
        was = __hip_atomic_exchange(&v.satisfied[my_p], 1u, __ATOMIC_RELAXED, HX_AGENT);
        b = v.waiter_off[my_p];
        e = v.waiter_off[my_p + 1];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the data land before any release
    if (__ballot(lane < N && was != 0)) {  // src/hclib-promise.c:206-207
        if (lane == 0) dev_error(v.err, kErrDoublePut);
        return;
    }
    // concatenated waiter lists: promise i's waiters at [pre_i, pre_i + n_i)
    // (wave-uniform copies, read before any divergent branch)
    uint32_t ub[N], un[N], upre[N], total = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        ub[i] = (uint32_t)__builtin_amdgcn_readlane((int)b, i);
        un[i] = (uint32_t)__builtin_amdgcn_readlane((int)e, i) - ub[i];
        upre[i] = total;
        total += un[i];
    }
    if (total > 64) {  // long lists: promise by promise (already published)
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const uint32_t bi = ub[i], ei = ub[i] + un[i];
            uint32_t rel = 0;
            for (uint32_t k0 = bi; k0 < ei; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)lane;
                if (k < ei) {
                    const uint32_t c = v.waiters[k];
                    if (add_agent(&v.deps[c], (uint32_t)-1) == 1u) {
                        st_agent(&v.ready[add_agent(v.tail, 1u)], c);
                        ++rel;
                    }
                }
            }
            w.puts += 1;
            w.releases += (unsigned long long)wave_sum((int)rel);
        }
        return;
    }
    // lane k: waiter k of the concatenation
    uint32_t idx = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
        if ((uint32_t)lane >= upre[i] && (uint32_t)lane < upre[i] + un[i]) idx = ub[i] + ((uint32_t)lane - upre[i]);
    uint32_t t = kDagEmpty;
    if ((uint32_t)lane < total) {
        const uint32_t c = v.waiters[idx];
        if (add_agent(&v.deps[c], (uint32_t)-1) == 1u) t = c;
    }
    uint32_t rel = 0;
    const unsigned long long m = __ballot(t != kDagEmpty);
    if (m && w.next == kDagEmpty) {  // keep one released task (see dag_put_one)
        const int leader = __builtin_ctzll(m);
        w.next = (uint32_t)__builtin_amdgcn_readlane((int)t, leader);
        w.skip_lane = leader;
        if (lane == leader) {
            w.skip_pos = add_agent(v.tail, 1u);
            t = kDagEmpty;
            ++rel;
        }
    }
    if (t != kDagEmpty) {
        st_agent(&v.ready[add_agent(v.tail, 1u)], t);
        ++rel;
    }
    w.puts += N;
    w.releases += (unsigned long long)wave_sum((int)rel);
}

// Kind concept:
//   struct Ctx;   // per-launch parameters (passed by value)
//   __device__ static void run(const Ctx&, DagWave&, uint32_t task,
//                              const uint32_t *payload);
//        a wave-wide body: every lane enters; dag_get reads the futures it
//        awaited, dag_put satisfies promises (wave-uniform calls).
//
// A wave runs the task its own puts kept (w.next) before taking a ticket;
// that task's ready-list slot is then marked kDagSkip, and the wave whose
// ticket lands on it takes another ticket. Every slot below ntasks is thus
// filled exactly once, and a wave leaves on a ticket >= ntasks.
template <class Kind>
__device__ void run_dag_worker(const typename Kind::Ctx &ctx, const DagView &view) {
    DagWave w{view, 0, 0, kDagEmpty, 0, 0};
    const int lane = lane_id();
    unsigned long long ran = 0;
    while (true) {
        uint32_t t = kDagEmpty;
        bool kept = false;
        uint32_t pend_pos = 0;
        int pend_lane = 0;
        if (w.next != kDagEmpty) {
            t = w.next;
            w.next = kDagEmpty;
            kept = true;
            pend_pos = w.skip_pos;
            pend_lane = w.skip_lane;
        } else {
            uint32_t ticket = 0;
            if (lane == 0) ticket = add_agent(view.head, 1u);
            ticket = (uint32_t)__shfl((int)ticket, 0, 64);
            if (ticket >= view.ntasks) break;
            if (lane == 0) {
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while ((t = ld_agent(&view.ready[ticket])) == kDagEmpty) {
                    if (ld_agent(view.err)) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * view.spin_ms) {
                        dev_error(view.err, kErrSpinTimeout);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            t = (uint32_t)__shfl((int)t, 0, 64);
            if (t == kDagSkip) continue;
            if (t == kDagEmpty) break;
        }
        if (t >= view.ntasks) {
            if (lane == 0) dev_error(view.err, kErrBadTask);
            break;
        }
        acquire_agent();
        Kind::run(ctx, w, t, view.payload + (size_t)t * view.payload_words);
        ++ran;
        if (kept && lane == pend_lane) st_agent(&view.ready[pend_pos], kDagSkip);
    }
    if (lane == 0) {
        add_agent(&view.stats[0], ran);
        add_agent(&view.stats[1], w.puts);
        add_agent(&view.stats[2], w.releases);
    }
}

// Workgroup tasks: Kind::run_group(ctx, t, payload, wave) is a body every
// wave of the workgroup enters (returns false after a device error); wave 0
// takes the tickets, as run_dag_worker does, and after the body — every
// wave's stores drained, then a barrier — runs Kind::put(ctx, DagWave&, t),
// the task's puts. `slot` is one LDS word for the task id broadcast.
// Concept additions: run_group and put as above, and kSc1Payload: true when
// the bodies read what other tasks wrote only with agent-scope (sc1) loads,
// so no acquire fence (an L2 invalidate) is needed before a body.
// A Kind of run_dag_group may declare its puts up front —
//   static constexpr int kPutN;  // promises every task puts, 1..64
//   static void promises(const Ctx&, uint32_t task, uint32_t (&p)[kPutN]);
//   static void datums(const Ctx&, uint32_t task, unsigned long long (&d)[kPutN]);
// — in place of put(): the put is then split around the task (see below).
template <class K, class = void>
struct group_put_n { static constexpr int value = 0; };
template <class K>
struct group_put_n<K, decltype((void)K::kPutN)> { static constexpr int value = K::kPutN; };

// Optional: static constexpr bool kTagged = true — the Kind's bodies publish
// their outputs as tagged words and their readers poll the tags, so a put
// need not wait for the outputs' stores to drain before it releases the
// waiters (run_dag_group skips that drain). Such a put counts `satisfied` up
// instead of exchanging it (no result to wait for): a double put leaves 2,
// which hclib_hip_dag_end reports after the launch. Its datums are published
// without a drain too: they are for the host (read after the launch), not
// for device readers of the promise.
template <class K, class = void>
struct group_tagged { static constexpr bool value = false; };
template <class K>
struct group_tagged<K, decltype((void)K::kTagged)> { static constexpr bool value = K::kTagged; };

// Optional: static constexpr bool kReserve = true — every put takes one ready
// slot per waiter entry of its promises with one tail fetch-add issued beside
// its counter decrements, and fills them at once: a released task's id, or
// kDagSkip (kept, or not released). The put's other releases then reach the
// ready list one round trip sooner than through the helper's append at the
// next task; the list holds view.nslots entries (hclib_hip_dag_begin), and
// tickets run to that count. Waiter lists of more than 64 entries per task
// take the same reserved form 64 entries at a time (not prefetched). Only
// tagged Kinds may reserve (static_assert in run_dag_group).
template <class K, class = void>
struct group_reserve { static constexpr bool value = false; };
template <class K>
struct group_reserve<K, decltype((void)K::kReserve)> { static constexpr bool value = K::kReserve; };

// Optional: static void after_body(const Ctx&, uint32_t task), run by every
// thread once every wave has finished the task's body (before its put).
template <class K, class = void>
struct has_after_body : std::false_type {};
template <class K>
struct has_after_body<K, decltype((void)&K::after_body)> : std::true_type {};
template <class Kind>
__device__ __forceinline__ void group_after_body(const typename Kind::Ctx &ctx, uint32_t t) {
    if constexpr (has_after_body<Kind>::value) Kind::after_body(ctx, t);
}

// State the waves of one workgroup share across its tasks (LDS).
struct DagGroupShared {
    uint32_t slot;        // the task wave 0 found
    uint32_t nwait;       // waiters of the running task's promises (> 64: not prefetched)
    uint32_t npend;       // tasks the last put released for the ready list
    uint32_t skip;        // 1: the last put kept a task (its ready slot is a skip)
    uint32_t dbl;         // the running task put a promise twice
    uint32_t fail;        // a wave's body failed (device error): every wave leaves
    uint32_t waiter[64];  // their ids, concatenated in promise order
    uint32_t pend[64];
};

// The workgroup form of run_dag_worker: one task at a time, every wave of the
// workgroup in Kind::run_group (a band of the tile each, an ingress and an
// egress wave, ...). Wave 0 takes tickets and puts. With kPutN the put is
// split so that one memory round trip past the task's own drain stays on the
// chain from a task to its successor:
//   * while the task runs, the last wave loads the waiter lists of its
//     promises (static: the CSR the host built) into LDS;
//   * at its end the same wave stores the datums and marks the promises
//     satisfied behind the drain of its own outputs; after the task's barrier
//     wave 0 decrements the waiters' counters, keeps one released task and
//     leaves the others in LDS;
//   * the last wave appends those (and the kept task's skip) to the ready
//     list while the next task (the kept one) already runs.
template <class Kind>
__device__ void run_dag_group(const typename Kind::Ctx &ctx, const DagView &view, uint32_t *slot_unused) {
    (void)slot_unused;
    constexpr int N = group_put_n<Kind>::value;
    constexpr bool kTagged = group_tagged<Kind>::value;
    constexpr bool kReserve = group_reserve<Kind>::value;
    static_assert(!kReserve || N > 0, "reserved puts use the split put");
    // a reserved put counts `satisfied` up (no exchange to wait for), so its
    // double puts are found by hclib_hip_dag_end like a tagged Kind's: only
    // tagged Kinds may reserve
    static_assert(!kReserve || kTagged, "reserved puts need a tagged Kind");
    const uint32_t nslots = kReserve ? view.nslots : view.ntasks;
    static_assert(!kTagged || (N > 0 && Kind::kSc1Payload), "tagged puts use the split put of sc1 payloads");
    __shared__ DagGroupShared sh;
    DagWave w{view, 0, 0, kDagEmpty, 0, 0};
    const int lane = lane_id(), wave = (int)(threadIdx.x >> 6), nwaves = (int)(blockDim.x >> 6);
    const int helper = nwaves - 1;
    unsigned long long ran = 0;
    // diagnostic build (HX_STAMPS): wave 0's cycles taking tasks / running
    // bodies / putting, into stats[3..5]
    unsigned long long cyc[3] = {0, 0, 0}, tsx = 0;
    auto stamp = [&](int k) {
#if defined(HX_STAMPS) && HX_STAMPS
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (tsx) cyc[k] += now - tsx;
        tsx = now;
#else
        (void)k;
#endif
    };
    if (threadIdx.x == 0) {
        sh.npend = 0;
        sh.skip = 0;
        sh.fail = 0;
    }
    __syncthreads();
    stamp(0);
    while (true) {
        bool kept = false;
        uint32_t pend_pos = 0;
        int pend_lane = 0;
        if (wave == 0) {
            uint32_t t = kDagEmpty;
            while (true) {
                if (w.next != kDagEmpty) {
                    t = w.next;
                    w.next = kDagEmpty;
                    kept = true;
                    pend_pos = w.skip_pos;
                    pend_lane = w.skip_lane;
                    break;
                }
                uint32_t ticket = 0;
                if (lane == 0) ticket = add_agent(view.head, 1u);
                ticket = (uint32_t)__shfl((int)ticket, 0, 64);
                t = kDagEmpty;
                if (ticket >= nslots) break;
                if (lane == 0) {
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    while ((t = ld_agent(&view.ready[ticket])) == kDagEmpty) {
                        if (ld_agent(view.err)) break;
                        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * view.spin_ms) {
                            dev_error(view.err, kErrSpinTimeout);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                t = (uint32_t)__shfl((int)t, 0, 64);
                if (t != kDagSkip) break;
            }
            if (t != kDagEmpty && t >= view.ntasks) {
                if (lane == 0) dev_error(view.err, kErrBadTask);
                t = kDagEmpty;
            }
            if (lane == 0) sh.slot = t;
        }
        __syncthreads();
        const uint32_t t = sh.slot;
        __syncthreads();  // the slot is rewritten only after this barrier
        if (t == kDagEmpty) break;
        if (N > 0 && wave == helper) {
            // the previous put's releases: one tail fetch-add for all of them,
            // while the task runs (a put that released any task kept one, so
            // wave 0 never waits on the ready list for these: see kept)
            const uint32_t np = sh.npend, sk = sh.skip;
            if (np + sk) {
                uint32_t base = 0;
                if (lane == 0) base = add_agent(view.tail, np + sk);
                base = (uint32_t)__builtin_amdgcn_readfirstlane(base);
                if ((uint32_t)lane < np) st_agent(&view.ready[base + (uint32_t)lane], sh.pend[lane]);
                if (sk && lane == 0) st_agent(&view.ready[base + np], kDagSkip);
            }
        }
        if (!Kind::kSc1Payload) acquire_agent();
        stamp(0);
#if HX_DAG_TRACE
        if (view.trace && threadIdx.x == 0) {
            unsigned long long *r = view.trace + (size_t)t * kDagTraceWords;
            r[1] = __builtin_amdgcn_s_memrealtime();
            r[4] = kept ? 1ull : 0ull;
            r[5] = blockIdx.x;
        }
#endif
        if constexpr (N > 0) {
            if (wave == helper) {
                // prefetch the waiter lists of the task's promises (the CSR is
                // static); wave 0 reads them after the task's barrier
                uint32_t p[N];
                Kind::promises(ctx, t, p);
                uint32_t my_p = 0, b = 0, e = 0;
#pragma unroll
                for (int i = 0; i < N; ++i)
                    if (lane == i) my_p = p[i];
                if (lane < N) {
                    b = view.waiter_off[my_p];
                    e = view.waiter_off[my_p + 1];
                }
                uint32_t ub[N], un[N], upre[N], total = 0;
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    ub[i] = (uint32_t)__builtin_amdgcn_readlane((int)b, i);
                    un[i] = (uint32_t)__builtin_amdgcn_readlane((int)e, i) - ub[i];
                    upre[i] = total;
                    total += un[i];
                }
                if (total <= 64) {
                    uint32_t idx = 0;
#pragma unroll
                    for (int i = 0; i < N; ++i)
                        if ((uint32_t)lane >= upre[i] && (uint32_t)lane < upre[i] + un[i])
                            idx = ub[i] + ((uint32_t)lane - upre[i]);
                    if ((uint32_t)lane < total) sh.waiter[lane] = view.waiters[idx];
                }
                if (lane == 0) sh.nwait = total;
            }
        }
        const bool ok = Kind::run_group(ctx, t, view.payload + (size_t)t * view.payload_words, wave);
        uint32_t was = 0;
        if constexpr (N > 0) {
            // the helper (usually the wave storing the task's last outputs)
            // publishes the datums and marks the promises satisfied behind the
            // same drain as its outputs
            if (wave == helper && sh.nwait <= 64) {
                uint32_t p[N];
                unsigned long long d[N];
                Kind::promises(ctx, t, p);
                Kind::datums(ctx, t, d);
                uint32_t my_p = 0;
                unsigned long long my_d = 0;
#pragma unroll
                for (int i = 0; i < N; ++i)
                    if (lane == i) {
                        my_p = p[i];
                        my_d = d[i];
                    }
                if (lane < N) {
                    st_agent(&view.datum[my_p], my_d);
                    if constexpr (kTagged)  // no result to wait for: a second put leaves 2 (hclib_hip_dag_end)
                        __hip_atomic_fetch_add(&view.satisfied[my_p], 1u, __ATOMIC_RELAXED, HX_AGENT);
                    else
                        was = __hip_atomic_exchange(&view.satisfied[my_p], 1u, __ATOMIC_RELAXED, HX_AGENT);
                }
            }
        }
        // every wave's outputs are visible before wave 0 releases the waiters:
        // sc1 payloads need only the drain, plain stores the agent release
        // (another XCD's L2 must not serve stale lines)
        if constexpr (kTagged) {
            // no drain: the readers poll the outputs' tags; a double put is
            // found after the launch (a satisfied count of 2)
            if (wave == helper && lane == 0) sh.dbl = 0u;
        } else {
            if constexpr (Kind::kSc1Payload) vm_drain();
            else release_agent();
            if constexpr (N > 0) {
                if (wave == helper) {
                    const bool dbl = __ballot(lane < N && was != 0) != 0;  // src/hclib-promise.c:206-207
                    if (lane == 0) sh.dbl = dbl ? 1u : 0u;
                }
            }
        }
        // (an LDS flag and a plain barrier: __syncthreads_or reads the
        // workgroup size from memory and so waits for every store in flight)
        if (!ok) sh.fail = 1u;
        __syncthreads();
        if (sh.fail) break;
        // every wave is done with the task: the Kind's between-task work
        // (e.g. resetting its LDS hand-off flags so the next body needs no
        // barrier of its own)
        group_after_body<Kind>(ctx, t);
        stamp(1);
#if HX_DAG_TRACE
        if (view.trace && threadIdx.x == 0) view.trace[(size_t)t * kDagTraceWords + 2] = __builtin_amdgcn_s_memrealtime();
#endif
        if constexpr (N > 0) {
            if (wave == 0) {
                const uint32_t nwait = sh.nwait;
                if (nwait > 64) {
                    uint32_t p[N];
                    unsigned long long d[N];
                    Kind::promises(ctx, t, p);
                    Kind::datums(ctx, t, d);
                    if constexpr (kReserve) {
                        // long waiter lists (not prefetched, so the helper did not
                        // publish): the datums and satisfied counts here, then
                        // the reserved release 64 waiter entries at a time, all
                        // nwait slots taken with one tail fetch-add
                        uint32_t my_p = 0;
                        unsigned long long my_d = 0;
#pragma unroll
                        for (int i = 0; i < N; ++i)
                            if (lane == i) {
                                my_p = p[i];
                                my_d = d[i];
                            }
                        if (lane < N) {
                            st_agent(&view.datum[my_p], my_d);
                            __hip_atomic_fetch_add(&view.satisfied[my_p], 1u, __ATOMIC_RELAXED, HX_AGENT);
                        }
                        uint32_t base = 0;
                        if (lane == 0) base = add_agent(view.tail, nwait);
                        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                        // a put past the reserved slots (a promise put twice):
                        // no release, no ready write, a device error
                        const bool fits = base + nwait <= nslots;
                        if (!fits && lane == 0) dev_error(view.err, kErrDoublePut);
                        uint32_t off = 0, rel = 0;
#pragma unroll
                        for (int i = 0; i < N; ++i) {
                            const uint32_t bi = view.waiter_off[p[i]], ei = view.waiter_off[p[i] + 1];
                            for (uint32_t k0 = bi; fits && k0 < ei; k0 += 64) {
                                const uint32_t k = k0 + (uint32_t)lane;
                                uint32_t rt = kDagEmpty;
                                if (k < ei) {
                                    const uint32_t c = view.waiters[k];
                                    if (add_agent(&view.deps[c], (uint32_t)-1) == 1u) rt = c;
                                }
                                const unsigned long long m = __ballot(rt != kDagEmpty);
                                int kept_lane = -1;
                                if (m && w.next == kDagEmpty) {
                                    kept_lane = __builtin_ctzll(m);
                                    w.next = (uint32_t)__builtin_amdgcn_readlane((int)rt, kept_lane);
                                }
                                if (k < ei)
                                    st_agent(&view.ready[base + off + (k - bi)],
                                             (rt != kDagEmpty && lane != kept_lane) ? rt : kDagSkip);
                                rel += (uint32_t)__builtin_popcountll(m);
                            }
                            off += ei - bi;
                        }
                        w.puts += N;
                        w.releases += rel;
                    } else {
                        // long waiter lists: the ordinary batched put (it appends
                        // its releases itself)
                        dag_put_n<N, Kind::kSc1Payload>(w, p, d);
                        if (w.next != kDagEmpty && lane == w.skip_lane) st_agent(&view.ready[w.skip_pos], kDagSkip);
                    }
                    if (lane == 0) {
                        sh.npend = 0;
                        sh.skip = 0;
                    }
                } else if (kReserve) {
                    // one slot per waiter entry, taken beside the decrements
                    uint32_t base = 0, rt = kDagEmpty, c = 0;
                    if (lane == 0) base = add_agent(view.tail, nwait);
                    if ((uint32_t)lane < nwait) {
                        c = sh.waiter[lane];
                        if (add_agent(&view.deps[c], (uint32_t)-1) == 1u) rt = c;
#if HX_DAG_TRACE
                        if (view.trace && rt == c) {
                            view.trace[(size_t)c * kDagTraceWords + 0] = __builtin_amdgcn_s_memrealtime();
                            view.trace[(size_t)c * kDagTraceWords + 6] = t;
                        }
#endif
                    }
                    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                    // a put past the reserved slots (a promise put twice, which
                    // tagged puts otherwise report only after the launch): no
                    // ready write beyond the list, a device error at once
                    const bool fits = base + nwait <= nslots;
                    if (!fits && lane == 0) dev_error(view.err, kErrDoublePut);
                    const unsigned long long m = fits ? __ballot(rt != kDagEmpty) : 0ull;
                    int kept_lane = -1;
                    if (m) {  // keep the first released task (see dag_put_one)
                        kept_lane = __builtin_ctzll(m);
                        w.next = (uint32_t)__builtin_amdgcn_readlane((int)rt, kept_lane);
                    }
                    if (fits && (uint32_t)lane < nwait)
                        st_agent(&view.ready[base + (uint32_t)lane], (rt != kDagEmpty && lane != kept_lane) ? rt : kDagSkip);
                    if (lane == 0) {
                        sh.npend = 0;
                        sh.skip = 0;
                    }
                    w.puts += N;
                    w.releases += (unsigned long long)__builtin_popcountll(m);
                    w.skip_lane = 0;
                } else {
                    const bool dbl = sh.dbl != 0;
                    if (dbl && lane == 0) dev_error(view.err, kErrDoublePut);
                    uint32_t rt = kDagEmpty;
                    if (!dbl && (uint32_t)lane < nwait) {
                        const uint32_t c = sh.waiter[lane];
                        if (add_agent(&view.deps[c], (uint32_t)-1) == 1u) rt = c;
#if HX_DAG_TRACE
                        if (view.trace && rt == c) {
                            view.trace[(size_t)c * kDagTraceWords + 0] = __builtin_amdgcn_s_memrealtime();
                            view.trace[(size_t)c * kDagTraceWords + 6] = t;
                        }
#endif
                    }
                    unsigned long long m = __ballot(rt != kDagEmpty);
                    uint32_t skip = 0;
                    if (m) {  // keep the first released task (see dag_put_one)
                        const int leader = __builtin_ctzll(m);
                        w.next = (uint32_t)__builtin_amdgcn_readlane((int)rt, leader);
                        m &= m - 1;
                        skip = 1;
                    }
                    // the others, compacted, for the helper wave's append
                    if ((m >> lane) & 1ull) {
                        const uint32_t r = (uint32_t)__builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        sh.pend[r] = rt;
                    }
                    if (lane == 0) {
                        sh.npend = (uint32_t)__builtin_popcountll(m);
                        sh.skip = skip;
                    }
                    w.puts += N;
                    w.releases += (unsigned long long)(__builtin_popcountll(m) + skip);
                }
                // the kept task's ready slot is appended by the helper wave
                w.skip_lane = 0;
            }
            // (sh.pend / npend / skip reach the helper through the next
            // task's slot barrier)
        } else {
            if (wave == 0) {
                Kind::put(ctx, w, t);
                if (kept && lane == pend_lane) st_agent(&view.ready[pend_pos], kDagSkip);
            }
        }
        stamp(2);
#if HX_DAG_TRACE
        if (view.trace && threadIdx.x == 0) view.trace[(size_t)t * kDagTraceWords + 3] = __builtin_amdgcn_s_memrealtime();
#endif
        ++ran;
    }
    if (wave == 0 && lane == 0) {
        add_agent(&view.stats[0], ran);
        add_agent(&view.stats[1], w.puts);
        add_agent(&view.stats[2], w.releases);
#if defined(HX_STAMPS) && HX_STAMPS
        for (int k = 0; k < 3; ++k) add_agent(&view.stats[3 + k], cyc[k]);
#endif
    }
}

}  // namespace hx
