// hx_dyn.h — dynamic device dataflow: device tasks create promises and
// async_await tasks during a launch.
//
// The reference's promise machinery as running tasks use it:
//   hclib_promise_create          src/hclib-promise.c:55-83
//   hclib_promise_put             src/hclib-promise.c:203-245 (mark satisfied,
//                                 walk the waiter list, release each waiter)
//   spawn_await / async_await     src/hclib-runtime.c:596-644,
//                                 inc/hclib-async.h:248-290
//   register_on_all_promise_dependencies / _register_if_promise_not_ready
//                                 src/hclib-promise.c:132-195 (a task parks on
//                                 an unsatisfied future's waiter list)
// hx_dag.h runs a DAG the host fixed before the launch; here the graph grows
// on the device. A promise is {datum, head}: head is kDynOpen (not put, no
// waiters), a wait node (not put, waiters listed) or kDynPut (put: the list
// is closed). A new task's dependency counter starts at its futures + 1 (a
// guard); for each future a wait node is pushed onto the promise's list with
// one compare-and-swap unless the promise is already put (then that future
// counts as satisfied), and dropping the guard releases the task if nothing
// is pending. A put publishes the datum, swaps the head for kDynPut (a second
// put finds kDynPut: the reference's single-assignment HASSERT, here a device
// error) and walks the list it took, decrementing each waiter. A released
// task enters a ticket-ordered ready list; persistent waves take tickets.
// Termination: `live` counts tasks created and not yet finished (a task
// finishes after its own creations and puts), so a wave whose ticket is
// still empty leaves when live reaches 0; tasks parked on promises nobody
// puts keep live above 0 and end in the bounded-spin timeout, the
// reference's end_finish deadlock.
//
// Memory protocol (hx_common.h; MI355X_MICROARCH.md "Valid forms"): payload
// words, wait nodes and data are stored with agent-scope (sc1, write-through)
// stores and drained before the atomic that publishes them; readers use
// agent-scope loads. dyn_put<false> also releases at agent scope (a fence),
// for tasks that wrote their outputs with plain stores; run_dyn_worker
// acquires before a body unless Kind::kSc1Payload.
#pragma once

#include "hx_common.h"

namespace hx {

constexpr uint32_t kDynOpen = 0xffffffffu;  // promise head: not put, no waiters
constexpr uint32_t kDynPut = 0xfffffffeu;   // promise head: put
constexpr uint32_t kDynEmpty = 0xffffffffu; // ready-list slot not filled yet
constexpr int kDynMaxFutures = 8;           // futures per dyn_async_await (the reference's MAX_NUM_WAITS is 4;
                                            // more go through a task that awaits the rest)
constexpr int kDynMaxPayload = 16;          // payload words per task

enum : uint32_t { kErrDynDoublePut = 7, kErrDynPool = 8 };

// Device view of one dynamic launch (hclib_hip_dyn_launch_t).
struct DynView {
    unsigned long long *datum;  // [pcap]
    uint32_t *phead;            // [pcap] kDynOpen / kDynPut / first wait node
    uint32_t *wtask, *wnext;    // [wcap] wait nodes: the waiting task, the next node
    uint32_t *tdeps;            // [tcap] pending futures (+1 while the creator registers)
    uint32_t *tpay;             // [tcap * payload_words]
    uint32_t *ready;            // [rcap] ticket-ordered ready list
    uint32_t *ctl;              // [0] head, [64] tail, [128] live, [192] err, [256] next task,
                                // [320] next promise, [384] next wait node (one 256-B line each)
    unsigned long long *stats;  // [0] tasks run [1] puts [2] tasks created [3] releases [4] promises
    uint32_t tcap, pcap, wcap, rcap, payload_words, spin_ms;
};

struct DynWave {
    DynView v;
    unsigned long long ran, puts, created, releases, promises;
};

__device__ __forceinline__ uint32_t *dyn_head(const DynView &v) { return v.ctl; }
__device__ __forceinline__ uint32_t *dyn_tail(const DynView &v) { return v.ctl + 64; }
__device__ __forceinline__ uint32_t *dyn_live(const DynView &v) { return v.ctl + 128; }
__device__ __forceinline__ uint32_t *dyn_err(const DynView &v) { return v.ctl + 192; }

// lane-level: append task t to the ready list
__device__ __forceinline__ void dyn_enqueue(const DynView &v, uint32_t t) {
    const uint32_t pos = add_agent(dyn_tail(v), 1u);
    if (pos >= v.rcap) {
        dev_error(dyn_err(v), kErrDynPool);
        return;
    }
    st_agent(&v.ready[pos], t);
}

// hclib_promise_create, n at once (wave-uniform): the first id of n new
// promises, not put; kDynOpen when the pool is exhausted (device error set).
__device__ __forceinline__ uint32_t dyn_promises(DynWave &w, uint32_t n) {
    uint32_t base = 0;
    if (lane_id() == 0) base = add_agent(w.v.ctl + 320, n);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
    if ((unsigned long long)base + n > w.v.pcap) {
        if (lane_id() == 0) dev_error(dyn_err(w.v), kErrDynPool);
        return kDynOpen;
    }
    w.promises += n;
    return base;
}

// hclib_future_get on the device (the future of promise p; p put).
__device__ __forceinline__ unsigned long long dyn_get(const DynWave &w, uint32_t p) {
    return ld_agent(&w.v.datum[p]);
}

// hclib_promise_put (wave-uniform: every lane passes the same p and datum).
// SC1: the putting task wrote what its waiters read with agent-scope stores,
// so draining them is the release (no fence).
template <bool SC1 = false>
__device__ __forceinline__ void dyn_put(DynWave &w, uint32_t p, unsigned long long datum) {
    const DynView &v = w.v;
    if (SC1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else release_agent();
    uint32_t rel = 0;
    if (lane_id() == 0) {
        if (p >= v.pcap) {
            dev_error(dyn_err(v), kErrBadTask);
        } else {
            st_agent(&v.datum[p], datum);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the datum lands before any release
            uint32_t n = __hip_atomic_exchange(&v.phead[p], kDynPut, __ATOMIC_RELAXED, HX_AGENT);
            if (n == kDynPut) {  // src/hclib-promise.c:206-207
                dev_error(dyn_err(v), kErrDynDoublePut);
            } else {
                // the waiters that registered before the swap (src/hclib-promise.c:218-240)
                while (n != kDynOpen) {
                    const uint32_t t = ld_agent(&v.wtask[n]), nx = ld_agent(&v.wnext[n]);
                    if (add_agent(&v.tdeps[t], (uint32_t)-1) == 1u) {
                        dyn_enqueue(v, t);
                        ++rel;
                    }
                    n = nx;
                }
            }
        }
    }
    w.puts += 1;
    w.releases += (uint32_t)__builtin_amdgcn_readfirstlane((int)rel);
}

// async_await / spawn_await, one task per active lane: payload words
// pay[0 .. payload_words) and futures futs[0 .. nfut) (nfut <= kDynMaxFutures;
// kDynOpen entries are skipped, as NULL futures are). Returns the lane's new
// task id (kDynEmpty for inactive lanes or on pool exhaustion).
template <bool SC1 = false>
__device__ __forceinline__ uint32_t dyn_async_await(DynWave &w, bool active, const uint32_t *pay,
                                                    const uint32_t *futs, int nfut) {
    const DynView &v = w.v;
    const unsigned long long m = __ballot(active);
    if (!m) return kDynEmpty;
    if (!SC1) release_agent();  // what the creator wrote is visible to the new task
    const int lane = lane_id();
    const int leader = __builtin_ctzll(m);
    const uint32_t count = (uint32_t)__popcll(m);
    uint32_t base = 0;
    if (lane == leader) {
        base = add_agent(v.ctl + 256, count);
        add_agent(dyn_live(v), count);  // live before anything can release them
    }
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const uint32_t t = base + rank;
    const bool ok = active && t < v.tcap && nfut >= 0 && nfut <= kDynMaxFutures;
    if (active && !ok) dev_error(dyn_err(v), t < v.tcap ? kErrBadTask : kErrDynPool);
    uint32_t nodes = 0;
    if (ok) {
        // (bounded unrolled loops keep the caller's small arrays in registers)
#pragma unroll
        for (int k = 0; k < kDynMaxPayload; ++k)
            if (k < (int)v.payload_words) st_agent(&v.tpay[(size_t)t * v.payload_words + k], pay[k]);
        uint32_t nf = 0;
#pragma unroll
        for (int k = 0; k < kDynMaxFutures; ++k) nf += (k < nfut && futs[k] != kDynOpen) ? 1u : 0u;
        st_agent(&v.tdeps[t], nf + 1u);
        if (nf) {
            nodes = add_agent(v.ctl + 384, nf);
            if (nodes + nf > v.wcap) {
                dev_error(dyn_err(v), kErrDynPool);
                nf = 0;
            }
            uint32_t q = 0;
#pragma unroll
            for (int k = 0; k < kDynMaxFutures; ++k)
                if (k < nfut && futs[k] != kDynOpen && q < nf) st_agent(&v.wtask[nodes + q++], t);
        }
        nodes = nf ? nodes : kDynOpen;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // payload, counter, nodes land first
    if (ok) {
        // register on every future not yet put (src/hclib-promise.c:132-195)
        uint32_t sat = 0, q = 0;
#pragma unroll
        for (int k = 0; k < kDynMaxFutures; ++k) {
            if (k >= nfut) continue;
            const uint32_t p = futs[k];
            if (p == kDynOpen) continue;
            if (nodes == kDynOpen) {  // no node (pool exhausted): counted satisfied, error already set
                ++sat;
                continue;
            }
            const uint32_t n = nodes + q++;
            uint32_t h = ld_agent(&v.phead[p]);
            while (true) {
                if (h == kDynPut) {  // already put: nothing to wait for
                    ++sat;
                    break;
                }
                st_agent(&v.wnext[n], h);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the link lands before the node is visible
                // on failure h becomes the head seen, and the loop retries
                if (__hip_atomic_compare_exchange_strong(&v.phead[p], &h, n, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         HX_AGENT))
                    break;
            }
        }
        // drop the guard and the futures already satisfied
        if (add_agent(&v.tdeps[t], (uint32_t)-(int)(sat + 1u)) == sat + 1u) dyn_enqueue(v, t);
    }
    w.created += count;
    return ok ? t : kDynEmpty;
}

// Kind concept:
//   struct Ctx;
//   static constexpr bool kSc1Payload;  // bodies read other tasks' outputs only with agent-scope loads
//   __device__ static void run(const Ctx&, DynWave&, uint32_t task, const uint32_t *payload);
//        a wave-wide body; dyn_promises / dyn_put / dyn_get / dyn_async_await
//        are wave-uniform calls (async_await one task per active lane).
template <class Kind>
__device__ void run_dyn_worker(const typename Kind::Ctx &ctx, const DynView &view) {
    DynWave w{view, 0, 0, 0, 0, 0};
    const int lane = lane_id();
    while (true) {
        uint32_t ticket = 0;
        if (lane == 0) ticket = add_agent(dyn_head(view), 1u);
        ticket = (uint32_t)__builtin_amdgcn_readfirstlane((int)ticket);
        if (ticket >= view.rcap) break;
        uint32_t t = kDynEmpty;
        bool done = false;
        if (lane == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while ((t = ld_agent(&view.ready[ticket])) == kDynEmpty) {
                // the slot first, then live: a task enqueued here is live
                // until this wave runs it, so live == 0 means it never comes
                if (ld_agent(dyn_live(view)) == 0u || ld_agent(dyn_err(view))) {
                    done = true;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * view.spin_ms) {
                    dev_error(dyn_err(view), kErrSpinTimeout);
                    done = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
        done = __builtin_amdgcn_readfirstlane((int)done) != 0;
        if (done) break;
        if (t >= view.tcap) {
            if (lane == 0) dev_error(dyn_err(view), kErrBadTask);
            break;
        }
        if (!Kind::kSc1Payload) acquire_agent();
        // the payload was written by another wave during this launch: read it
        // with agent-scope loads (a plain load could hit a line this CU's L1
        // or the L2 cached before the words were written, e.g. while reading
        // a neighbouring task's payload)
        uint32_t pay[kDynMaxPayload];
#pragma unroll
        for (int k = 0; k < kDynMaxPayload; ++k)
            pay[k] = k < (int)view.payload_words ? ld_agent(&view.tpay[(size_t)t * view.payload_words + k]) : 0u;
        Kind::run(ctx, w, t, pay);
        ++w.ran;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // its creations and puts are out
        if (lane == 0) add_agent(dyn_live(view), (uint32_t)-1);
    }
    if (lane == 0) {
        add_agent(&view.stats[0], w.ran);
        add_agent(&view.stats[1], w.puts);
        add_agent(&view.stats[2], w.created);
        add_agent(&view.stats[3], w.releases);
        add_agent(&view.stats[4], w.promises);
    }
}

}  // namespace hx
