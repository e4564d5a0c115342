// hx_finish.h — nested finish scopes for device task kinds.
//
// The reference's finish (src/hclib-runtime.c:1219-1277, src/inc/
// hclib-finish.h:6-10) is a counter of live tasks plus a parent pointer;
// end_finish blocks the task that opened it (help-first, src/hclib-runtime.c:
// 1067-1119) and then the code after the finish runs. A GPU task has no
// stack to block on, so here the code after the finish is a CONTINUATION:
//
//   a task that opens a scope (finish { async ...; async ...; }) calls
//   finish_open with the number of tasks it spawns into the scope and a
//   continuation word of its own choosing; the spawned tasks carry the scope
//   id in their templates;
//
//   a task that completes calls finish_check_out(scope, value, cont): ONE
//   agent-scope 64-bit atomic adds its value and checks out (word =
//   count << 56 | 56-bit sum); the task that brings the count to zero runs
//   the continuation inline — cont(cont_word, sum) returns the value the
//   scope hands to ITS parent — and checks out of the parent the same way
//   (the work-shift of help_finish: whoever finishes last runs what follows).
//   At the outermost scope the value is stored to the arena's root word.
//
// Scopes are bump-allocated, one agent atomic per wave for all lanes that
// open one in a batch. Counts are at most 255 spawned tasks per scope.
#pragma once

#include "hx_common.h"

namespace hx {

constexpr uint32_t kScopeRoot = 0xffffffffu;
constexpr unsigned long long kScopeOne = 1ull << 56;
constexpr unsigned long long kScopeSumMask = kScopeOne - 1;

struct alignas(16) FinishScope {
    unsigned long long word;  // live tasks << 56 | sum of their values (mod 2^56)
    uint32_t parent;          // enclosing scope, or kScopeRoot
    uint32_t cont;            // the opener's continuation word
};

struct FinishArena {
    FinishScope *scopes;
    uint32_t *next;                 // bump allocator
    uint32_t cap;
    unsigned long long *root_value;  // the outermost scope's value lands here
};

// Lanes with `open` set each open a scope of `count` (1..255) tasks under
// `parent`; returns the lane's scope id (kScopeRoot for lanes that do not
// open one, or on arena exhaustion, which is reported through err).
// Called by the whole wave.
// `blk` (optional): two words of the calling wave's LDS, {next, end} of a
// block of scope ids the wave took from the arena (kScopeBlock at a time, one
// agent atomic per block instead of one per open), zeroed before its first
// open. Wave-uniform state in LDS, not in registers: a lane inactive at an
// update would keep a stale register copy (divergent batches).
constexpr uint32_t kScopeBlock = 256;
__device__ __forceinline__ uint32_t finish_open(const FinishArena &a, bool open, uint32_t parent, uint32_t count,
                                                uint32_t cont, uint32_t *err, uint32_t *blk = nullptr) {
    const unsigned long long m = __ballot(open);
    if (!m) return kScopeRoot;
    const int leader = __builtin_ctzll(m);
    const uint32_t k = (uint32_t)__popcll(m);
    const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    uint32_t s = 0;
    if (blk && k <= kScopeBlock) {
        // the rest of the current block first, then a new block (ids need not
        // be contiguous: only the last block of each wave leaves ids unused)
        const uint32_t nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)blk[0]),
                       end = (uint32_t)__builtin_amdgcn_readfirstlane((int)blk[1]);
        const uint32_t left = end - nxt;
        if (k <= left) {
            s = nxt + rank;
            if (lane_id() == leader) blk[0] = nxt + k;
        } else {
            uint32_t b = 0;
            if (lane_id() == leader) b = add_agent(a.next, kScopeBlock);
            b = (uint32_t)__builtin_amdgcn_readlane((int)b, leader);
            s = rank < left ? nxt + rank : b + (rank - left);
            if (lane_id() == leader) {
                blk[0] = b + (k - left);
                blk[1] = b + kScopeBlock;
            }
        }
        asm volatile("" ::: "memory");
    } else {
        uint32_t base = 0;
        if (lane_id() == leader) base = add_agent(a.next, k);
        s = (uint32_t)__builtin_amdgcn_readlane((int)base, leader) + rank;
    }
    if (!open) return kScopeRoot;
    if (s >= a.cap || count == 0 || count > 255) {
        dev_error(err, s >= a.cap ? kErrArena : kErrBadTask);
        return kScopeRoot;
    }
    FinishScope *f = &a.scopes[s];
    st_agent(&f->word, (unsigned long long)count << 56);
    st_agent(&f->parent, parent);
    st_agent(&f->cont, cont);
    return s;
}

// Check out of scope s with `value`; the last task out runs
// cont(cont_word, sum) -> value for the parent, and so on up. Returns the
// number of continuations this lane ran.
template <class Cont>
__device__ __forceinline__ uint32_t finish_check_out(const FinishArena &a, uint32_t s, unsigned long long value,
                                                     Cont &&cont) {
    uint32_t ran = 0;
    unsigned long long v = value & kScopeSumMask;
    while (s != kScopeRoot) {
        if (s >= a.cap) return ran;  // (never: an LDS or stale id here would be a protocol bug, not a fault)
        FinishScope *f = &a.scopes[s];
        // {parent, cont} never change after the open: loaded beside the
        // check-out (one round trip per chain step, not two)
        const unsigned long long pc = ld_agent((const unsigned long long *)&f->parent);
        unsigned long long old = add_agent(&f->word, v - kScopeOne), add = v;
        if ((old & kScopeSumMask) + v > kScopeSumMask) {
            // the sum carried into the count byte: take the carry back out with
            // a second check-out of value 0 (whoever brings the count to 1
            // last, this one or a sibling, is the last task out; the sum stays
            // mod 2^56 as documented)
            old = add_agent(&f->word, (unsigned long long)0 - kScopeOne);
            add = 0;
        }
        if ((old >> 56) != 1) return ran;  // a sibling is still running
        const unsigned long long sum = (old + add) & kScopeSumMask;
        v = cont((uint32_t)(pc >> 32), sum) & kScopeSumMask;
        ++ran;
        s = (uint32_t)pc;
    }
    st_agent(a.root_value, v);
    return ran;
}

// finish_check_out split in two, so that an HBM check-out's round trip
// overlaps other work: finish_issue starts the step on scope s (its atomic
// and the {parent, cont} load), finish_resolve — called a batch later —
// takes the result: not the last task out: done; the last: the continuation,
// and the parent's step is issued in turn (root: the value is stored). One
// step per lane in flight (q.s == kScopeRoot: none).
struct FinishInFlight {
    unsigned long long old = 0, pc = 0, v = 0;
    uint32_t s = kScopeRoot;
};

__device__ __forceinline__ void finish_issue(const FinishArena &a, FinishInFlight &q, uint32_t s,
                                             unsigned long long v) {
    if (s >= a.cap) return;  // (never; see finish_check_out)
    FinishScope *f = &a.scopes[s];
    q.s = s;
    q.v = v & kScopeSumMask;
    q.pc = ld_agent((const unsigned long long *)&f->parent);
    q.old = add_agent(&f->word, q.v - kScopeOne);
}

template <class Cont>
__device__ __forceinline__ uint32_t finish_resolve(const FinishArena &a, FinishInFlight &q, Cont &&cont) {
    if (q.s == kScopeRoot) return 0;
    unsigned long long old = q.old, add = q.v;
    if ((old & kScopeSumMask) + q.v > kScopeSumMask) {  // see finish_check_out (synchronous, rare)
        old = add_agent(&a.scopes[q.s].word, (unsigned long long)0 - kScopeOne);
        add = 0;
    }
    q.s = kScopeRoot;
    if ((old >> 56) != 1) return 0;
    const unsigned long long v = cont((uint32_t)(q.pc >> 32), (old + add) & kScopeSumMask) & kScopeSumMask;
    const uint32_t p = (uint32_t)q.pc;
    if (p == kScopeRoot) st_agent(a.root_value, v);
    else finish_issue(a, q, p, v);
    return 1;
}

// every step still in flight, to its end (before the wave goes idle)
template <class Cont>
__device__ __forceinline__ uint32_t finish_drain(const FinishArena &a, FinishInFlight &q, Cont &&cont) {
    uint32_t ran = 0;
    while (q.s != kScopeRoot) ran += finish_resolve(a, q, cont);
    return ran;
}

// ------------------------------------------------ wave-local scopes (LDS)
// Most scopes open and close inside one wave: its two (or k) tasks are pushed
// onto the wave's own ring and popped by it again (LIFO), usually in the
// same batch. Those scopes live in the wave's LDS (LocalScopes): open is a
// pop from an LDS free list, check-out an LDS atomic (~100 cycles instead of
// an agent-scope round trip of microseconds), the last task out frees the
// slot. A scope becomes visible to other waves only when one of its tasks
// leaves the wave (a spilled chunk, an inbox, the global ring): the Kind's
// export hook then PROMOTES it — and every LDS ancestor on its chain — to an
// HBM scope of the arena (finish_promote): the HBM copy takes the LDS word
// as it stands and the LDS slot forwards to it, so the owner's later
// check-outs of that scope go to HBM too. Forwarded slots are never reused
// (a ring item may still name them); when the free list runs dry, scopes
// are opened in HBM (their LDS parents promoted first: an HBM scope never
// names an LDS parent, since the wave that closes it may be another). Only
// the owning wave touches its
// LocalScopes, and one wave's LDS operations complete in issue order, so
// nothing but the check-out needs an atomic.
constexpr uint32_t kScopeLds = 0x40000000u;  // scope id bit: an LDS slot of the running wave

template <int N>
struct LocalScopes {
    unsigned long long word[N];  // live tasks << 56 | sum (as FinishScope::word)
    // {parent, cont, fwd, mark}: fwd = 0, or 1 + the HBM scope this slot was
    // promoted to; mark = the promotion round that last visited the slot.
    // One 16-byte LDS read per check-out step, issued beside its atomic
    hx_u32x4 meta[N];
    uint32_t freelist[N];
    uint32_t nfree;
    uint32_t epoch;  // promotion rounds (finish_promote)
    uint32_t cnt;    // finish_promote's slot count
    // every lane of the wave calls init once before the first open
    __device__ void init() {
        for (int i = lane_id(); i < N; i += 64) {
            freelist[i] = (uint32_t)(N - 1 - i);
            meta[i] = hx_u32x4{kScopeRoot, 0u, 0u, 0u};
        }
        if (lane_id() == 0) {
            nfree = N;
            epoch = 0;
        }
        asm volatile("" ::: "memory");
    }
};

__device__ __forceinline__ bool scope_is_lds(uint32_t s) { return s != kScopeRoot && (s & kScopeLds); }

// The scope a lane's exported item must name: its LDS scope promoted to HBM
// (with every unpromoted LDS ancestor), or `s` itself. All scopes one call
// promotes take ONE arena allocation: every lane marks the unpromoted slots
// on its chain (round `epoch`), the wave numbers the marked slots, takes that
// many HBM ids with one atomic, forwards each slot and writes its HBM copy
// (parents resolved through the forwards just set). Called by the whole wave.
template <int N>
__device__ __forceinline__ uint32_t finish_promote(const FinishArena &a, LocalScopes<N> &ls, uint32_t s,
                                                   uint32_t *err) {
    const int lane = lane_id();
    const int lead = __builtin_ctzll(__ballot(1));  // the first active lane does the scalar work
    constexpr uint32_t kMask = kScopeLds - 1;
    auto unpromoted = [&](uint32_t x) { return scope_is_lds(x) && ls.meta[x & kMask].z == 0; };
    auto resolve = [&](uint32_t x) { return scope_is_lds(x) ? ls.meta[x & kMask].z - 1 : x; };
    if (!__ballot(unpromoted(s))) return resolve(s);
    const uint32_t ep = (uint32_t)__builtin_amdgcn_readfirstlane((int)ls.epoch) + 1u;
    // 1. mark every unpromoted slot on every lane's chain
    for (uint32_t x = s; unpromoted(x);) {
        hx_u32x4 *m = &ls.meta[x & kMask];
        if (m->w == ep) break;  // another lane's walk got here first
        m->w = ep;
        x = m->x;
    }
    asm volatile("" ::: "memory");
    // 2. number the marked slots, one allocation. The active lanes (any
    // subset: export hooks run under divergent control flow) take slots
    // rank, rank + na, ...; each lane's range comes from an LDS counter
    const unsigned long long act = __ballot(1);
    const int na = __popcll(act);
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    if (lane == lead) ls.cnt = 0;
    asm volatile("" ::: "memory");
    uint32_t mine = 0;
    for (int i = rank; i < N; i += na) mine += (ls.meta[i].w == ep && ls.meta[i].z == 0) ? 1u : 0u;
    const uint32_t off = __hip_atomic_fetch_add(&ls.cnt, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)ls.cnt);
    uint32_t base = 0;
    if (lane == lead) base = add_agent(a.next, tot);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
    if (base + tot > a.cap) {
        // out of arena (reported; the launch fails): close this round so a
        // later promotion never takes its stale marks for its own
        if (lane == lead) {
            dev_error(err, kErrArena);
            ls.epoch = ep;
        }
        asm volatile("" ::: "memory");
        return kScopeRoot;
    }
    uint32_t h = base + off;
    for (int i = rank; i < N; i += na)
        if (ls.meta[i].w == ep && ls.meta[i].z == 0) ls.meta[i].z = 1u + h++;
    asm volatile("" ::: "memory");
    // 3. the HBM copies (every parent is now root, HBM or forwarded)
    for (int i = rank; i < N; i += na) {
        if (ls.meta[i].w == ep) {
            const hx_u32x4 m = ls.meta[i];
            FinishScope *f = &a.scopes[m.z - 1];
            st_agent(&f->word, ls.word[i]);
            st_agent(&f->parent, resolve(m.x));
            st_agent(&f->cont, m.y);
        }
    }
    if (lane == lead) ls.epoch = ep;
    asm volatile("" ::: "memory");
    return resolve(s);
}

// An open that prefers the wave's LDS: lanes with `open` each get an LDS
// scope while the free list lasts, the rest HBM scopes (finish_open).
template <int N>
__device__ __forceinline__ uint32_t finish_open_local(const FinishArena &a, LocalScopes<N> &ls, bool open,
                                                      uint32_t parent, uint32_t count, uint32_t cont, uint32_t *err,
                                                      uint32_t *blk = nullptr) {
    const unsigned long long m = __ballot(open);
    if (!m) return kScopeRoot;
    const uint32_t k = (uint32_t)__popcll(m);
    const uint32_t nf = (uint32_t)__builtin_amdgcn_readfirstlane((int)ls.nfree);
    // (wave-uniform: finish_open reports a bad count itself)
    if (nf < k || __ballot(open && (count == 0 || count > 255))) {
        // the free list ran dry: HBM scopes, whose parents must be HBM scopes
        // too (another wave may close them and check out of their parent)
        const uint32_t par = finish_promote(a, ls, open ? parent : kScopeRoot, err);
        return finish_open(a, open, par, count, cont, err, blk);
    }
    const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    uint32_t s = kScopeRoot;
    if (open) {
        const uint32_t slot = ls.freelist[nf - 1 - rank];
        ls.word[slot] = (unsigned long long)count << 56;
        ls.meta[slot] = hx_u32x4{parent, cont, 0u, 0u};
        s = kScopeLds | slot;
    }
    if (lane_id() == __builtin_ctzll(m)) ls.nfree = nf - k;  // (lane 0 may be inactive: an open lane)
    asm volatile("" ::: "memory");
    return s;
}

// finish_check_out over LDS and HBM scopes (a chain may cross from the
// wave's LDS into HBM, never back: an HBM scope's parent is never an
// unpromoted LDS slot). One LDS round trip per LDS step: the slot's meta
// read is issued beside its atomic (a forwarded slot's word is dead, so the
// stray add there is harmless).
// With q (a free in-flight slot), the chain's first HBM step is issued into
// it rather than waited for (finish_issue / finish_resolve). The walk runs
// in lock step: per step one LDS atomic (its meta read beside it) per lane
// still climbing; slots freed in a step go onto the free list by ballot rank
// (no returning atomic), the list's length kept in a scalar until the end.
template <int N, class Cont>
__device__ __forceinline__ uint32_t finish_check_out_local(const FinishArena &a, LocalScopes<N> &ls, uint32_t s,
                                                           unsigned long long value, Cont &&cont,
                                                           FinishInFlight *q = nullptr, uint32_t *steps = nullptr) {
    uint32_t ran = 0;  // scopes this lane completed (joins)
    unsigned long long v = value & kScopeSumMask;
    uint32_t nf = (uint32_t)__builtin_amdgcn_readfirstlane((int)ls.nfree);
    bool go = true, hbm = false, freed_any = false;
    while (__ballot(go)) {
        if (steps) ++*steps;  // (diagnostics: lock-step iterations)
        bool freeing = false;
        uint32_t slot = 0;
        if (go) {
            if (s == kScopeRoot) {
                st_agent(a.root_value, v);
                go = false;
            } else if (!scope_is_lds(s)) {
                hbm = true;
                go = false;
            } else {
                slot = s & (kScopeLds - 1);
                if (slot >= (uint32_t)N) {  // (never; see finish_check_out)
                    go = false;
                } else {
                    // the atomic first, the record read behind it: both in
                    // flight together (one round trip per step)
                    unsigned long long *wp = &ls.word[slot];
                    const hx_u32x4 *mp = &ls.meta[slot];
                    unsigned long long old = __hip_atomic_fetch_add(wp, v - kScopeOne, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP),
                                       add = v;
                    const hx_u32x4 meta = *mp;
                    if (meta.z) {
                        s = meta.z - 1;  // promoted: the HBM copy counts from here on
                    } else {
                        if ((old & kScopeSumMask) + v > kScopeSumMask) {  // see finish_check_out
                            old = __hip_atomic_fetch_add(&ls.word[slot], (unsigned long long)0 - kScopeOne,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            add = 0;
                        }
                        if ((old >> 56) != 1) {
                            go = false;
                        } else {
                            freeing = true;
                            v = cont(meta.y, (old + add) & kScopeSumMask) & kScopeSumMask;
                            ++ran;
                            s = meta.x;
                        }
                    }
                }
            }
        }
        const unsigned long long fm = __ballot(freeing);
        if (freeing)
            ls.freelist[nf + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u))] =
                slot;
        nf += (uint32_t)__popcll(fm);
        freed_any = freed_any || fm != 0;
    }
    if (freed_any) ls.nfree = nf;  // (every active lane: the same value)
    asm volatile("" ::: "memory");
    if (hbm) {
        if (q && q->s == kScopeRoot) finish_issue(a, *q, s, v);
        else ran += finish_check_out(a, s, v, cont);
    }
    return ran;
}

// A scope that needs no continuation: pass the sum up unchanged.
struct PassSum {
    __device__ unsigned long long operator()(uint32_t, unsigned long long sum) const { return sum; }
};

}  // namespace hx
