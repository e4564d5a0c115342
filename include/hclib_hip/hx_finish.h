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
__device__ __forceinline__ uint32_t finish_open(const FinishArena &a, bool open, uint32_t parent, uint32_t count,
                                                uint32_t cont, uint32_t *err) {
    const unsigned long long m = __ballot(open);
    if (!m) return kScopeRoot;
    const int leader = __builtin_ctzll(m);
    uint32_t base = 0;
    if (lane_id() == leader) base = add_agent(a.next, (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    if (!open) return kScopeRoot;
    const uint32_t s = base + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
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
        const uint32_t cw = ld_agent(&f->cont);
        v = cont(cw, sum) & kScopeSumMask;
        ++ran;
        s = ld_agent(&f->parent);
    }
    st_agent(a.root_value, v);
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
    uint32_t parent[N];
    uint32_t cont[N];
    uint32_t fwd[N];       // 0, or 1 + the HBM scope this slot was promoted to
    uint32_t freelist[N];
    uint32_t nfree;
    // every lane of the wave calls init once before the first open
    __device__ void init() {
        for (int i = lane_id(); i < N; i += 64) {
            freelist[i] = (uint32_t)(N - 1 - i);
            fwd[i] = 0;
        }
        if (lane_id() == 0) nfree = N;
        asm volatile("" ::: "memory");
    }
};

__device__ __forceinline__ bool scope_is_lds(uint32_t s) { return s != kScopeRoot && (s & kScopeLds); }

// The scope a lane's exported item must name: its LDS scope promoted to HBM
// (with every unpromoted LDS ancestor, top-most first), or `s` itself.
// Called by the whole wave.
template <int N>
__device__ __forceinline__ uint32_t finish_promote(const FinishArena &a, LocalScopes<N> &ls, uint32_t s,
                                                   uint32_t *err) {
    const int lead = __builtin_ctzll(__ballot(1));  // the first active lane does the scalar work
    auto unpromoted = [&](uint32_t x) { return scope_is_lds(x) && ls.fwd[x & (kScopeLds - 1)] == 0; };
    auto resolve = [&](uint32_t x) { return scope_is_lds(x) ? ls.fwd[x & (kScopeLds - 1)] - 1 : x; };
    for (int guard = 0; guard < 4 * N + 64; ++guard) {
        const unsigned long long m = __ballot(unpromoted(s));
        if (!m) break;
        // the top-most unpromoted ancestor of the first such lane's scope
        uint32_t top = (uint32_t)__builtin_amdgcn_readlane((int)s, __builtin_ctzll(m));
        for (int d = 0; d < N; ++d) {
            const uint32_t p = ls.parent[top & (kScopeLds - 1)];
            if (!unpromoted(p)) break;
            top = p;
        }
        top = (uint32_t)__builtin_amdgcn_readfirstlane((int)top);
        const uint32_t slot = top & (kScopeLds - 1);
        uint32_t h = 0;
        if (lane_id() == lead) h = add_agent(a.next, 1u);
        h = (uint32_t)__builtin_amdgcn_readfirstlane((int)h);
        if (h >= a.cap) {
            if (lane_id() == lead) dev_error(err, kErrArena);
            return kScopeRoot;
        }
        if (lane_id() == lead) {
            FinishScope *f = &a.scopes[h];
            st_agent(&f->word, ls.word[slot]);
            st_agent(&f->parent, resolve(ls.parent[slot]));
            st_agent(&f->cont, ls.cont[slot]);
            ls.fwd[slot] = h + 1;
        }
        asm volatile("" ::: "memory");
    }
    return resolve(s);
}

// An open that prefers the wave's LDS: lanes with `open` each get an LDS
// scope while the free list lasts, the rest HBM scopes (finish_open).
template <int N>
__device__ __forceinline__ uint32_t finish_open_local(const FinishArena &a, LocalScopes<N> &ls, bool open,
                                                      uint32_t parent, uint32_t count, uint32_t cont, uint32_t *err) {
    const unsigned long long m = __ballot(open);
    if (!m) return kScopeRoot;
    const uint32_t k = (uint32_t)__popcll(m);
    const uint32_t nf = (uint32_t)__builtin_amdgcn_readfirstlane((int)ls.nfree);
    // (wave-uniform: finish_open reports a bad count itself)
    if (nf < k || __ballot(open && (count == 0 || count > 255))) {
        // the free list ran dry: HBM scopes, whose parents must be HBM scopes
        // too (another wave may close them and check out of their parent)
        const uint32_t par = finish_promote(a, ls, open ? parent : kScopeRoot, err);
        return finish_open(a, open, par, count, cont, err);
    }
    const uint32_t rank = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    uint32_t s = kScopeRoot;
    if (open) {
        const uint32_t slot = ls.freelist[nf - 1 - rank];
        ls.word[slot] = (unsigned long long)count << 56;
        ls.parent[slot] = parent;
        ls.cont[slot] = cont;
        ls.fwd[slot] = 0;
        s = kScopeLds | slot;
    }
    if (lane_id() == __builtin_ctzll(m)) ls.nfree = nf - k;  // (lane 0 may be inactive: an open lane)
    asm volatile("" ::: "memory");
    return s;
}

// finish_check_out over LDS and HBM scopes (a chain may cross from the
// wave's LDS into HBM, never back: an HBM scope's parent is never an
// unpromoted LDS slot)
template <int N, class Cont>
__device__ __forceinline__ uint32_t finish_check_out_local(const FinishArena &a, LocalScopes<N> &ls, uint32_t s,
                                                           unsigned long long value, Cont &&cont) {
    uint32_t ran = 0;
    unsigned long long v = value & kScopeSumMask;
    while (s != kScopeRoot) {
        if (!scope_is_lds(s)) return ran + finish_check_out(a, s, v, cont);
        const uint32_t slot = s & (kScopeLds - 1);
        if (slot >= (uint32_t)N) return ran;  // (never; see finish_check_out)
        const uint32_t f = ls.fwd[slot];
        if (f) {  // promoted: the HBM copy counts from here on
            s = f - 1;
            continue;
        }
        unsigned long long old = __hip_atomic_fetch_add(&ls.word[slot], v - kScopeOne, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP),
                           add = v;
        if ((old & kScopeSumMask) + v > kScopeSumMask) {  // see finish_check_out
            old = __hip_atomic_fetch_add(&ls.word[slot], (unsigned long long)0 - kScopeOne, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
            add = 0;
        }
        if ((old >> 56) != 1) return ran;
        const unsigned long long sum = (old + add) & kScopeSumMask;
        const uint32_t cw = ls.cont[slot], par = ls.parent[slot];
        // the slot is free again
        const uint32_t pos = __hip_atomic_fetch_add(&ls.nfree, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ls.freelist[pos] = slot;
        v = cont(cw, sum) & kScopeSumMask;
        ++ran;
        s = par;
    }
    st_agent(a.root_value, v);
    return ran;
}

// A scope that needs no continuation: pass the sum up unchanged.
struct PassSum {
    __device__ unsigned long long operator()(uint32_t, unsigned long long sum) const { return sum; }
};

}  // namespace hx
