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

// A scope that needs no continuation: pass the sum up unchanged.
struct PassSum {
    __device__ unsigned long long operator()(uint32_t, unsigned long long sum) const { return sum; }
};

}  // namespace hx
