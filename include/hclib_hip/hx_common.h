// hx_common.h — shared device/host helpers for the MI355X hclib module.
//
// Inter-workgroup protocol (MI355X_MICROARCH.md "Workgroup dispatch, XCD
// placement & inter-workgroup visibility", cdna_hip_programming.md G16):
// every word another workgroup reads is written and read with agent-scope
// atomics (global_* sc1: bypasses the per-CU L1, write-through past the
// per-XCD L2), published behind `s_waitcnt vmcnt(0)` + an agent release
// fence, and consumed after an agent acquire fence. Spins are bounded and
// report through a device error word instead of hanging the GPU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define HX_AGENT __HIP_MEMORY_SCOPE_AGENT

namespace hx {

// ------------------------------------------------------------------ errors
enum DevError : uint32_t {
    kErrNone = 0,
    kErrQueueFull = 1,
    kErrStackOverflow = 2,
    kErrSpinTimeout = 3,
    kErrDepthTable = 4,
    kErrArena = 5,
    kErrBadTask = 6,
};

__device__ __forceinline__ void dev_error(uint32_t *err, uint32_t code) {
    uint32_t zero = 0;
    __hip_atomic_compare_exchange_strong(err, &zero, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         HX_AGENT);
}

// the same for a word shared with other GPUs (first error wins)
__device__ __forceinline__ void dev_error_sys(uint32_t *err, uint32_t code) {
    uint32_t zero = 0;
    __hip_atomic_compare_exchange_strong(err, &zero, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
}

// --------------------------------------------------------- agent atomics
template <typename T>
__device__ __forceinline__ T ld_agent(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, HX_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, HX_AGENT);
}
template <typename T>
__device__ __forceinline__ T add_agent(T *p, T v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, HX_AGENT);
}
template <typename T>
__device__ __forceinline__ bool cas_agent(T *p, T expected, T desired) {
    return __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_RELAXED,
                                                __ATOMIC_RELAXED, HX_AGENT);
}

// system-scope forms: words shared with other GPUs (cross-GPU work sharing,
// hx_sched.h GlobalView) — coherent across devices, not only across the XCDs
// of one
template <typename T>
__device__ __forceinline__ T ld_sys(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void st_sys(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T add_sys(T *p, T v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ bool cas_sys(T *p, T expected, T desired) {
    return __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM);
}

// 16-byte agent-scope (sc1, write-through) store and load: MI355X_MICROARCH.md
// prices a dword sc1 store at ~6x, a dwordx2 at 2.7x the per-byte time of a
// dwordx4 one. The load waits for itself (inline asm is invisible to the
// compiler's waitcnt pass); ld_sc1_x4x2 issues two before one wait.
typedef uint32_t hx_u32x4 __attribute__((ext_vector_type(4)));
// The s_nop: a store of more than 8 bytes reads its data registers after
// issue, and the compiler's hazard recognizer does not cover an inline-asm
// store, so a VALU write of those registers right behind it (the next
// store's address, built in the same registers) corrupted the stored data
// (UTS T1: nodes lost and duplicated in 42 of 60 launches when the chunk
// payload's reads moved ahead of its ticket and the schedule tightened).
// RULE for every inline-asm store of dwordx3 / dwordx4 in this tree: the
// same asm statement ends the store with `s_nop N`, N >= 1, right after it
// (tests/test_asm_hazards.py enforces it on the CPU suite)
__device__ __forceinline__ void st_sc1_x4(void *p, uint4 v) {
    const hx_u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 2" ::"v"(p), "v"(x) : "memory");
}
__device__ __forceinline__ void ld_sc1_x4x2(const void *p, uint4 &a, uint4 &b) {
    hx_u32x4 x, y;
    asm volatile("global_load_dwordx4 %0, %2, off sc1\n"
                 "global_load_dwordx4 %1, %2, off offset:16 sc1\n"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(x), "=&v"(y)
                 : "v"(p)
                 : "memory");
    a = make_uint4(x.x, x.y, x.z, x.w);
    b = make_uint4(y.x, y.y, y.z, y.w);
}

// A dword agent-scope store as inline asm: the same global_store_dword sc1
// as st_agent, but invisible to the compiler's waitcnt pass, which would
// otherwise wait (vmcnt(0)) for it before the next write to its data
// register — and so for every load issued since (the scheduler's hand-off
// words: the loop's next batch body overwrites those registers at once)
__device__ __forceinline__ void st_sc1_u32(uint32_t *p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// s_waitcnt vmcnt(0) the compiler's waitcnt pass can see (an inline-asm wait
// is opaque to it: stores it still believes in flight make it insert a
// vmcnt(0) before the next write to their data VGPRs — which also waits for
// any load issued since, e.g. the one-batch-late hunger read).
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Producer side of a hand-off: drain this wave's stores, then release.
__device__ __forceinline__ void release_agent() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// Consumer side: invalidate this CU's L1 before reading handed-off bytes.
__device__ __forceinline__ void acquire_agent() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------ LDS flags
// Words that the waves of one workgroup hand to each other through LDS
// (inbox states, counts). The LDS performs one wave's DS operations in issue
// order, so a flag stored after the data it guards is seen after that data
// by a wave that reads the flag first. These go through address-space-3
// pointers: a `volatile` (or atomic) access through a generic pointer
// compiles to a FLAT operation, which waits for the wave's global memory
// traffic too (vmcnt) and leaves the DS queue, so it is not ordered with the
// wave's ds_write of the data.
typedef __attribute__((address_space(3))) uint32_t hx_lds_u32;
__device__ __forceinline__ uint32_t lds_load(const uint32_t *p) {
    asm volatile("" ::: "memory");
    const uint32_t v = __hip_atomic_load((const hx_lds_u32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    return v;
}
__device__ __forceinline__ void lds_store(uint32_t *p, uint32_t v) {
    asm volatile("" ::: "memory");
    __hip_atomic_store((hx_lds_u32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ bool lds_cas(uint32_t *p, uint32_t expected, uint32_t desired) {
    asm volatile("" ::: "memory");
    const bool ok = __hip_atomic_compare_exchange_strong((hx_lds_u32 *)p, &expected, desired, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    return ok;
}

// ------------------------------------------------------------ wave utils
// hclib_get_current_worker / hclib_get_num_workers in device code
// (src/hclib-runtime.c:194-226): a device worker is one wave of the launch,
// numbered 0 .. num_workers() - 1 across the grid (UTS.cpp:104-106,220-221
// index per-worker state by it)
__device__ __forceinline__ int current_worker() {
    return (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}
__device__ __forceinline__ int num_workers() { return (int)(gridDim.x * (blockDim.x >> 6)); }

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// XCD (XCC) id of the executing CU: speed hint only, never correctness.
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ int wave_incl_max_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(v, d, 64);
        if (lane >= d) v = v > t ? v : t;
    }
    return v;
}

__device__ __forceinline__ int wave_bcast(int v, int src) { return __shfl(v, src, 64); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        T t = __shfl_xor(v, d, 64);
        v = v > t ? v : t;
    }
    return v;
}

__device__ __forceinline__ void sleep_short() { __builtin_amdgcn_s_sleep(2); }

}  // namespace hx
