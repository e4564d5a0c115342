// modules/hip — the GPU locale type and its memory operations as an HClib
// plug-in module (libhclib_hip.so), loaded like any other module by
// hclib_launch / hclib_init when `deps` names "hip" (src/hclib-runtime.c:
// 294-317: dlopen of libhclib_<dep>.so, whose static initialiser runs
// HCLIB_REGISTER_MODULE).
//
// The MI355X counterpart of the reference's modules/cuda/src/hclib_cuda.cpp:
//   pre-init   registers the "GPU" locale type and its metadata functions
//              (hclib_cuda.cpp:156-167): every GPU locale of the graph gets
//              an hclib_hip_locale_metadata_t naming its HIP device ("GPU<k>"
//              is device k, otherwise the order of appearance)
//   post-init  registers the locale type's memory callbacks
//              (hclib_cuda.cpp:169-174): hipMalloc / hipFree / a hipMalloc +
//              copy realloc / hipMemsetAsync / hipMemcpyAsync, the copy with
//              MUST_USE priority
//   finalize   drains the module stream
// Every callback runs on the process's bound gfx950 device (one GPU per
// process, the multi-GPU launch's rank model) through the module's C ABI
// (include/hclib_hip.h: hclib_hip_init / hclib_hip_device / hclib_hip_stream)
// and completes before it returns, so the future the runtime puts after it
// (src/hclib-mem.c:59-191) means the data is in place. Nothing here touches
// the device until the first callback runs: a program can load a locality
// graph with GPU locales on a host without one.
//
// hclib_hip_module_counts() reports how many times each callback ran, so a
// program (tests/c/mem_locale.c, tests/c/locality_file.c) can check that its
// memory operations at a GPU locale went through this module.
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>

#include <hip/hip_runtime.h>

#include "../../../include/hclib.h"
#include "../../../include/hclib-module.h"
#include "../../../include/hclib_hip.h"

namespace {

int gpu_locale_id = -1;
int gpus_so_far = 0;
std::atomic<unsigned long long> counts[6];  // alloc, realloc, free, memset, copy, metadata populated

[[noreturn]] void fail(const char *who, const char *what) {
    fprintf(stderr, "hclib: %s: %s\n", who, what);
    abort();
}

// the stream of the device the locale names; binds the process to it on the
// first use (a second device is an error: one rank drives one GPU)
hipStream_t bound_stream(const hclib_locale_t *l, const char *who) {
    const hclib_hip_locale_metadata_t *m = (const hclib_hip_locale_metadata_t *)l->metadata;
    const int want = m ? m->device : 0;
    const int have = hclib_hip_device();
    if (have < 0) {
        if (hclib_hip_init(want) != HCLIB_HIP_OK) {
            fprintf(stderr, "hclib: %s: the hip module could not bind a gfx950 device: %s\n", who,
                    hclib_hip_last_error());
            abort();
        }
    } else if (have != want) {
        char msg[160];
        snprintf(msg, sizeof(msg), "this process drives GPU %d; GPU %d needs a process of its own", have, want);
        fail(who, msg);
    }
    return (hipStream_t)hclib_hip_stream();
}

size_t metadata_size() { return sizeof(hclib_hip_locale_metadata_t); }

void metadata_populate(hclib_locale_t *locale) {
    hclib_hip_locale_metadata_t *m = (hclib_hip_locale_metadata_t *)locale->metadata;
    const char *s = locale->lbl ? locale->lbl + 3 : "";  // "GPU<k>"
    m->device = (*s && isdigit((unsigned char)*s)) ? atoi(s) : gpus_so_far;
    gpus_so_far++;
    counts[5]++;
}

void *allocation_func(size_t nbytes, hclib_locale_t *locale) {
    bound_stream(locale, "hclib_allocate_at");
    void *p = nullptr;
    if (hipMalloc(&p, nbytes ? nbytes : 1) != hipSuccess) fail("hclib_allocate_at", "hipMalloc failed");
    counts[0]++;
    return p;
}

void free_func(void *ptr, hclib_locale_t *locale) {
    (void)locale;
    if (ptr && hipFree(ptr) != hipSuccess) fail("hclib_free_at", "hipFree failed");
    counts[2]++;
}

void *reallocation_func(void *ptr, size_t nbytes, hclib_locale_t *locale) {
    hipStream_t s = bound_stream(locale, "hclib_reallocate_at");
    void *q = nullptr;
    if (hipMalloc(&q, nbytes ? nbytes : 1) != hipSuccess) fail("hclib_reallocate_at", "hipMalloc failed");
    if (ptr) {
        size_t old = 0;
        if (hipMemPtrGetInfo(ptr, &old) != hipSuccess) fail("hclib_reallocate_at", "not a device allocation");
        if (hipMemcpyAsync(q, ptr, old < nbytes ? old : nbytes, hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            fail("hclib_reallocate_at", "copy failed");
        if (hipFree(ptr) != hipSuccess) fail("hclib_reallocate_at", "hipFree failed");
    }
    counts[1]++;
    return q;
}

void memset_func(void *ptr, int val, size_t nbytes, hclib_locale_t *locale) {
    hipStream_t s = bound_stream(locale, "hclib_memset_at");
    if (hipMemsetAsync(ptr, val, nbytes, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        fail("hclib_memset_at", "hipMemsetAsync failed");
    counts[3]++;
}

// either side (or both) at a GPU locale: hipMemcpyDefault infers the
// direction from the pointers (hclib_cuda.cpp:103-139 picks it by locale)
void copy_func(hclib_locale_t *dst_locale, void *dst, hclib_locale_t *src_locale, void *src, size_t nbytes) {
    const bool dst_gpu = (int)dst_locale->type == gpu_locale_id, src_gpu = (int)src_locale->type == gpu_locale_id;
    if (!dst_gpu && !src_gpu) fail("hclib_async_copy", "no GPU locale involved");
    hipStream_t s = bound_stream(dst_gpu ? dst_locale : src_locale, "hclib_async_copy");
    if (hipMemcpyAsync(dst, src, nbytes, hipMemcpyDefault, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        fail("hclib_async_copy", "hipMemcpyAsync failed");
    counts[4]++;
}

HCLIB_MODULE_PRE_INITIALIZATION_FUNC(hip_pre_initialize) {
    gpu_locale_id = (int)hclib_add_known_locale_type("GPU");
    gpus_so_far = 0;
    hclib_add_locale_metadata_functions(gpu_locale_id, metadata_size, metadata_populate);
}

HCLIB_MODULE_INITIALIZATION_FUNC(hip_post_initialize) {
    hclib_register_alloc_func(gpu_locale_id, allocation_func);
    hclib_register_realloc_func(gpu_locale_id, reallocation_func);
    hclib_register_free_func(gpu_locale_id, free_func);
    hclib_register_memset_func(gpu_locale_id, memset_func);
    hclib_register_copy_func(gpu_locale_id, copy_func, MUST_USE);
}

HCLIB_MODULE_INITIALIZATION_FUNC(hip_finalize) {
    if (hclib_hip_device() >= 0) (void)hipStreamSynchronize((hipStream_t)hclib_hip_stream());
}

}  // namespace

HCLIB_REGISTER_MODULE("hip", hip_pre_initialize, hip_post_initialize, hip_finalize)

extern "C" {
// calls of each callback so far: alloc, realloc, free, memset, copy, GPU
// locales whose metadata this module populated
__attribute__((visibility("default"))) void hclib_hip_module_counts(unsigned long long out[6]) {
    for (int i = 0; i < 6; ++i) out[i] = counts[i].load();
}
// the locale type id this module registered ("GPU"), -1 before pre-init
__attribute__((visibility("default"))) int hclib_hip_module_gpu_type(void) { return gpu_locale_id; }
}
