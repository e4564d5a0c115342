/*
 * hclib.h — the HClib C API (drop-in surface) of the MI355X build.
 *
 * Same names, prototypes, struct layouts and error behaviour as the
 * reference's public C API, so HClib C programs compile unchanged against
 * this header and link against hclib_amd/lib/libhclib_amd.so:
 *
 *   this header                         reference
 *   ----------------------------------  -------------------------------------
 *   hclib_launch / hclib_init / _finalize  inc/hclib.h:67-73
 *   hclib_async / _nb / _future            inc/hclib.h:111-125
 *   hclib_forasync / _future               inc/hclib.h:205-214
 *   hclib_start_finish / hclib_end_finish
 *     / _nonblocking(_helper)              inc/hclib.h:219-231
 *   hclib_promise_* / hclib_future_*       inc/hclib-promise.h:96-156
 *   hclib_loop_domain_t                    inc/hclib-task.h:53-58
 *   hclib_promise_t / hclib_future_t       inc/hclib-promise.h:65-90
 *   hclib_get_num_workers / _current_worker,
 *   hclib_get_closest_locale, hclib_print_runtime_stats,
 *   hclib_current_time_ns/ms               inc/hclib.h:64-80, 251; inc/hclib-rt.h
 *   hclib_add_module_init_function         inc/hclib-module.h:64, 79-82
 *
 * and, through the headers it includes (same split as the reference's inc/):
 *   hclib-task.h        hclib_task_t (96 B), loop_dist_func
 *   hclib-async-struct.h spawn / spawn_at / spawn_await / spawn_await_at
 *   hclib-rt.h          hclib_worker_state, ws_key, current_ws(), HASSERT
 *   hclib-module.h      module plug-in ABI, per-worker module state
 *   hclib-locality-graph.h  locales, the locality graph, locality queries
 *
 * Execution model on MI355X: the calling thread is the host
 * control thread. Functions registered as device task kinds or device loop
 * bodies (hclib_hip_register_*, below) execute on the GPU: hclib_async of a
 * device kind becomes a persistent-megakernel launch whose internal
 * async/finish/promise traffic runs on device counters; hclib_forasync of a
 * device body becomes one grid-stride launch. Other functions are host
 * tasks: they run on the control thread, help-first inside end_finish, as
 * the reference's help_finish does (src/hclib-runtime.c:1067-1119); a
 * forasync of a host loop body becomes one host task per tile of the
 * reference's FLAT/RECURSIVE lowering (src/hclib.c:110-473).
 * Errors abort with a message, like the reference's HASSERT/exit paths.
 */
#ifndef HCLIB_H_
#define HCLIB_H_

#include <assert.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* the reference's hclib.h pulls in the common macros, the task record and the
 * promise API (inc/hclib.h:35-37); the module ABI and the locality graph are
 * part of the same surface here (inc/hclib-module.h, inc/hclib-locality-graph.h) */
#include "hclib_common.h"
#include "hclib-task.h"
#include "hclib-promise.h"
#include "hclib-module.h"
#include "hclib-async-struct.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------- types */
typedef void (*async_fct_t)(void *arg);
typedef void *(*future_fct_t)(void *arg);

typedef int forasync_mode_t;
#define FORASYNC_MODE_RECURSIVE 1
#define FORASYNC_MODE_FLAT 0

typedef void (*forasync1D_Fct_t)(void *arg, int index);
typedef void (*forasync2D_Fct_t)(void *arg, int index_outer, int index_inner);
typedef void (*forasync3D_Fct_t)(void *arg, int index_outer, int index_mid, int index_inner);

/* ---------------------------------------------------------- lifecycle */
void hclib_init(const char **module_dependencies, int n_module_dependencies, const int instrument);
void hclib_finalize(const int instrument);
void hclib_launch(async_fct_t fct_ptr, void *arg, const char **deps, int ndeps);

unsigned long long hclib_current_time_ns(void);
unsigned long long hclib_current_time_ms(void);

/* -------------------------------------------------------------- tasks */
void hclib_async(generic_frame_ptr fp, void *arg, hclib_future_t **futures, const int nfutures,
                 hclib_locale_t *locale);
void hclib_async_nb(generic_frame_ptr fp, void *arg, hclib_locale_t *locale);
hclib_future_t *hclib_async_future(future_fct_t fp, void *arg, hclib_future_t **futures,
                                   const int nfutures, hclib_locale_t *locale);

void hclib_forasync(void *forasync_fct, void *argv, int dim, hclib_loop_domain_t *domain,
                    forasync_mode_t mode);
hclib_future_t *hclib_forasync_future(void *forasync_fct, void *argv, int dim,
                                      hclib_loop_domain_t *domain, forasync_mode_t mode);

void hclib_start_finish(void);
void hclib_end_finish(void);
hclib_future_t *hclib_end_finish_nonblocking(void);
void hclib_end_finish_nonblocking_helper(hclib_promise_t *event);

/* ------------------------------------------------------------ queries */
/* run ready tasks from the control thread before continuing
 * (src/hclib-runtime.c:1142-1217: non-blocking tasks until none is left,
 * a blocking one ends the yield) */
void hclib_yield(hclib_locale_t *locale);
/* inc/hclib.h:61, src/hclib-runtime.c:1365-1368: tasks queued on the calling
 * worker (the host control thread's ready list) */
size_t hclib_current_worker_backlog(void);
void hclib_print_runtime_stats(FILE *fp);

/* --------------------------------------- locales and memory operations */
/* inc/hclib.h:130-150, src/hclib-mem.c:23-241. Modules register per locale
 * TYPE the callbacks that allocate / free / set / copy memory at a locale
 * (hclib-module.h); the *_at calls run them as tasks at the locale and
 * return futures. Built in: the host ("sysmem": malloc/realloc/free/memset/
 * memcpy, MAY_USE) and the GPU ("GPU": hipMalloc / hipFree / hipMemsetAsync
 * / hipMemcpyAsync on the module stream; its copy callback is MUST_USE, so
 * host<->GPU copies go through it). */
#define HCLIB_ASYNC_COPY_USE_FUTURE_AS_SRC ((void *)0x1)

/* this build's extensions: a locale's type id and name, and indexed access
 * (locale 0 = system memory, then the GPU locales) */
int hclib_get_locale_type(hclib_locale_t *locale);
const char *hclib_get_locale_type_name(int type);
hclib_locale_t *hclib_get_locale(int index);

/* loop distribution functions (inc/hclib.h:93-95); id HCLIB_DEFAULT_LOOP_DIST
 * places every tile at the central place */
#ifndef HCLIB_DEFAULT_LOOP_DIST
#define HCLIB_DEFAULT_LOOP_DIST 0
#endif
unsigned hclib_register_dist_func(loop_dist_func func);
loop_dist_func hclib_lookup_dist_func(unsigned id);

/* inc/hclib.h:89, 253, 262 */
void hclib_run_on_main_ctx(void (*fp)(void *), void *data);
void hclib_get_curr_task_info(void (**fp_out)(void *), void **args_out);
void hclib_default_queue_capacity(int *used, int *capacity);

hclib_future_t *hclib_allocate_at(size_t nbytes, hclib_locale_t *locale);
hclib_future_t *hclib_reallocate_at(void *ptr, size_t new_nbytes, hclib_locale_t *locale);
hclib_future_t *hclib_memset_at(void *ptr, int pattern, size_t nbytes, hclib_locale_t *locale);
void hclib_free_at(void *ptr, hclib_locale_t *locale);
hclib_future_t *hclib_async_copy(hclib_locale_t *dst_locale, void *dst, hclib_locale_t *src_locale,
                                 void *src, size_t nbytes, hclib_future_t **futures, const int nfutures);

/* --------------------------------------- modules/hip device task kinds */
/* A host function pointer cannot run on the GPU: programs name which of
 * their functions are device task kinds / loop bodies. The argument
 * layouts are the reference drivers' own structs. */
#define HCLIB_HIP_KIND_FIB 1 /* fib(void*) of test/fib/fib.c:57-71; arg = {int n; long res;} */
#define HCLIB_HIP_KIND_UTS 2 /* UTS search; arg = hclib_hip_uts_task_t below */

/* the metadata the hip plug-in module (libhclib_hip.so) attaches to every GPU-type locale
 * (hclib_add_locale_metadata_functions): the HIP device it stands for */
typedef struct {
    int device;
} hclib_hip_locale_metadata_t;

hclib_locale_t *hclib_hip_gpu_locale(int index);
void hclib_hip_register_async_kind(generic_frame_ptr fp, int kind);
void hclib_hip_register_forasync_body(void *forasync_fct, int body);

/* The kind table of the program's own device code: a HIP translation unit
 * the program links names, for a host function of the program, the launcher
 * that runs it on the bound GPU (HCLIB_HIP_DEVICE_ASYNC /
 * HCLIB_HIP_DEVICE_FORASYNC in include/hclib_hip_cpp.h register them before
 * main). An async of a registered function runs its launcher instead of the
 * host function; a forasync of a registered body enqueues the launcher's
 * sweep, which completes with the enclosing finish. Launchers return
 * HCLIB_HIP_OK or a negative HCLIB_HIP_E* code (include/hclib_hip.h); a
 * failing launcher ends the program with its message, as a failing device
 * kind does. Kinds and bodies outside the table are refused (the register
 * calls above only take the built-in ids). */
typedef int (*hclib_hip_async_launcher_t)(void *args);
typedef int (*hclib_hip_forasync_launcher_t)(void *args, int dim, hclib_loop_domain_t *domain, int mode,
                                             void *stream);
void hclib_hip_register_device_async(generic_frame_ptr fp, const char *name, hclib_hip_async_launcher_t launch);
void hclib_hip_register_device_forasync(void *forasync_fct, const char *name,
                                        hclib_hip_forasync_launcher_t launch);
/* registered device task kinds, and the name of one (NULL: not a kind) */
int hclib_hip_device_kind_count(void);
const char *hclib_hip_device_kind_name(generic_frame_ptr fp);

typedef struct {
    int type, shape_fn, gen_mx, root_id, non_leaf_bf, compute_gran;
    double b_0, non_leaf_prob, shift_depth;
    /* outputs, written when the enclosing finish ends */
    unsigned long long nodes, leaves, max_depth;
} hclib_hip_uts_task_t;

#ifdef __cplusplus
}
#endif

#endif /* HCLIB_H_ */
