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

/* default async arguments, inc/hclib_common.h:10-22 (the reference's hclib.h
 * pulls these and <stdlib.h>/<string.h>/<assert.h> in for its test programs) */
#define NO_PROP 0
#define NO_ARG NULL
#define NO_DATUM NULL
#define NO_FUTURE NULL
#define ANY_PLACE NULL
#define NO_ACCUM NULL

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------- types */
typedef void (*generic_frame_ptr)(void *);
typedef void (*async_fct_t)(void *arg);
typedef void *(*future_fct_t)(void *arg);

struct hclib_promise_st;
typedef struct _hclib_future_t {
    struct hclib_promise_st *owner;
} hclib_future_t;

struct hclib_task_t;
typedef struct hclib_promise_st {
    hclib_future_t future; /* must stay at offset 0 (test/fib/fib.c:108-110) */
    volatile int satisfied;
    void *volatile datum;
    struct hclib_task_t *volatile wait_list_head;
} hclib_promise_t;

#define MAX_NUM_WAITS 4

typedef struct {
    int low;
    int high;
    int stride;
    int tile;
} hclib_loop_domain_t;

/* the reference's locale record, inc/hclib-locality-graph.h:56-67 (programs
 * index hclib_get_all_locales() as an array, test/c/memory/allocate.c:42-47) */
typedef struct _hclib_locale_t {
    int id;
    unsigned type;
    const char *lbl;
    const char *special_type;
    void *metadata;
    void (**idle_funcs)(void);
    unsigned n_idle_funcs;
    int reachable;
    struct _hclib_deque_t *deques;
} hclib_locale_t;

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

/* ----------------------------------------------------------- promises */
hclib_promise_t *hclib_promise_create(void);
void hclib_promise_init(hclib_promise_t *promise);
hclib_future_t *hclib_get_future_for_promise(hclib_promise_t *promise);
hclib_promise_t **hclib_promise_create_n(size_t nb_promises, int null_terminated);
void hclib_promise_free_n(hclib_promise_t **promise, size_t nb_promises, int null_terminated);
void hclib_promise_free(hclib_promise_t *promise);
void *hclib_future_get(hclib_future_t *future);
void hclib_promise_put(hclib_promise_t *promise, void *datum);
void *hclib_future_wait(hclib_future_t *future);
int hclib_future_is_satisfied(hclib_future_t *future);

/* ------------------------------------------------------------ queries */
int hclib_get_num_workers(void);
/* run ready tasks from the control thread before continuing
 * (src/hclib-runtime.c:1142-1217: non-blocking tasks until none is left,
 * a blocking one ends the yield) */
void hclib_yield(hclib_locale_t *locale);
int hclib_get_current_worker(void);
/* inc/hclib.h:61, src/hclib-runtime.c:1365-1368: tasks queued on the calling
 * worker (the host control thread's ready list) */
size_t hclib_current_worker_backlog(void);
hclib_locale_t *hclib_get_closest_locale(void);
void hclib_print_runtime_stats(FILE *fp);

/* ------------------------------------------------------------ modules */
typedef void (*hclib_module_pre_init_func_type)(void);
typedef void (*hclib_module_post_init_func_type)(void);
typedef void (*hclib_module_finalize_func_type)(void);
int hclib_add_module_init_function(const char *lbl, hclib_module_pre_init_func_type pre,
                                   hclib_module_post_init_func_type post,
                                   hclib_module_finalize_func_type finalize);

/* --------------------------------------- locales and memory operations */
/* inc/hclib-locality-graph.h:123, inc/hclib-module.h:14-15, 49-97,
 * inc/hclib.h:130-150, src/hclib-mem.c:23-241. Modules register per locale
 * TYPE the callbacks that allocate / free / set / copy memory at a locale;
 * the *_at calls run them as tasks at the locale and return futures. This
 * build registers the host ("sysmem": malloc/realloc/free/memset/memcpy)
 * and the GPU ("GPU": hipMalloc / hipFree / hipMemsetAsync /
 * hipMemcpyAsync on the module stream; its copy callback is MUST_USE, so
 * host<->GPU copies go through it). */
#define MUST_USE 1
#define MAY_USE 2
#define HCLIB_ASYNC_COPY_USE_FUTURE_AS_SRC ((void *)0x1)

typedef void *(*hclib_module_alloc_impl_func_type)(size_t, hclib_locale_t *);
typedef void *(*hclib_module_realloc_impl_func_type)(void *, size_t, hclib_locale_t *);
typedef void (*hclib_module_free_impl_func_type)(void *, hclib_locale_t *);
typedef void (*hclib_module_memset_impl_func_type)(void *, int, size_t, hclib_locale_t *);
typedef void (*hclib_module_copy_impl_func_type)(hclib_locale_t *, void *, hclib_locale_t *, void *, size_t);

int hclib_add_known_locale_type(const char *lbl);
int hclib_get_locale_type(hclib_locale_t *locale);
const char *hclib_get_locale_type_name(int type);
int hclib_get_num_locales(void);
hclib_locale_t *hclib_get_locale(int index); /* 0 = host, 1.. = GPUs */
hclib_locale_t *hclib_get_all_locales(void);  /* contiguous, hclib_get_num_locales() long */
int hclib_get_num_locales_of_type(int locale_type);
hclib_locale_t **hclib_get_all_locales_of_type(int type, int *out_count); /* malloc'd */
/* locality queries (src/hclib-locality-graph.c:829-837, 917-940, 1020-1022,
 * 1056-1170) over this runtime's graph: host system memory <-> bound GPU */
hclib_locale_t *hclib_get_master_place(void);
hclib_locale_t *hclib_get_central_place(void);
hclib_locale_t *hclib_get_closest_locale_of_type(hclib_locale_t *locale, int locale_type);
hclib_locale_t *hclib_get_closest_locale_of_types(hclib_locale_t *locale, int *locale_types, int n_locale_types);
hclib_locale_t **hclib_get_thread_private_locales(void); /* malloc'd, one per worker */
void hclib_locale_mark_special(hclib_locale_t *locale, const char *special_type);

/* loop distribution functions (inc/hclib-task.h:71-72, inc/hclib.h:93-95);
 * id HCLIB_DEFAULT_LOOP_DIST places every tile at the central place */
typedef hclib_locale_t *(*loop_dist_func)(const int, const hclib_loop_domain_t *, const hclib_loop_domain_t *,
                                          const int);
#ifndef HCLIB_DEFAULT_LOOP_DIST
#define HCLIB_DEFAULT_LOOP_DIST 0
#endif
unsigned hclib_register_dist_func(loop_dist_func func);
loop_dist_func hclib_lookup_dist_func(unsigned id);

/* inc/hclib.h:89, 253, 262 */
void hclib_run_on_main_ctx(void (*fp)(void *), void *data);
void hclib_get_curr_task_info(void (**fp_out)(void *), void **args_out);
void hclib_default_queue_capacity(int *used, int *capacity);

void hclib_register_alloc_func(int locale_type, hclib_module_alloc_impl_func_type func);
void hclib_register_realloc_func(int locale_type, hclib_module_realloc_impl_func_type func);
void hclib_register_free_func(int locale_type, hclib_module_free_impl_func_type func);
void hclib_register_memset_func(int locale_type, hclib_module_memset_impl_func_type func);
void hclib_register_copy_func(int locale_type, hclib_module_copy_impl_func_type func, int priority);

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

hclib_locale_t *hclib_hip_gpu_locale(int index);
void hclib_hip_register_async_kind(generic_frame_ptr fp, int kind);
void hclib_hip_register_forasync_body(void *forasync_fct, int body);

typedef struct {
    int type, shape_fn, gen_mx, root_id, non_leaf_bf, compute_gran;
    double b_0, non_leaf_prob, shift_depth;
    /* outputs, written when the enclosing finish ends */
    unsigned long long nodes, leaves, max_depth;
} hclib_hip_uts_task_t;

#ifdef __cplusplus
}
#endif

#define HCLIB_REGISTER_MODULE(module_name, module_pre_init_func, module_post_init_func,        \
                              module_finalize_func)                                           \
    static const int ____hclib_module_init = hclib_add_module_init_function(                  \
        module_name, module_pre_init_func, module_post_init_func, module_finalize_func);

#endif /* HCLIB_H_ */
