/*
 * hclib-module.h — the module plug-in ABI (MI355X build).
 *
 * Same names, types and registration macros as the reference's
 * inc/hclib-module.h:14-106, so a module written for HClib (e.g. the
 * reference's modules/system/src/hclib_system.cpp) compiles unchanged:
 *   MUST_USE / MAY_USE                                  :14-15
 *   hclib_module_{pre_init,post_init,finalize}_func_type :21-31
 *   hclib_state_adder / hclib_state_releaser            :36-42
 *   hclib_locale_metadata_{size,populate}_func_type     :48-49
 *   hclib_module_{alloc,realloc,free,memset,copy}_impl_func_type :52-59
 *   HCLIB_MODULE_*_FUNC / HCLIB_REGISTER_MODULE          :61-64
 *   registration + per-worker module state functions    :79-106
 *
 * Loading (src/hclib-runtime.c:294-317): hclib_launch/hclib_init dlopen
 * $HCLIB_ROOT/lib/libhclib_<dep>.so for every name in `deps` (and
 * $HCLIB_MODULE_PATH/libhclib_<dep>.so first, when set); the library's
 * static initialiser runs HCLIB_REGISTER_MODULE. A missing library is a
 * warning, as in the reference. "hip" is this project's plug-in module
 * libhclib_hip.so (hclib_amd/csrc/modules/hclib_hip_module.hip, built beside
 * libhclib_amd.so): it registers the "GPU" locale type, its metadata and its
 * memory callbacks through this ABI, as modules/cuda does in the reference.
 */
#ifndef HCLIB_MODULE_H
#define HCLIB_MODULE_H

#include <stddef.h>

#include "hclib-locality-graph.h"

#define MUST_USE 1
#define MAY_USE 2

typedef void (*hclib_module_pre_init_func_type)();
typedef void (*hclib_module_post_init_func_type)();
typedef void (*hclib_module_finalize_func_type)();

typedef void (*hclib_state_adder)(void *state, void *user_data, int tid);
typedef void (*hclib_state_releaser)(void *state, void *user_data);

typedef size_t (*hclib_locale_metadata_size_func_type)();
typedef void (*hclib_locale_metadata_populate_func_type)(hclib_locale_t *);

typedef void *(*hclib_module_alloc_impl_func_type)(size_t, hclib_locale_t *);
typedef void *(*hclib_module_realloc_impl_func_type)(void *, size_t, hclib_locale_t *);
typedef void (*hclib_module_free_impl_func_type)(void *, hclib_locale_t *);
typedef void (*hclib_module_memset_impl_func_type)(void *, int, size_t, hclib_locale_t *);
typedef void (*hclib_module_copy_impl_func_type)(hclib_locale_t *, void *, hclib_locale_t *, void *, size_t);

#define HCLIB_MODULE_PRE_INITIALIZATION_FUNC(module_init_funcname) void module_init_funcname()
#define HCLIB_MODULE_INITIALIZATION_FUNC(module_init_funcname) void module_init_funcname()
#ifdef __cplusplus
#define HCLIB_REGISTER_MODULE(module_name, module_pre_init_func, module_post_init_func,        \
                              module_finalize_func)                                           \
    const static int ____hclib_module_init = hclib_add_module_init_function(                  \
        module_name, module_pre_init_func, module_post_init_func, module_finalize_func);
#else
/* C has no dynamic initialisers: the same registration from a constructor */
#define HCLIB_REGISTER_MODULE(module_name, module_pre_init_func, module_post_init_func,        \
                              module_finalize_func)                                           \
    __attribute__((constructor)) static void ____hclib_module_ctor(void) {                   \
        hclib_add_module_init_function(module_name, module_pre_init_func, module_post_init_func, \
                                       module_finalize_func);                                 \
    }
#endif

#ifdef __cplusplus
extern "C" {
#endif
int hclib_add_module_init_function(const char *lbl, hclib_module_pre_init_func_type pre,
                                   hclib_module_post_init_func_type post,
                                   hclib_module_finalize_func_type finalize);

/* src/hclib-locality-graph.c:322-367 runs these on every locale of the type
 * when the graph is built: metadata = malloc(size_func()), then populate */
void hclib_add_locale_metadata_functions(int locale_id, hclib_locale_metadata_size_func_type size_func,
                                         hclib_locale_metadata_populate_func_type populate_func);

void hclib_register_alloc_func(int locale_id, hclib_module_alloc_impl_func_type func);
void hclib_register_realloc_func(int locale_id, hclib_module_realloc_impl_func_type func);
void hclib_register_free_func(int locale_id, hclib_module_free_impl_func_type func);
void hclib_register_memset_func(int locale_id, hclib_module_memset_impl_func_type func);
void hclib_register_copy_func(int locale_id, hclib_module_copy_impl_func_type func, int priority);

void hclib_call_module_pre_init_functions(void);
void hclib_call_module_post_init_functions(void);
void hclib_call_finalize_functions(void);

/* src/hclib_module.c:129-160: a module reserves state_size bytes in every
 * worker's module_state; cb(state, user_data, worker id) initialises each.
 * Returns the offset (state id) hclib_get_curr_worker_module_state takes. */
unsigned hclib_add_per_worker_module_state(size_t state_size, hclib_state_adder cb, void *user_data);
void *hclib_get_curr_worker_module_state(const unsigned state_id);
void hclib_release_per_worker_module_state(const unsigned state_id, hclib_state_releaser cb, void *user_data);
#ifdef __cplusplus
}
#endif

#endif
