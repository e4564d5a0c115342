/*
 * hclib-rt.h — worker state and runtime queries of the HClib C API (MI355X build).
 *
 * Mirrors the reference's inc/hclib-rt.h:
 *   hclib_worker_state   inc/hclib-rt.h:80-111 (same field order; the fiber
 *                        pointers are opaque here: this build has no fibers)
 *   ws_key / CURRENT_WS_INTERNAL / current_ws()   inc/hclib-rt.h:56, 140-143
 *   HASSERT / HASSERT_STATIC                      inc/hclib-rt.h:116-138
 *
 * Workers of this build: the HOST has one worker, the control
 * thread that calls hclib_launch (worker 0); it runs every host task help-
 * first. The GPU's workers are the megakernel's waves; their ids and count
 * are the device locale's (hclib_hip_num_workers(), and device code reads
 * its own wave id). hclib_get_num_workers() / hclib_get_current_worker() /
 * current_ws() answer for the host, where C code runs.
 */
#ifndef HCLIB_RT_H_
#define HCLIB_RT_H_

#include <assert.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

#ifdef __cplusplus
extern "C" {
#endif

extern pthread_key_t ws_key;
struct hclib_context;
struct finish_t;
struct _hclib_worker_paths;
struct _hclib_lite_ctx;

typedef struct _hclib_worker_state {
    struct hclib_context *context;
    struct _hclib_worker_paths *paths;
    pthread_t t;
    struct finish_t *current_finish;
    struct _hclib_lite_ctx *curr_ctx;
    struct _hclib_lite_ctx *root_ctx;
    int id;
    int nworkers;
    char *module_state; /* per-worker module state, hclib_add_per_worker_module_state */
    int base_intra_socket_workers;
    int limit_intra_socket_workers;
    void *curr_task; /* the hclib_task_t this worker is running */
} __attribute__((aligned(128))) hclib_worker_state;

#define HCLIB_MACRO_CONCAT(x, y) _HCLIB_MACRO_CONCAT_IMPL(x, y)
#define _HCLIB_MACRO_CONCAT_IMPL(x, y) x##y

#ifdef HC_ASSERTION_CHECK
#define HASSERT(cond)                                                                        \
    {                                                                                        \
        if (!(cond)) {                                                                       \
            if (pthread_getspecific(ws_key)) {                                               \
                fprintf(stderr, "W%d: assertion failure\n", hclib_get_current_worker());    \
            }                                                                                \
            assert(cond);                                                                    \
        }                                                                                    \
    }
#else
#define HASSERT(cond)
#endif

#if defined(static_assert) || __cplusplus >= 201103L
#define HASSERT_STATIC static_assert
#elif __STDC_VERSION__ >= 201112L
#define HASSERT_STATIC _Static_assert
#endif

#define CURRENT_WS_INTERNAL ((hclib_worker_state *)pthread_getspecific(ws_key))

int hclib_get_current_worker(void);
hclib_worker_state *current_ws(void);

typedef void (*generic_frame_ptr)(void *);

int hclib_get_num_workers(void);
void hclib_start_finish(void);
void hclib_end_finish(void);
/* inc/hclib-rt.h:153 (src/hclib-runtime.c:1319-1321): the harness's own
 * timing of the user region, in seconds; HCLIB_STATS reports it */
void hclib_user_harness_timer(double dur);

#ifdef __cplusplus
}
#endif

#include "hclib-promise.h"

#endif /* HCLIB_RT_H_ */
