/*
 * hclib-task.h — the task record and loop domains (MI355X build).
 *
 * Same layout as the reference's inc/hclib-task.h:
 *   hclib_task_t         :32-44, 96 bytes on LP64 (the header-only C++ layer
 *                        of the reference allocates it and hands it to spawn*,
 *                        inc/hclib-async.h:125-134; the runtime frees it after
 *                        the task ran, src/hclib-runtime.c:477)
 *   hclib_loop_domain_t  :53-58 (16 bytes, int32 bounds)
 *   loop_dist_func       :71-72
 *   get/set_current_finish :100-106
 * A task whose _fp is a registered device task kind runs on the GPU locale
 * (hclib.h, hclib_hip_register_async_kind); every other task on the host.
 */
#ifndef HCLIB_TASK_H_
#define HCLIB_TASK_H_

#include "hclib-locality-graph.h"
#include "hclib-rt.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MAX_HCLIB_ASYNC_ARG_SIZE (sizeof(void *) + sizeof(void *))

typedef struct hclib_task_t {
    generic_frame_ptr _fp;
    void *args;
    struct finish_t *current_finish;
    hclib_future_t *waiting_on[MAX_NUM_WAITS];
    hclib_future_t **waiting_on_extra; /* NULL-terminated futures past MAX_NUM_WAITS */
    int waiting_on_index;
    hclib_locale_t *locale;
    int non_blocking;
    struct hclib_task_t *next_waiter;
} hclib_task_t;

typedef struct {
    int low;
    int high;
    int stride;
    int tile;
} hclib_loop_domain_t;

typedef hclib_locale_t *(*loop_dist_func)(const int, const hclib_loop_domain_t *, const hclib_loop_domain_t *,
                                          const int);

static inline struct finish_t *get_current_finish(hclib_task_t *t) { return t->current_finish; }
static inline void set_current_finish(hclib_task_t *t, struct finish_t *finish) { t->current_finish = finish; }

#ifdef __cplusplus
}
#endif

#endif
