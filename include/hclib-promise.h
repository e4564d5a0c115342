/*
 * hclib-promise.h — promises and futures of the HClib C API (MI355X build).
 *
 * Same types, layouts and prototypes as the reference's inc/hclib-promise.h:
 *   MAX_NUM_WAITS                    inc/hclib-promise.h:62
 *   hclib_future_t / hclib_promise_t inc/hclib-promise.h:65-90 (the future at
 *                                    offset 0: test/fib/fib.c:108-110 casts)
 *   hclib_promise_* / hclib_future_* inc/hclib-promise.h:96-156
 * Host promises live in host memory; device promises are the megakernel's
 * dependency counters (include/hclib_hip/hx_dag.h).
 */
#ifndef HCLIB_PROMISE_H_
#define HCLIB_PROMISE_H_

#include <stdlib.h>

#define MAX_NUM_WAITS 4

#ifdef __cplusplus
extern "C" {
#endif

struct hclib_promise_st;

typedef struct _hclib_future_t {
    struct hclib_promise_st *owner;
} hclib_future_t;

struct hclib_task_t;
typedef struct hclib_promise_st {
    hclib_future_t future;
    volatile int satisfied;
    void *volatile datum;
    struct hclib_task_t *volatile wait_list_head;
} hclib_promise_t;

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

#ifdef __cplusplus
}
#endif

#endif /* HCLIB_PROMISE_H_ */
