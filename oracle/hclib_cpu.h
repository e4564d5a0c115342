/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
 *
 * hclib_cpu: a from-scratch C restatement of HClib's CPU work-stealing
 * scheduler (the thing the MI355X megakernel replaces), used as
 *   (1) the CPU baseline that bench.py times on the GPU box's host cores
 *       ("cpu_baseline.kind": "port"), and
 *   (2) a semantic cross-check of the async/finish/promise/forasync rules.
 * Names carry an `ohc_` prefix so they can never be confused with (or bind
 * to) the product's hclib_* symbols.
 *
 * Algorithm followed (reference file:line):
 *   - per-worker bounded THE deque, owner push/pop at the tail, thieves CAS
 *     the head, steal chunk 1 ............ src/hclib-deque.c:50-139
 *   - victim scan 0..N-1 (no hwloc) ...... src/hclib-locality-graph.c:843-888
 *   - finish = counter starting at 1, help-first end_finish that runs every
 *     found task inline ("work-shift") ... src/hclib-runtime.c:431-446,
 *                                          1067-1119, 1219-1277
 *   - promises with a lock-free waiter list, chained registration over a
 *     task's futures ...................... src/hclib-promise.c:132-245
 *   - forasync FLAT / RECURSIVE lowering .. src/hclib.c:110-473
 */
#ifndef HCLIB_ORACLE_CPU_H
#define HCLIB_ORACLE_CPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void (*ohc_fn_t)(void *);

typedef struct ohc_promise ohc_promise_t;
typedef struct {
    ohc_promise_t *owner;
} ohc_future_t;

struct ohc_task;
struct ohc_promise {
    ohc_future_t future; /* offset 0, as inc/hclib-promise.h:69-70 */
    volatile int satisfied;
    void *volatile datum;
    struct ohc_task *volatile wait_list_head;
};

typedef struct {
    int low, high, stride, tile;
} ohc_loop_domain_t;

#define OHC_MAX_NUM_WAITS 4

/* Runs fn(arg) as the root task inside a root finish on `nworkers` workers
 * (worker 0 = the calling thread), then joins (hclib_launch,
 * src/hclib-runtime.c:1460-1478). */
void ohc_launch(int nworkers, ohc_fn_t fn, void *arg);

void ohc_async(ohc_fn_t fn, void *arg, ohc_future_t **futures, int nfutures);
void ohc_start_finish(void);
void ohc_end_finish(void);
int ohc_num_workers(void);
int ohc_current_worker(void);

void ohc_promise_init(ohc_promise_t *p);
ohc_promise_t *ohc_promise_create(void);
void ohc_promise_free(ohc_promise_t *p);
void ohc_promise_put(ohc_promise_t *p, void *datum);
void *ohc_future_get(ohc_future_t *f);
void *ohc_future_wait(ohc_future_t *f);

typedef void (*ohc_forasync1d_fn_t)(void *arg, int i);
void ohc_forasync1d(ohc_forasync1d_fn_t fn, void *arg, ohc_loop_domain_t *dom, int mode);

/* Scheduler statistics since the last launch (HCLIB_STATS analogue,
 * src/hclib-runtime.c:83-104). */
typedef struct {
    uint64_t executed_tasks;
    uint64_t steals;
    uint64_t end_finishes;
} ohc_stats_t;
void ohc_get_stats(ohc_stats_t *out);

/* ---- workloads (hclib_cpu_workloads.c) ---- */
double ohc_now(void);
long ohc_fib(int nworkers, int n, int ddt, double *seconds);
int ohc_uts(int nworkers, const void *params /* ora_uts_params_t */, uint64_t *nodes,
            uint64_t *leaves, uint64_t *max_depth, double *seconds);
int ohc_sw(int nworkers, const signed char *s1, size_t n1, const signed char *s2, size_t n2,
           int tw, int th, double *seconds);
void ohc_triad(int nworkers, float *a, const float *b, const float *c, float s, int n, int tile,
               int mode, double *seconds);

#ifdef __cplusplus
}
#endif
#endif
