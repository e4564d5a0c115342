/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see hclib_cpu.h for the reference map).
 *
 * CPU work-stealing runtime restated from HClib's scheduler. It is written
 * from the reference's algorithm, not its code: one bounded THE deque per
 * worker, help-first finish, waiter-list promises, FLAT/RECURSIVE forasync.
 * The fiber machinery (src/inc/litectx.h) is not restated: the reference's
 * end_finish path runs every found task inline (help_finish passes
 * on_fresh_ctx=1, src/hclib-runtime.c:1087), which is what this does too.
 */
#define _GNU_SOURCE
#include "hclib_cpu.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define OHC_DEQUE_CAP (1 << 20) /* INIT_DEQUE_CAPACITY, src/inc/hclib-deque.h:51 */

typedef struct ohc_finish {
    struct ohc_finish *parent;
    volatile int counter;
    ohc_promise_t *finish_dep;
} ohc_finish_t;

typedef struct ohc_task {
    ohc_fn_t fp;
    void *args;
    ohc_finish_t *finish;
    ohc_future_t *waiting_on[OHC_MAX_NUM_WAITS];
    int waiting_on_index;
    struct ohc_task *next_waiter;
} ohc_task_t;

typedef struct {
    volatile int head;
    char pad0[60];
    volatile int tail;
    char pad1[60];
    ohc_task_t **data;
} ohc_deque_t;

typedef struct {
    ohc_deque_t dq;
    ohc_finish_t *current_finish;
    ohc_stats_t stats;
    char pad[64];
} ohc_worker_t;

#define SENTINEL ((ohc_task_t *)0x1)
#define SATISFIED ((ohc_task_t *)0x2)

static ohc_worker_t *g_workers;
static int g_nworkers;
static volatile int g_done;
static __thread int t_wid = -1;

static inline void mfence(void) { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
static inline int cas_int(volatile int *p, int old, int nw) {
    return __atomic_compare_exchange_n((int *)p, &old, nw, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
}

/* deque_push, src/hclib-deque.c:50-64 */
static int deque_push(ohc_deque_t *d, ohc_task_t *t) {
    int size = d->tail - d->head;
    if (size == OHC_DEQUE_CAP) return 0;
    d->data[d->tail % OHC_DEQUE_CAP] = t;
    mfence();
    d->tail++;
    return 1;
}

/* deque_steal, src/hclib-deque.c:75-106 (chunk 1) */
static ohc_task_t *deque_steal(ohc_deque_t *d) {
    int head = d->head;
    mfence();
    int tail = d->tail;
    if (tail - head <= 0) return NULL;
    ohc_task_t *t = d->data[head % OHC_DEQUE_CAP];
    if (cas_int(&d->head, head, head + 1)) return t;
    return NULL;
}

/* deque_pop, src/hclib-deque.c:111-139 */
static ohc_task_t *deque_pop(ohc_deque_t *d) {
    mfence();
    int tail = d->tail - 1;
    d->tail = tail;
    mfence();
    int head = d->head;
    int size = tail - head;
    if (size < 0) {
        d->tail = d->head;
        return NULL;
    }
    ohc_task_t *t = d->data[tail % OHC_DEQUE_CAP];
    if (size > 0) return t;
    if (!cas_int(&d->head, head, head + 1)) t = NULL;
    d->tail = d->head;
    return t;
}

static void check_in(ohc_finish_t *f) {
    if (f) __atomic_add_fetch(&f->counter, 1, __ATOMIC_SEQ_CST);
}

static void check_out(ohc_finish_t *f) {
    if (f) {
        int old = __atomic_fetch_sub(&f->counter, 1, __ATOMIC_SEQ_CST);
        if (old == 1 && f->finish_dep) ohc_promise_put(f->finish_dep, f);
    }
}

static void schedule(ohc_task_t *t) {
    if (!deque_push(&g_workers[t_wid].dq, t)) {
        fprintf(stderr, "ohc: deque full\n");
        abort();
    }
}

/* _register_if_promise_not_ready, src/hclib-promise.c:132-166 */
static int register_if_not_ready(ohc_task_t *t, ohc_future_t *f) {
    ohc_promise_t *p = f->owner;
    ohc_task_t *head = p->wait_list_head;
    while (head != SATISFIED) {
        t->next_waiter = head;
        if (__atomic_compare_exchange_n((ohc_task_t **)&p->wait_list_head, &head, t, 0,
                                        __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST))
            return 1;
    }
    return 0;
}

/* register_on_all_promise_dependencies, src/hclib-promise.c:171-195 */
static int register_all(ohc_task_t *t) {
    while (t->waiting_on_index < OHC_MAX_NUM_WAITS - 1) {
        t->waiting_on_index++;
        ohc_future_t *f = t->waiting_on[t->waiting_on_index];
        if (f && register_if_not_ready(t, f)) return 0;
    }
    return 1;
}

void ohc_promise_init(ohc_promise_t *p) {
    p->satisfied = 0;
    p->datum = NULL;
    p->wait_list_head = SENTINEL;
    p->future.owner = p;
}

ohc_promise_t *ohc_promise_create(void) {
    ohc_promise_t *p = (ohc_promise_t *)malloc(sizeof(*p));
    ohc_promise_init(p);
    return p;
}

void ohc_promise_free(ohc_promise_t *p) { free(p); }

/* hclib_promise_put, src/hclib-promise.c:203-245 */
void ohc_promise_put(ohc_promise_t *p, void *datum) {
    p->datum = datum;
    __atomic_store_n(&p->satisfied, 1, __ATOMIC_SEQ_CST);
    ohc_task_t *list = __atomic_exchange_n((ohc_task_t **)&p->wait_list_head, SATISFIED,
                                           __ATOMIC_SEQ_CST);
    while (list != SENTINEL) {
        ohc_task_t *next = list->next_waiter;
        if (register_all(list)) schedule(list);
        list = next;
    }
}

void *ohc_future_get(ohc_future_t *f) { return f->owner->datum; }

static void execute(ohc_task_t *t) {
    ohc_worker_t *w = &g_workers[t_wid];
    ohc_finish_t *saved = w->current_finish;
    w->current_finish = t->finish;
    w->stats.executed_tasks++;
    t->fp(t->args);
    check_out(t->finish);
    g_workers[t_wid].current_finish = saved;
    free(t);
}

/* find_and_run_task, src/hclib-runtime.c:646-694 (pop, else steal over
 * victims 0..N-1 as locale_steal_task does without hwloc). */
static int find_and_run(void) {
    ohc_task_t *t = deque_pop(&g_workers[t_wid].dq);
    if (!t) {
        for (int v = 0; v < g_nworkers && !t; v++) t = deque_steal(&g_workers[v].dq);
        if (t) g_workers[t_wid].stats.steals++;
    }
    if (!t) return 0;
    execute(t);
    return 1;
}

/* spawn_handler, src/hclib-runtime.c:572-617 */
void ohc_async(ohc_fn_t fn, void *arg, ohc_future_t **futures, int nfutures) {
    ohc_task_t *t = (ohc_task_t *)calloc(1, sizeof(*t));
    t->fp = fn;
    t->args = arg;
    ohc_finish_t *f = g_workers[t_wid].current_finish;
    check_in(f);
    t->finish = f;
    if (nfutures > OHC_MAX_NUM_WAITS) {
        fprintf(stderr, "ohc: too many futures\n");
        abort();
    }
    for (int i = 0; i < nfutures; i++) t->waiting_on[i] = futures[i];
    t->waiting_on_index = -1;
    if (nfutures == 0 || register_all(t)) schedule(t);
}

/* hclib_start_finish, src/hclib-runtime.c:1219-1247 */
void ohc_start_finish(void) {
    ohc_worker_t *w = &g_workers[t_wid];
    ohc_finish_t *f = (ohc_finish_t *)calloc(1, sizeof(*f));
    f->counter = 1;
    f->parent = w->current_finish;
    check_in(f->parent);
    w->current_finish = f;
}

/* hclib_end_finish + help_finish, src/hclib-runtime.c:1249-1277, 1067-1119 */
void ohc_end_finish(void) {
    ohc_finish_t *f = g_workers[t_wid].current_finish;
    g_workers[t_wid].stats.end_finishes++;
    while (__atomic_load_n(&f->counter, __ATOMIC_ACQUIRE) > 1) find_and_run();
    g_workers[t_wid].current_finish = f->parent;
    check_out(f->parent);
    free(f);
}

/* hclib_future_wait without fibers: help while waiting. */
void *ohc_future_wait(ohc_future_t *fut) {
    while (!__atomic_load_n(&fut->owner->satisfied, __ATOMIC_ACQUIRE)) find_and_run();
    return fut->owner->datum;
}

int ohc_num_workers(void) { return g_nworkers; }
int ohc_current_worker(void) { return t_wid; }

typedef struct {
    int wid;
} ohc_thread_arg_t;

/* core_work_loop, src/hclib-runtime.c:705-724 */
static void *worker_main(void *raw) {
    t_wid = ((ohc_thread_arg_t *)raw)->wid;
    while (!__atomic_load_n(&g_done, __ATOMIC_ACQUIRE)) find_and_run();
    return NULL;
}

void ohc_launch(int nworkers, ohc_fn_t fn, void *arg) {
    if (nworkers < 1) nworkers = 1;
    g_nworkers = nworkers;
    g_done = 0;
    g_workers = (ohc_worker_t *)calloc((size_t)nworkers, sizeof(ohc_worker_t));
    for (int i = 0; i < nworkers; i++)
        g_workers[i].dq.data = (ohc_task_t **)calloc(OHC_DEQUE_CAP, sizeof(ohc_task_t *));
    pthread_t *th = (pthread_t *)calloc((size_t)nworkers, sizeof(pthread_t));
    ohc_thread_arg_t *ta = (ohc_thread_arg_t *)calloc((size_t)nworkers, sizeof(*ta));
    t_wid = 0;
    for (int i = 1; i < nworkers; i++) {
        ta[i].wid = i;
        pthread_create(&th[i], NULL, worker_main, &ta[i]);
    }
    ohc_start_finish();
    fn(arg);
    ohc_end_finish();
    __atomic_store_n(&g_done, 1, __ATOMIC_RELEASE);
    for (int i = 1; i < nworkers; i++) pthread_join(th[i], NULL);
    free(th);
    free(ta);
    /* keep g_workers until the next launch so stats stay readable */
    for (int i = 0; i < nworkers; i++) free(g_workers[i].dq.data), g_workers[i].dq.data = NULL;
}

void ohc_get_stats(ohc_stats_t *out) {
    memset(out, 0, sizeof(*out));
    for (int i = 0; g_workers && i < g_nworkers; i++) {
        out->executed_tasks += g_workers[i].stats.executed_tasks;
        out->steals += g_workers[i].stats.steals;
        out->end_finishes += g_workers[i].stats.end_finishes;
    }
}

/* ---- forasync (src/hclib.c:110-473), 1-D ---- */
typedef struct {
    ohc_forasync1d_fn_t fn;
    void *arg;
    ohc_loop_domain_t loop;
} ohc_fa1d_t;

static void fa_runner(void *raw) {
    ohc_fa1d_t *f = (ohc_fa1d_t *)raw;
    for (int i = f->loop.low; i < f->loop.high; i += f->loop.stride) f->fn(f->arg, i);
}

static void fa_runner_free(void *raw) {
    fa_runner(raw);
    free(raw);
}

static void fa_recursive_free(void *raw);

static void fa_recursive(void *raw) {
    ohc_fa1d_t *f = (ohc_fa1d_t *)raw;
    while ((f->loop.high - f->loop.low) > f->loop.tile) {
        int mid = (f->loop.high + f->loop.low) / 2;
        ohc_fa1d_t *up = (ohc_fa1d_t *)malloc(sizeof(*up));
        *up = *f;
        up->loop.low = mid;
        ohc_async(fa_recursive_free, up, NULL, 0);
        f->loop.high = mid;
    }
    fa_runner(f);
}

static void fa_recursive_free(void *raw) {
    fa_recursive(raw);
    free(raw);
}

void ohc_forasync1d(ohc_forasync1d_fn_t fn, void *arg, ohc_loop_domain_t *dom, int mode) {
    if (dom->tile == -1) dom->tile = ((dom->high - dom->low) + g_nworkers - 1) / g_nworkers;
    ohc_loop_domain_t l = *dom;
    if (mode == 1) {
        ohc_fa1d_t *f = (ohc_fa1d_t *)malloc(sizeof(*f));
        f->fn = fn;
        f->arg = arg;
        f->loop = l;
        /* forasync_internal calls the recursive lowering inline */
        fa_recursive_free(f);
        return;
    }
    int nb_chunks = l.high / l.tile;
    int size = l.tile * nb_chunks;
    int low0;
    for (low0 = l.low; low0 < size; low0 += l.tile) {
        ohc_fa1d_t *f = (ohc_fa1d_t *)malloc(sizeof(*f));
        f->fn = fn;
        f->arg = arg;
        f->loop.low = low0;
        f->loop.high = low0 + l.tile;
        f->loop.stride = l.stride;
        f->loop.tile = l.tile;
        ohc_async(fa_runner_free, f, NULL, 0);
    }
    if (size < l.high) {
        ohc_fa1d_t *f = (ohc_fa1d_t *)malloc(sizeof(*f));
        f->fn = fn;
        f->arg = arg;
        f->loop.low = low0;
        f->loop.high = l.high;
        f->loop.stride = l.stride;
        f->loop.tile = l.tile;
        ohc_async(fa_runner_free, f, NULL, 0);
    }
}
