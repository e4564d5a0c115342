/*
 * spawn_api.c — the task-record and plug-in boundary of the C ABI.
 *
 * Drives what the reference's header-only C++ layer and its modules bind
 * (SURVEY §8b):
 *   spawn / spawn_at / spawn_await / spawn_await_at  inc/hclib-async-struct.h:49-54
 *     with a caller-built hclib_task_t (inc/hclib-task.h:32-44, 96 bytes),
 *     as inc/hclib-async.h:125-134 builds it, including more than
 *     MAX_NUM_WAITS futures (the NULL-terminated waiting_on_extra of
 *     src/hclib-runtime.c:589-610);
 *   current_ws() / hclib_get_current_worker          inc/hclib-rt.h:140-143
 *   HCLIB_REGISTER_MODULE pre/post/finalize order,
 *   per-worker module state, locale metadata         inc/hclib-module.h:62-106
 *   hclib_get_curr_task_info from the entrypoint     src/hclib.c:475-480
 * and asserts like the reference's test programs ("Check results: OK").
 */
#include <assert.h>
#include <stdio.h>
#include <string.h>

#include "hclib.h"

#define N_FUT 7 /* > MAX_NUM_WAITS: three futures go to waiting_on_extra */

static int order[64];
static int norder = 0;
static int module_calls[3];
static unsigned state_id;
static int metadata_populated = 0;

typedef struct {
    int magic;
    int tid;
} my_state_t;

static size_t meta_size(void) { return sizeof(long); }
static void meta_populate(hclib_locale_t *l) {
    *(long *)l->metadata = 1000 + l->id;
    metadata_populated++;
}
static void state_adder(void *state, void *user, int tid) {
    my_state_t *s = (my_state_t *)state;
    s->magic = *(int *)user;
    s->tid = tid;
}
static void state_releaser(void *state, void *user) {
    (void)user;
    ((my_state_t *)state)->magic = -1;
}

static void my_pre(void) {
    module_calls[0]++;
    assert(module_calls[1] == 0);
    /* register metadata on system-memory locales before the graph is built */
    hclib_add_locale_metadata_functions(hclib_add_known_locale_type("sysmem"), meta_size, meta_populate);
}
static void my_post(void) {
    module_calls[1]++;
    assert(module_calls[0] == 1);
    static int magic = 4242;
    state_id = hclib_add_per_worker_module_state(sizeof(my_state_t), state_adder, &magic);
}
static void my_fin(void) {
    module_calls[2]++;
    hclib_release_per_worker_module_state(state_id, state_releaser, NULL);
}
HCLIB_REGISTER_MODULE("spawn_api_test", my_pre, my_post, my_fin)

static void record(void *arg) { order[norder++] = (int)(long)arg; }

static hclib_task_t *make_task(generic_frame_ptr fp, void *arg) {
    hclib_task_t *t = (hclib_task_t *)calloc(1, sizeof(hclib_task_t));
    t->_fp = fp;
    t->args = arg;
    return t;
}

typedef struct {
    hclib_promise_t *p[N_FUT];
    int ran;
} gate_t;

static void gated(void *arg) {
    gate_t *g = (gate_t *)arg;
    for (int i = 0; i < N_FUT; i++) assert(hclib_future_is_satisfied(hclib_get_future_for_promise(g->p[i])));
    g->ran = 1;
    record((void *)99);
}

static void putter(void *arg) {
    hclib_promise_t *p = (hclib_promise_t *)arg;
    hclib_promise_put(p, p);
}

static void entrypoint(void *arg) {
    /* the root task reports the user's function and argument */
    void (*fp)(void *) = NULL;
    void *a = NULL;
    hclib_get_curr_task_info(&fp, &a);
    assert(fp == entrypoint && a == arg);

    /* worker state: the host control thread is worker 0 of 1 */
    hclib_worker_state *ws = current_ws();
    assert(ws && ws->id == 0 && ws->nworkers == 1);
    assert(hclib_get_current_worker() == 0 && hclib_get_num_workers() == 1);
    assert(ws == CURRENT_WS_INTERNAL);
    my_state_t *st = (my_state_t *)hclib_get_curr_worker_module_state(state_id);
    assert(st->magic == 4242 && st->tid == 0);

    /* locale metadata ran for system memory */
    hclib_locale_t *sys = hclib_get_central_place();
    assert(sys && strcmp(sys->lbl, "sysmem") == 0);
    assert(metadata_populated >= 1 && sys->metadata && *(long *)sys->metadata == 1000 + sys->id);

    /* spawn / spawn_at: tasks run when the finish ends, newest first (the
     * owner end of the deque) */
    hclib_start_finish();
    spawn(make_task(record, (void *)1));
    spawn_at(make_task(record, (void *)2), hclib_get_closest_locale());
    hclib_end_finish();
    assert(norder == 2 && order[0] == 2 && order[1] == 1);

    /* spawn_await with 7 futures: the task parks on the first unsatisfied
     * one and re-registers on the next as each is put (src/hclib-promise.c:
     * 132-245), through the extras; it runs only after the last put */
    gate_t g;
    g.ran = 0;
    hclib_future_t *futs[N_FUT];
    for (int i = 0; i < N_FUT; i++) {
        g.p[i] = hclib_promise_create();
        futs[i] = hclib_get_future_for_promise(g.p[i]);
    }
    norder = 0;
    hclib_start_finish();
    hclib_task_t *t = make_task(gated, &g);
    spawn_await(t, futs, N_FUT);
    assert(t->waiting_on_extra && t->waiting_on_extra[N_FUT - MAX_NUM_WAITS] == NULL);
    size_t before = hclib_current_worker_backlog();
    /* put them in reverse order from tasks; the gated task must stay parked
     * until the final put */
    for (int i = N_FUT - 1; i >= 1; i--) {
        hclib_promise_put(g.p[i], g.p[i]);
        assert(!g.ran && hclib_current_worker_backlog() == before);
    }
    spawn_await_at(make_task(putter, g.p[0]), NULL, 0, hclib_get_closest_locale());
    hclib_end_finish();
    assert(g.ran == 1 && norder == 1 && order[0] == 99);
    for (int i = 0; i < N_FUT; i++) hclib_promise_free(g.p[i]);

    /* spawn_await_at on an already satisfied future runs at once */
    hclib_promise_t *done = hclib_promise_create();
    hclib_promise_put(done, NULL);
    hclib_future_t *df = hclib_get_future_for_promise(done);
    norder = 0;
    hclib_start_finish();
    spawn_await_at(make_task(record, (void *)7), &df, 1, hclib_get_closest_locale());
    hclib_end_finish();
    assert(norder == 1 && order[0] == 7);
    hclib_promise_free(done);
}

int main(int argc, char **argv) {
    (void)argc;
    (void)argv;
    assert(sizeof(hclib_task_t) == 96);
    assert(sizeof(hclib_worker_state) == 128);
    const char *deps[] = {"system"};
    int cookie = 5;
    hclib_launch(entrypoint, &cookie, deps, 1);
    assert(module_calls[0] == 1 && module_calls[1] == 1 && module_calls[2] == 1);
    printf("Check results: OK\n");
    return 0;
}
