/* Host-task promise semantics through include/hclib.h (no GPU needed).
 * Restates test/c/promise/asyncAwait1.c (a chain of n asyncs, each awaiting
 * promise i-1 and putting promise i, released by one put of promise 0),
 * test/c/promise/future0.c (a chain of hclib_async_future) and
 * test/c/finish1.c-style nested finish counting. Prints "Check results: OK". */
#include <assert.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include "hclib.h"

static int order[64];
static int norder = 0;

static void await_fct(void *raw) {
    void **argv = (void **)raw;
    int index = *((int *)argv[0]);
    hclib_future_t *f = (hclib_future_t *)argv[1];
    hclib_promise_t *out = (hclib_promise_t *)argv[2];
    int prev = *((int *)hclib_future_get(f));
    assert(prev == index - 1);
    order[norder++] = index;
    int *v = (int *)malloc(sizeof(int));
    *v = index;
    hclib_promise_put(out, v);
}

static void *future_fct(void *arg) {
    long v = (long)arg;
    return (void *)(v + 1);
}

static int counter = 0;
static void leaf(void *arg) { (void)arg; counter++; }
static void spawner(void *arg) {
    int n = *(int *)arg;
    hclib_start_finish();
    for (int i = 0; i < n; i++) hclib_async(leaf, NULL, NULL, 0, NULL);
    hclib_end_finish();
    assert(counter == n);
}

static void info_fct(void *arg) {
    void (*fp)(void *) = NULL;
    void *a = NULL;
    hclib_get_curr_task_info(&fp, &a);
    assert(fp == info_fct && a == arg);
    counter++;
}
static hclib_locale_t *my_dist(const int dim, const hclib_loop_domain_t *sub, const hclib_loop_domain_t *all,
                               const int mode) {
    (void)dim; (void)sub; (void)all; (void)mode;
    return hclib_get_master_place();
}
static void on_main(void *arg) { *(int *)arg = 42; }

static void entrypoint(void *arg) {
    (void)arg;
    int n = 5;
    hclib_promise_t **p = (hclib_promise_t **)malloc(sizeof(hclib_promise_t *) * (n + 1));
    hclib_start_finish();
    for (int i = 0; i <= n; i++) p[i] = hclib_promise_create();
    for (int i = n; i >= 1; i--) {
        void **argv = (void **)malloc(sizeof(void *) * 3);
        argv[0] = malloc(sizeof(int));
        *((int *)argv[0]) = i;
        argv[1] = hclib_get_future_for_promise(p[i - 1]);
        argv[2] = p[i];
        hclib_future_t *fut = hclib_get_future_for_promise(p[i - 1]);
        hclib_async(await_fct, argv, &fut, 1, NULL);
    }
    int *zero = (int *)malloc(sizeof(int));
    *zero = 0;
    hclib_promise_put(p[0], zero);
    hclib_end_finish();
    for (int i = 0; i < n; i++) assert(order[i] == i + 1);
    assert(*(int *)hclib_future_get(hclib_get_future_for_promise(p[n])) == n);

    /* chain of async_future, each depending on the previous */
    hclib_future_t *f = hclib_async_future(future_fct, (void *)0L, NULL, 0, NULL);
    for (int i = 0; i < 9; i++) {
        long prev = (long)hclib_future_wait(f);
        f = hclib_async_future(future_fct, (void *)prev, &f, 1, NULL);
    }
    assert((long)hclib_future_wait(f) == 10);

    /* nested finish scopes + nonblocking end_finish */
    int k = 7;
    hclib_start_finish();
    hclib_async(spawner, &k, NULL, 0, NULL);
    hclib_end_finish();
    hclib_start_finish();
    hclib_async(leaf, NULL, NULL, 0, NULL);
    hclib_future_t *done = hclib_end_finish_nonblocking();
    hclib_future_wait(done);
    assert(counter == k + 1);

    /* backlog (src/hclib-runtime.c:1365-1368): queued, not yet run tasks on
     * this worker; the awaiting task is not queued until its future is put */
    hclib_promise_t *gate = hclib_promise_create();
    hclib_future_t *gf = hclib_get_future_for_promise(gate);
    size_t before = hclib_current_worker_backlog();
    hclib_start_finish();
    hclib_async(leaf, NULL, NULL, 0, NULL);
    hclib_async(leaf, NULL, NULL, 0, NULL);
    hclib_async(leaf, NULL, &gf, 1, NULL);
    assert(hclib_current_worker_backlog() == before + 2);
    hclib_promise_put(gate, NULL);
    assert(hclib_current_worker_backlog() == before + 3);
    hclib_end_finish();
    assert(hclib_current_worker_backlog() == before);
    assert(counter == k + 4);

    /* task info, queue capacity, main context, locality queries, loop
     * distribution functions (inc/hclib.h:87-95, 253-262) */
    static int token;
    hclib_start_finish();
    hclib_async(info_fct, &token, NULL, 0, NULL);
    int used = -1, cap = -1;
    hclib_default_queue_capacity(&used, &cap);
    assert(used == (int)hclib_current_worker_backlog() && used >= 1 && cap == 1 << 20);
    hclib_end_finish();
    assert(counter == k + 5);
    int flag = 0;
    hclib_run_on_main_ctx(on_main, &flag);
    assert(flag == 42);
    hclib_locale_t *central = hclib_get_central_place();
    assert(central == hclib_get_master_place() && central == hclib_get_closest_locale());
    assert(hclib_get_closest_locale_of_type(central, hclib_get_locale_type(central)) == central);
    int types[2] = {12345, hclib_get_locale_type(central)};
    assert(hclib_get_closest_locale_of_types(central, types, 2) == central);
    assert(hclib_get_closest_locale_of_type(central, 12345) == NULL);
    hclib_locale_t **priv = hclib_get_thread_private_locales();
    assert(priv[0] == central);
    free(priv);
    hclib_locale_t fresh;
    memset(&fresh, 0, sizeof(fresh));
    hclib_locale_mark_special(&fresh, "COMM");
    hclib_locale_mark_special(&fresh, "COMM");  /* same type again: allowed */
    assert(strcmp(fresh.special_type, "COMM") == 0);
    assert(hclib_lookup_dist_func(HCLIB_DEFAULT_LOOP_DIST)(1, NULL, NULL, 0) == central);
    unsigned id = hclib_register_dist_func(my_dist);
    assert(id >= 1 && hclib_lookup_dist_func(id) == my_dist);

    /* a NULL inline future is skipped, not a terminator
     * (src/hclib-promise.c:171-180): futures {f0, NULL, f2, f3, f4} — the
     * task waits for every non-NULL one, including the extra f4 */
    {
        hclib_promise_t *q[5];
        hclib_future_t *fs[5];
        for (int i = 0; i < 5; i++) {
            q[i] = hclib_promise_create();
            fs[i] = hclib_get_future_for_promise(q[i]);
        }
        fs[1] = NULL;
        const int c0 = counter;
        hclib_start_finish();
        hclib_async(leaf, NULL, fs, 5, NULL);
        hclib_promise_put(q[0], NULL);
        hclib_yield(NULL);
        assert(counter == c0);
        hclib_promise_put(q[2], NULL);
        hclib_promise_put(q[3], NULL);
        hclib_yield(NULL);
        assert(counter == c0); /* still waiting on the extra future f4 */
        hclib_promise_put(q[4], NULL);
        hclib_end_finish();
        assert(counter == c0 + 1);
    }
}

int main(void) {
    const char *deps[] = {"system"};
    hclib_launch(entrypoint, NULL, deps, 1);
    printf("Check results: OK\n");
    return 0;
}
