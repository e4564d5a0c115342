/* The four host symbols the round-3 review found missing from the boundary:
 *   hclib_user_harness_timer       inc/hclib-rt.h:153, src/hclib-runtime.c:1319-1321
 *   locale_num_tasks               inc/hclib-locality-graph.h:102, src/hclib-locality-graph.c:760-768
 *   locale_register_idle_task      inc/hclib-locality-graph.h:105, src/hclib-locality-graph.c:807-813
 *   locale_run_idle_tasks          inc/hclib-locality-graph.h:104, src/hclib-locality-graph.c:815-827
 * Host-only (runs without a GPU): tasks are queued at a locale inside a
 * finish and counted before the finish runs them; idle functions registered
 * at the worker's steal-path locales run once per locale_run_idle_tasks, in
 * registration order; the harness timer shows up in the HCLIB_STATS report.
 */
#include <stdio.h>
#include <stdlib.h>

#include "hclib.h"

static int ran = 0;
static int order[8], norder = 0;

static void task(void *arg) { ran += *(int *)arg; }
static void idle_a(void) { order[norder++] = 1; }
static void idle_b(void) { order[norder++] = 2; }

static void body(void *arg) {
    (void)arg;
    hclib_locale_t *here = hclib_get_closest_locale();
    static int one = 1;
    int ok = 1;
    const unsigned before = locale_num_tasks(here);
    hclib_start_finish();
    for (int i = 0; i < 5; ++i) hclib_async(task, &one, NULL, 0, here);
    hclib_async(task, &one, NULL, 0, NULL); /* no locale: queued at the closest one */
    const unsigned queued = locale_num_tasks(here);
    if (queued != before + 6) {
        printf("locale_num_tasks: %u queued, expected %u\n", queued, before + 6);
        ok = 0;
    }
    hclib_end_finish();
    if (ran != 6 || locale_num_tasks(here) != before) {
        printf("tasks ran %d (expected 6), %u still queued\n", ran, locale_num_tasks(here));
        ok = 0;
    }

    hclib_worker_state *ws = current_ws();
    hclib_locale_t *first = ws->paths->steal_path->locales[0];
    locale_register_idle_task(first, idle_a);
    locale_register_idle_task(first, idle_b);
    locale_run_idle_tasks(ws);
    locale_run_idle_tasks(ws);
    if (norder != 4 || order[0] != 1 || order[1] != 2 || order[2] != 1 || order[3] != 2) {
        printf("idle functions ran %d times in the wrong order\n", norder);
        ok = 0;
    }
    hclib_user_harness_timer(1.25);
    printf("Check results: %s\n", ok ? "OK" : "FAILED");
    if (!ok) exit(1);
}

int main(void) {
    const char *deps[] = {"system"};
    hclib_launch(body, NULL, deps, 0);
    (void)deps;
    return 0;
}
