/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * The reference's workload drivers restated on the hclib_cpu runtime:
 *   fib ........ test/fib/fib.c:57-71 (async/finish), 113-141 (DDT), 151-186
 *   UTS ........ test/uts/UTS.cpp:85-252, 383-402 (per-worker steal stacks,
 *                20-node chunk release as asyncs, work-first DFS)
 *   SW ......... test/smithwaterman/smith_waterman.cpp:119-239 (3-future tiles)
 *   triad ...... hclib_forasync 1-D over a[i] = b[i] + s*c[i]
 * Each returns the parallel-region wall time the reference drivers print.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hclib_cpu.h"
#include "uts_oracle.h"

double ohc_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ------------------------------- fib ---------------------------------- */
typedef struct {
    int n;
    long res;
} fib_args_t;

static void fib_task(void *raw) {
    fib_args_t *a = (fib_args_t *)raw;
    if (a->n < 2) {
        a->res = a->n;
        return;
    }
    fib_args_t l = {a->n - 1, 0}, r = {a->n - 2, 0};
    ohc_start_finish();
    ohc_async(fib_task, &l, NULL, 0);
    ohc_async(fib_task, &r, NULL, 0);
    ohc_end_finish();
    a->res = l.res + r.res;
}

typedef struct fib_ddt {
    int n;
    long resval;
    ohc_promise_t *res;
    ohc_promise_t *subres[3];
} fib_ddt_t;

static fib_ddt_t *ddt_new(int n) {
    fib_ddt_t *a = (fib_ddt_t *)malloc(sizeof(*a));
    a->n = n;
    a->res = ohc_promise_create();
    a->subres[2] = NULL;
    return a;
}

static void fib_ddt_res(void *raw) {
    fib_ddt_t *a = (fib_ddt_t *)raw;
    fib_ddt_t *l = (fib_ddt_t *)ohc_future_get(&a->subres[0]->future);
    fib_ddt_t *r = (fib_ddt_t *)ohc_future_get(&a->subres[1]->future);
    a->resval = l->resval + r->resval;
    ohc_promise_put(a->res, a);
    ohc_promise_free(l->res);
    free(l);
    ohc_promise_free(r->res);
    free(r);
}

static void fib_ddt_task(void *raw) {
    fib_ddt_t *a = (fib_ddt_t *)raw;
    if (a->n < 2) {
        a->resval = a->n;
        ohc_promise_put(a->res, a);
        return;
    }
    fib_ddt_t *l = ddt_new(a->n - 1), *r = ddt_new(a->n - 2);
    a->subres[0] = l->res;
    a->subres[1] = r->res;
    ohc_async(fib_ddt_task, l, NULL, 0);
    ohc_async(fib_ddt_task, r, NULL, 0);
    ohc_future_t *f[2] = {&a->subres[0]->future, &a->subres[1]->future};
    ohc_async(fib_ddt_res, a, f, 2);
}

static void fib_noop(void *raw) { (void)raw; }

typedef struct {
    int n, ddt;
    long answer;
    double secs;
} fib_main_t;

static void fib_main(void *raw) {
    fib_main_t *m = (fib_main_t *)raw;
    double t0 = ohc_now();
    if (!m->ddt) {
        fib_args_t a = {m->n, 0};
        ohc_start_finish();
        ohc_async(fib_task, &a, NULL, 0);
        ohc_end_finish();
        m->answer = a.res;
    } else {
        fib_ddt_t *a = ddt_new(m->n);
        ohc_start_finish();
        ohc_async(fib_ddt_task, a, NULL, 0);
        ohc_future_t *f = &a->res->future;
        ohc_async(fib_noop, a, &f, 1);
        ohc_end_finish();
        m->answer = a->resval;
        ohc_promise_free(a->res);
        free(a);
    }
    m->secs = ohc_now() - t0;
}

long ohc_fib(int nworkers, int n, int ddt, double *seconds) {
    fib_main_t m = {n, ddt, 0, 0};
    ohc_launch(nworkers, fib_main, &m);
    if (seconds) *seconds = m.secs;
    return m.answer;
}

/* ------------------------------- UTS ---------------------------------- */
#define UTS_CHUNK 20            /* chunkSize, UTS.cpp:44 */
#define UTS_MAXSTACK 1048576    /* MAXSTACKDEPTH, UTS.cpp:41 */

typedef struct {
    uint32_t st[5];
    int height;
    int type;
} uts_node_t;

typedef struct {
    long local_work;
    uint64_t nodes, leaves, max_depth;
    uts_node_t *stack;
    int head, tail;
    char pad[64];
} uts_ss_t;

static uts_ss_t *g_ss;
static const ora_uts_params_t *g_up;

static void uts_par_search(void);

/* push_surplusNodes, UTS.cpp:137-146 */
static void uts_chunk_task(void *raw) {
    uts_ss_t *ss = &g_ss[ohc_current_worker()];
    ss->local_work = UTS_CHUNK;
    ss->head = UTS_CHUNK;
    ss->tail = 0;
    memcpy(ss->stack, raw, sizeof(uts_node_t) * UTS_CHUNK);
    free(raw);
    uts_par_search();
}

/* genChildren, UTS.cpp:154-210 */
static void uts_gen_children(uts_node_t *parent, uts_ss_t *ss) {
    if ((uint64_t)parent->height > ss->max_depth) ss->max_depth = parent->height;
    int nc = ora_uts_num_children(g_up, parent->type, parent->height, parent->st);
    int ct = ora_uts_child_type(g_up, parent->height);
    if (nc > 0) {
        if (nc + ss->head - ss->tail >= UTS_MAXSTACK) {
            fprintf(stderr, "ohc uts: worker stack out of memory\n");
            exit(10);
        }
        for (int i = 0; i < nc; i++) {
            uts_node_t *child = &ss->stack[ss->head++];
            child->type = ct;
            child->height = parent->height + 1;
            for (int g = 0; g < g_up->compute_gran; g++) ora_rng_spawn(parent->st, child->st, i);
            ss->local_work++;
            if (ss->local_work > 2 * UTS_CHUNK) {
                uts_node_t *work = (uts_node_t *)malloc(sizeof(uts_node_t) * UTS_CHUNK);
                memcpy(work, &ss->stack[ss->tail], sizeof(uts_node_t) * UTS_CHUNK);
                ss->tail += UTS_CHUNK;
                ss->local_work -= UTS_CHUNK;
                ohc_async(uts_chunk_task, work, NULL, 0);
            }
        }
    } else {
        ss->leaves++;
    }
}

/* parTreeSearch + ss_get_work, UTS.cpp:219-232, 383-402 */
static void uts_par_search(void) {
    uts_ss_t *ss = &g_ss[ohc_current_worker()];
    while (ss->local_work != 0) {
        ss->head--;
        uts_node_t parent = ss->stack[ss->head];
        ss->local_work--;
        ss->nodes++;
        uts_gen_children(&parent, ss);
        ss = &g_ss[ohc_current_worker()];
    }
}

static void uts_root_task(void *raw) {
    (void)raw;
    uts_ss_t *ss = &g_ss[ohc_current_worker()];
    uts_node_t *root = &ss->stack[ss->head];
    root->type = g_up->type;
    root->height = 0;
    ora_rng_init(root->st, g_up->root_id);
    ss->head++;
    ss->local_work++;
    uts_par_search();
}

typedef struct {
    double secs;
} uts_main_t;

static void uts_main(void *raw) {
    uts_main_t *m = (uts_main_t *)raw;
    double t0 = ohc_now();
    ohc_start_finish();
    ohc_async(uts_root_task, NULL, NULL, 0);
    ohc_end_finish();
    m->secs = ohc_now() - t0;
}

int ohc_uts(int nworkers, const void *params, uint64_t *nodes, uint64_t *leaves,
            uint64_t *max_depth, double *seconds) {
    if (nworkers < 1) nworkers = 1;
    g_up = (const ora_uts_params_t *)params;
    g_ss = (uts_ss_t *)calloc((size_t)nworkers, sizeof(uts_ss_t));
    for (int i = 0; i < nworkers; i++) {
        g_ss[i].stack = (uts_node_t *)malloc(sizeof(uts_node_t) * UTS_MAXSTACK);
        if (!g_ss[i].stack) return -1;
    }
    uts_main_t m = {0};
    ohc_launch(nworkers, uts_main, &m);
    uint64_t n = 0, l = 0, d = 0;
    for (int i = 0; i < nworkers; i++) {
        n += g_ss[i].nodes;
        l += g_ss[i].leaves;
        if (g_ss[i].max_depth > d) d = g_ss[i].max_depth;
        free(g_ss[i].stack);
    }
    free(g_ss);
    g_ss = NULL;
    *nodes = n;
    *leaves = l;
    *max_depth = d;
    if (seconds) *seconds = m.secs;
    return 0;
}

/* ---------------------------- Smith-Waterman --------------------------- */
static const signed char sw_m[5][5] = {
    {-1, -1, -1, -1, -1}, {-1, 2, -4, -2, -4}, {-1, -4, 2, -4, -2},
    {-1, -2, -4, 2, -4}, {-1, -4, -2, -4, 2},
};

typedef struct {
    ohc_promise_t bottom_row, right_column, bottom_right;
} sw_tile_t;

typedef struct {
    sw_tile_t *tiles;
    int ntw, nth, tw, th;
    const signed char *s1, *s2;
} sw_ctx_t;

typedef struct {
    sw_ctx_t *ctx;
    int i, j;
} sw_task_t;

#define TILE(c, i, j) (&(c)->tiles[(size_t)(i) * ((c)->ntw + 1) + (j)])

/* the async_await body, smith_waterman.cpp:174-229 */
static void sw_tile_task(void *raw) {
    sw_task_t *t = (sw_task_t *)raw;
    sw_ctx_t *c = t->ctx;
    int i = t->i, j = t->j, tw = c->tw, th = c->th;
    int *above = (int *)ohc_future_get(&TILE(c, i - 1, j)->bottom_row.future);
    int *left = (int *)ohc_future_get(&TILE(c, i, j - 1)->right_column.future);
    int *diag = (int *)ohc_future_get(&TILE(c, i - 1, j - 1)->bottom_right.future);
    int W = tw + 1;
    int *cur = (int *)malloc(sizeof(int) * (size_t)(tw + 1) * (th + 1));
    cur[0] = diag[0];
    for (int r = 1; r <= th; r++) cur[r * W] = left[r - 1];
    for (int q = 1; q <= tw; q++) cur[q] = above[q - 1];
    for (int r = 1; r <= th; r++) {
        signed char c2 = c->s2[(size_t)(i - 1) * th + (r - 1)];
        for (int q = 1; q <= tw; q++) {
            signed char c1 = c->s1[(size_t)(j - 1) * tw + (q - 1)];
            int d = cur[(r - 1) * W + q - 1] + sw_m[c2][c1];
            int l = cur[r * W + q - 1] + sw_m[c1][0];
            int u = cur[(r - 1) * W + q] + sw_m[0][c2];
            int lt = (l > u) ? l : u;
            cur[r * W + q] = (lt > d) ? lt : d;
        }
    }
    int *br = (int *)malloc(sizeof(int));
    br[0] = cur[th * W + tw];
    ohc_promise_put(&TILE(c, i, j)->bottom_right, br);
    int *rc = (int *)malloc(sizeof(int) * th);
    for (int r = 0; r < th; r++) rc[r] = cur[(r + 1) * W + tw];
    ohc_promise_put(&TILE(c, i, j)->right_column, rc);
    int *brow = (int *)malloc(sizeof(int) * tw);
    for (int q = 0; q < tw; q++) brow[q] = cur[th * W + q + 1];
    ohc_promise_put(&TILE(c, i, j)->bottom_row, brow);
    free(cur);
    free(t);
}

typedef struct {
    sw_ctx_t *ctx;
    double secs;
} sw_main_t;

static void sw_main(void *raw) {
    sw_main_t *m = (sw_main_t *)raw;
    sw_ctx_t *c = m->ctx;
    double t0 = ohc_now();
    ohc_start_finish();
    for (int i = 1; i <= c->nth; i++) {
        for (int j = 1; j <= c->ntw; j++) {
            sw_task_t *t = (sw_task_t *)malloc(sizeof(*t));
            t->ctx = c;
            t->i = i;
            t->j = j;
            ohc_future_t *f[3] = {&TILE(c, i, j - 1)->right_column.future,
                                  &TILE(c, i - 1, j)->bottom_row.future,
                                  &TILE(c, i - 1, j - 1)->bottom_right.future};
            ohc_async(sw_tile_task, t, f, 3);
        }
    }
    ohc_end_finish();
    m->secs = ohc_now() - t0;
}

int ohc_sw(int nworkers, const signed char *s1, size_t n1, const signed char *s2, size_t n2,
           int tw, int th, double *seconds) {
    sw_ctx_t c;
    c.ntw = (int)(n1 / (size_t)tw);
    c.nth = (int)(n2 / (size_t)th);
    c.tw = tw;
    c.th = th;
    c.s1 = s1;
    c.s2 = s2;
    size_t nt = (size_t)(c.nth + 1) * (c.ntw + 1);
    c.tiles = (sw_tile_t *)calloc(nt, sizeof(sw_tile_t));
    for (size_t k = 0; k < nt; k++) {
        ohc_promise_init(&c.tiles[k].bottom_row);
        ohc_promise_init(&c.tiles[k].right_column);
        ohc_promise_init(&c.tiles[k].bottom_right);
    }
    /* boundary puts, smith_waterman.cpp:141-165 (before launch: no waiters) */
    int *a = (int *)malloc(sizeof(int));
    a[0] = 0;
    TILE(&c, 0, 0)->bottom_right.datum = a;
    TILE(&c, 0, 0)->bottom_right.satisfied = 1;
    TILE(&c, 0, 0)->bottom_right.wait_list_head = (void *)0x2;
    for (int j = 1; j <= c.ntw; j++) {
        int *row = (int *)malloc(sizeof(int) * tw);
        for (int q = 0; q < tw; q++) row[q] = -((j - 1) * tw + q + 1);
        ohc_promise_t *p = &TILE(&c, 0, j)->bottom_row;
        p->datum = row, p->satisfied = 1, p->wait_list_head = (void *)0x2;
        int *br = (int *)malloc(sizeof(int));
        br[0] = -(j * tw);
        p = &TILE(&c, 0, j)->bottom_right;
        p->datum = br, p->satisfied = 1, p->wait_list_head = (void *)0x2;
    }
    for (int i = 1; i <= c.nth; i++) {
        int *col = (int *)malloc(sizeof(int) * th);
        for (int r = 0; r < th; r++) col[r] = -((i - 1) * th + r + 1);
        ohc_promise_t *p = &TILE(&c, i, 0)->right_column;
        p->datum = col, p->satisfied = 1, p->wait_list_head = (void *)0x2;
        int *br = (int *)malloc(sizeof(int));
        br[0] = -(i * th);
        p = &TILE(&c, i, 0)->bottom_right;
        p->datum = br, p->satisfied = 1, p->wait_list_head = (void *)0x2;
    }
    sw_main_t m = {&c, 0};
    ohc_launch(nworkers, sw_main, &m);
    int score = ((int *)TILE(&c, c.nth, c.ntw)->bottom_row.datum)[tw - 1];
    for (size_t k = 0; k < nt; k++) {
        free(c.tiles[k].bottom_row.datum);
        free(c.tiles[k].right_column.datum);
        free(c.tiles[k].bottom_right.datum);
    }
    free(c.tiles);
    if (seconds) *seconds = m.secs;
    return score;
}

/* ------------------------------ triad --------------------------------- */
typedef struct {
    float *a;
    const float *b, *c;
    float s;
} triad_arg_t;

static void triad_body(void *raw, int i) {
    triad_arg_t *t = (triad_arg_t *)raw;
    t->a[i] = t->b[i] + t->s * t->c[i];
}

typedef struct {
    triad_arg_t *arg;
    int n, tile, mode;
    double secs;
} triad_main_t;

static void triad_main(void *raw) {
    triad_main_t *m = (triad_main_t *)raw;
    ohc_loop_domain_t d = {0, m->n, 1, m->tile};
    double t0 = ohc_now();
    ohc_start_finish();
    ohc_forasync1d(triad_body, m->arg, &d, m->mode);
    ohc_end_finish();
    m->secs = ohc_now() - t0;
}

void ohc_triad(int nworkers, float *a, const float *b, const float *c, float s, int n, int tile,
               int mode, double *seconds) {
    triad_arg_t arg = {a, b, c, s};
    triad_main_t m = {&arg, n, tile, mode, 0};
    ohc_launch(nworkers, triad_main, &m);
    if (seconds) *seconds = m.secs;
}
