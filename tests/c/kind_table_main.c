/* The C drop-in with device kinds from the program's own HIP object
 * (tests/hip/kind_table.hip, linked in): test/fib/fib.c's driver unchanged
 * but for the device kind, then a forasync of a device loop body over
 * GPU-locale memory (hclib_allocate_at / hclib_async_copy, src/hclib-mem.c),
 * FLAT and RECURSIVE, 1-D. `kind_table_main bad` registers an unknown
 * built-in kind id and must be refused. */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hclib.h"

long fib_iter(int n) {  /* test/fib/fib.c:38-46 */
    int i, x, y;
    for (i = 0, x = 1, y = 0; i <= n; i++) {
        int t = x;
        x = y;
        y += t;
    }
    return x;
}

typedef struct {
    int n;
    long res;
} FibArgs;

void fib(void *raw_args) {  /* test/fib/fib.c:57-71: the host body */
    FibArgs *args = raw_args;
    if (args->n < 2) {
        args->res = args->n;
    } else {
        FibArgs lhsArgs = {args->n - 1, 0};
        FibArgs rhsArgs = {args->n - 2, 0};
        hclib_start_finish();
        hclib_async(fib, &lhsArgs, NULL, 0, NULL);
        hclib_async(fib, &rhsArgs, NULL, 0, NULL);
        hclib_end_finish();
        args->res = lhsArgs.res + rhsArgs.res;
    }
}

typedef struct {
    int *y;
    const int *x;
} ScaleArgs;

void scale_body(void *raw_args, int i) {  /* the host body */
    ScaleArgs *a = raw_args;
    a->y[i] = 3 * a->x[i] + i;
}

#define N 100000

static void entry(void *unused) {
    (void)unused;
    if (hclib_hip_device_kind_count() < 1 || !hclib_hip_device_kind_name(fib) ||
        strcmp(hclib_hip_device_kind_name(fib), "fib") != 0) {
        fprintf(stderr, "fib is not in the kind table\n");
        exit(1);
    }
    /* the device task kind */
    for (int n = 0; n <= 25; n += 5) {
        FibArgs args = {n, -1};
        hclib_start_finish();
        hclib_async(fib, &args, NULL, 0, hclib_hip_gpu_locale(0));
        hclib_end_finish();
        printf("Fib(%d) = %ld = %ld\n", n, fib_iter(n), args.res);
        assert(args.res == fib_iter(n));
    }
    /* the device loop body over GPU-locale memory */
    hclib_locale_t *gpu = hclib_hip_gpu_locale(0), *host = hclib_get_closest_locale();
    int *hx = malloc(N * sizeof(int)), *hy = malloc(N * sizeof(int));
    for (int i = 0; i < N; ++i) hx[i] = i % 977 - 400;
    int *dx = hclib_future_wait(hclib_allocate_at(N * sizeof(int), gpu));
    int *dy = hclib_future_wait(hclib_allocate_at(N * sizeof(int), gpu));
    hclib_future_wait(hclib_async_copy(gpu, dx, host, hx, N * sizeof(int), NULL, 0));
    const int reps = getenv("KIND_TABLE_REPS") ? atoi(getenv("KIND_TABLE_REPS")) : 1;
    for (int it = 0; it < 2 * reps; ++it) {
        const int mode = it % 2;
        hclib_future_wait(hclib_memset_at(dy, 0, N * sizeof(int), gpu));
        ScaleArgs sa = {dy, dx};
        hclib_loop_domain_t dom = {0, N, 1, -1};
        hclib_start_finish();
        hclib_forasync(scale_body, &sa, 1, &dom, mode == 0 ? FORASYNC_MODE_FLAT : FORASYNC_MODE_RECURSIVE);
        hclib_end_finish();
        hclib_future_wait(hclib_async_copy(host, hy, gpu, dy, N * sizeof(int), NULL, 0));
        int bad = 0, first_bad = -1, last_bad = -1;
        for (int i = 0; i < N; ++i)
            if (hy[i] != 3 * hx[i] + i) {
                if (first_bad < 0) first_bad = i;
                last_bad = i;
                ++bad;
            }
        if (bad) {
            fprintf(stderr, "mode %d: %d wrong indices in [%d, %d]; y[%d] = %d, want %d (tile %d)\n", mode, bad,
                    first_bad, last_bad, first_bad, hy[first_bad], 3 * hx[first_bad] + first_bad, dom.tile);
            exit(1);
        }
        printf("forasync (%s) of the device body: %d indices OK\n", mode == 0 ? "FLAT" : "RECURSIVE", N);
    }
    /* R4 with device work (src/hclib.c:466-473, src/hclib-runtime.c:1280-1313):
     * forasync_future of the device body and a non-blocking finish around a
     * device task return futures at once; the host waits on them later */
    {
        hclib_future_wait(hclib_memset_at(dy, 0, N * sizeof(int), gpu));
        ScaleArgs sa = {dy, dx};
        hclib_loop_domain_t dom = {0, N, 1, -1};
        hclib_future_t *f = hclib_forasync_future(scale_body, &sa, 1, &dom, FORASYNC_MODE_RECURSIVE);
        FibArgs args = {20, -1};
        hclib_start_finish();
        hclib_async(fib, &args, NULL, 0, hclib_hip_gpu_locale(0));
        hclib_future_t *g = hclib_end_finish_nonblocking();
        hclib_future_wait(g);
        hclib_future_wait(f);
        hclib_future_wait(hclib_async_copy(host, hy, gpu, dy, N * sizeof(int), NULL, 0));
        for (int i = 0; i < N; ++i)
            if (hy[i] != 3 * hx[i] + i) {
                fprintf(stderr, "forasync_future: y[%d] = %d, want %d\n", i, hy[i], 3 * hx[i] + i);
                exit(1);
            }
        assert(args.res == fib_iter(20));
        printf("forasync_future + end_finish_nonblocking with device work: OK\n");
    }
    hclib_free_at(dx, gpu);
    hclib_free_at(dy, gpu);
    free(hx);
    free(hy);
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "bad") == 0) {
        hclib_hip_register_async_kind(fib, 99); /* refused: no such built-in kind */
        printf("unknown kind accepted\n");
        return 0;
    }
    const char *deps[] = {"system", "hip"};
    hclib_launch(entry, NULL, deps, 2);
    printf("Check results: OK\n");
    return 0;
}
