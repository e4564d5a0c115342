/* test/fib/fib.c (async/finish version, :57-71, :151-186) against the
 * MI355X build: the same fib task body and FibArgs struct; the only
 * addition is naming `fib` a device task kind. Usage: fib_gpu N
 *
 * fib_iter, FibArgs and fib() restate the reference's caller, whose
 * unchanged body is the point of this drop-in test. HClib: Copyright (c)
 * 2013-2015, Rice University, BSD 3-clause license (the reference
 * repository's LICENSE file); the rest of this file is this project's. */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>

#include "hclib.h"

long fib_iter(int n) {
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

void fib(void *raw_args) {
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

void taskMain(void *raw_args) {
    int n = *(int *)raw_args;
    FibArgs args = {n, 0};
    unsigned long long t0 = hclib_current_time_ns();
    hclib_start_finish();
    hclib_async(fib, &args, NULL, 0, hclib_hip_gpu_locale(0));
    hclib_end_finish();
    unsigned long long t1 = hclib_current_time_ns();
    printf("Fib(%d) = %ld = %ld (%.3f ms)\n", n, fib_iter(n), args.res, (t1 - t0) * 1e-6);
    assert(args.res == fib_iter(n));
}

int main(int argc, char **argv) {
    int n = argc > 1 ? atoi(argv[1]) : 30;
    hclib_hip_register_async_kind(fib, HCLIB_HIP_KIND_FIB);
    const char *deps[] = {"system", "hip"};
    hclib_launch(taskMain, &n, deps, 2);
    printf("Check results: OK\n");
    return 0;
}
