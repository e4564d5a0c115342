// Nested finish/async over host lambdas through include/hclib_cpp.h.
// Restates the checks of the reference's test/cpp/finish1.cpp (recursive
// finish scopes, one async each) and test/cpp/async0.cpp-style fan-out.
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>

#include "hclib_cpp.h"

#define NB_ASYNC 127

static int *ran = NULL;

static void spawn_async(volatile int *indices, int i) {
    if (i < NB_ASYNC) {
        hclib::finish([=]() {
            indices[i] = i;
            hclib::async([=]() {
                int idx = indices[i];
                assert(ran[idx] == -1);
                ran[idx] = idx;
            });
            spawn_async(indices, i + 1);
        });
        assert(ran[i] == i);  // the finish above joined the async
    }
}

int main() {
    const char *deps[] = {"system"};
    int fanout_sum = 0;
    hclib::launch(deps, 1, [&]() {
        volatile int *indices = (int *)malloc(sizeof(int) * NB_ASYNC);
        ran = (int *)malloc(sizeof(int) * NB_ASYNC);
        for (int i = 0; i < NB_ASYNC; i++) ran[i] = -1;
        hclib::finish([=]() { spawn_async(indices, 0); });
        free((void *)indices);
        // fan-out: 1000 asyncs joined by one finish
        int *cells = (int *)calloc(1000, sizeof(int));
        hclib::finish([=]() {
            for (int i = 0; i < 1000; ++i) hclib::async([=]() { cells[i] = i + 1; });
        });
        for (int i = 0; i < 1000; ++i) fanout_sum += cells[i];
        free(cells);
    });
    printf("Check results: ");
    for (int i = 0; i < NB_ASYNC; i++) assert(ran[i] == i);
    assert(fanout_sum == 1000 * 1001 / 2);
    free(ran);
    printf("OK\n");
    return 0;
}
