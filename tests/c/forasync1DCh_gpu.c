/* test/c/forasync1DCh.c (H1=1024, T1=33, FLAT) against the MI355X build:
 * same body and checks; forasync_fct1 is named a device loop body. */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>

#include "hclib.h"

#define H1 1024
#define T1 33

void forasync_fct1(void *argv, int idx) {
    int *ran = (int *)argv;
    assert(ran[idx] == -1);
    ran[idx] = idx;
}

void init_ran(int *ran, int size) {
    while (size > 0) {
        ran[size - 1] = -1;
        size--;
    }
}

void entrypoint(void *arg) {
    int *ran = (int *)arg;
    init_ran(ran, H1);
    hclib_loop_domain_t loop = {0, H1, 1, T1};
    hclib_start_finish();
    hclib_forasync((void *)forasync_fct1, (void *)ran, 1, &loop, FORASYNC_MODE_FLAT);
    hclib_end_finish();
}

int main(int argc, char **argv) {
    int *ran = (int *)malloc(H1 * sizeof(int));
    assert(ran);
    hclib_hip_register_forasync_body((void *)forasync_fct1, 2 /* HCLIB_HIP_BODY_IOTA_CHECK */);
    const char *deps[] = {"system", "hip"};
    hclib_launch(entrypoint, ran, deps, 2);
    for (int i = 0; i < H1; i++) assert(ran[i] == i);
    printf("Check results: OK\n");
    return 0;
}
