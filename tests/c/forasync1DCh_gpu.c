/* A chunked 1-D forasync whose body runs on the GPU through include/hclib.h.
 *
 * Scenario of the reference's test/c/forasync1DCh.c (a 1024-iteration FLAT
 * loop in tiles of 33; every slot is visited exactly once and receives its
 * own index), written here as a drop-in check of the device loop-body path:
 * the host function `mark_slot` is named a device loop body once
 * (hclib_hip_register_forasync_body -> the built-in IOTA_CHECK body, which
 * stores the index and flags any slot it finds already written), and the
 * program then calls hclib_forasync exactly as a CPU HClib program would.
 * Afterwards the host checks the slots itself. Prints "Check results: OK". */
#include <stdio.h>
#include <stdlib.h>

#include "hclib.h"

enum { kSlots = 1024, kTile = 33, kUnvisited = -1 };

/* host twin of the device body (never runs on the host in this program) */
void mark_slot(void *slots, int i) {
    int *s = (int *)slots;
    if (s[i] != kUnvisited) abort();
    s[i] = i;
}

static void run_loop(void *slots) {
    for (int i = 0; i < kSlots; i++) ((int *)slots)[i] = kUnvisited;
    hclib_loop_domain_t dom;
    dom.low = 0;
    dom.high = kSlots;
    dom.stride = 1;
    dom.tile = kTile;
    hclib_start_finish();
    hclib_forasync((void *)mark_slot, slots, 1, &dom, FORASYNC_MODE_FLAT);
    hclib_end_finish();
}

int main(void) {
    int *slots = (int *)calloc(kSlots, sizeof(int));
    if (!slots) return 2;
    hclib_hip_register_forasync_body((void *)mark_slot, 2 /* HCLIB_HIP_BODY_IOTA_CHECK */);
    const char *modules[2] = {"system", "hip"};
    hclib_launch(run_loop, slots, modules, 2);
    int bad = 0;
    for (int i = 0; i < kSlots; i++) bad += slots[i] != i;
    free(slots);
    if (bad) {
        printf("Check results: %d slots wrong\n", bad);
        return 1;
    }
    printf("Check results: OK\n");
    return 0;
}
