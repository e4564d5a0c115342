/* UTS through include/hclib.h: one async of the UTS task kind inside a
 * finish (test/uts/UTS.cpp:100-118), tree statistics printed like
 * uts_showStats (test/uts/uts.c:452-466). Usage: uts_gpu -t 1 -a 3 ... */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hclib.h"

void uts_root(void *arg) { (void)arg; /* host body never runs: device kind */ }

static hclib_hip_uts_task_t T;

void taskMain(void *arg) {
    (void)arg;
    unsigned long long t0 = hclib_current_time_ns();
    hclib_start_finish();
    hclib_async(uts_root, &T, NULL, 0, hclib_hip_gpu_locale(0));
    hclib_end_finish();
    unsigned long long t1 = hclib_current_time_ns();
    double s = (t1 - t0) * 1e-9;
    printf("Tree size = %llu, tree depth = %llu, num leaves = %llu (%.2f%%)\n", T.nodes,
           T.max_depth, T.leaves, T.leaves / (float)T.nodes * 100.0);
    printf("Wallclock time = %.3f sec, performance = %.0f nodes/sec\n", s, T.nodes / s);
}

int main(int argc, char **argv) {
    /* T1 defaults, test/uts/uts.c:366-375 */
    T.type = 1; T.shape_fn = 3; T.gen_mx = 10; T.b_0 = 4; T.root_id = 19;
    T.non_leaf_bf = 4; T.non_leaf_prob = 15.0 / 64.0; T.shift_depth = 0.5; T.compute_gran = 1;
    for (int i = 1; i + 1 < argc; i += 2) {
        const char *v = argv[i + 1];
        switch (argv[i][1]) {
        case 't': T.type = atoi(v); break;
        case 'a': T.shape_fn = atoi(v); break;
        case 'd': T.gen_mx = atoi(v); break;
        case 'b': T.b_0 = atof(v); break;
        case 'r': T.root_id = atoi(v); break;
        case 'm': T.non_leaf_bf = atoi(v); break;
        case 'q': T.non_leaf_prob = atof(v); break;
        case 'f': T.shift_depth = atof(v); break;
        case 'g': T.compute_gran = atoi(v); break;
        default: break;
        }
    }
    hclib_hip_register_async_kind(uts_root, HCLIB_HIP_KIND_UTS);
    const char *deps[] = {"system", "hip"};
    hclib_launch(taskMain, NULL, deps, 2);
    return 0;
}
