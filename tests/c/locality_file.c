/*
 * locality_file.c — a locality graph loaded from the reference's JSON
 * format (HCLIB_LOCALITY_FILE, src/hclib-locality-graph.c:372-573), with
 * GPU locales.
 *
 * Run with HCLIB_LOCALITY_FILE=tests/golden/locality/davinci.json (the
 * reference's locality_graphs/davinci.json: 12 workers, two sockets of six
 * L2s, two GPUs, an interconnect). Its module registers the locale types a
 * system module and a communication module would (L2, L3, Interconnect);
 * the GPU type comes from the hip plug-in module named in deps
 * (libhclib_hip.so, as the reference's modules/cuda registers it), with
 * metadata naming the HIP device. Checks the graph, worker 0's paths ("L2_$(id / 6)_$(id % 6)"
 * interpreted for id 0), the locality queries and breadth-first closest-
 * locale search (src/hclib-locality-graph.c:901-1165).
 * With argv[1] == "nointerconnect" the module does not register the
 * Interconnect type, and loading must fail like the reference's
 * ("Unknown locale type", exit 1); with "nohip" deps omit "hip", so the
 * file's GPU locales have no type (the same failure). With "gpu" the
 * program also allocates, fills and copies memory at the file's GPU0
 * locale and checks, through hclib_hip_module_counts (looked up in the
 * loaded module), that every operation ran the module's callbacks.
 */
#define _GNU_SOURCE /* RTLD_DEFAULT */
#include <assert.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hclib.h"

static int with_interconnect = 1, with_hip = 1, use_gpu = 0;
static int l2, l3, ic;

static void pre(void) {
    l2 = (int)hclib_add_known_locale_type("L2");
    l3 = (int)hclib_add_known_locale_type("L3");
    if (with_interconnect) ic = (int)hclib_add_known_locale_type("Interconnect");
}
HCLIB_REGISTER_MODULE("locality_test", pre, NULL, NULL)

static hclib_locale_t *by_label(const char *lbl) {
    hclib_locale_t *all = hclib_get_all_locales();
    for (int i = 0; i < hclib_get_num_locales(); i++)
        if (strcmp(all[i].lbl, lbl) == 0) return all + i;
    return NULL;
}

static void entrypoint(void *arg) {
    (void)arg;
    const int n = hclib_get_num_locales();
    assert(n == 18);
    hclib_locale_t *all = hclib_get_all_locales();
    assert(strcmp(all[0].lbl, "sysmem") == 0 && strcmp(all[17].lbl, "Interconnect") == 0);
    for (int i = 0; i < n; i++) assert(all[i].id == i && all[i].reachable == (i != 17 && i != 15 && i != 16));

    const int gpu = (int)hclib_add_known_locale_type("GPU");
    int ngpu = 0;
    hclib_locale_t **gpus = hclib_get_all_locales_of_type(gpu, &ngpu);
    assert(ngpu == 2 && hclib_get_num_locales_of_type(gpu) == 2);
    for (int k = 0; k < 2; k++) {
        char want[8];
        snprintf(want, sizeof(want), "GPU%d", k);
        assert(strcmp(gpus[k]->lbl, want) == 0);
        hclib_hip_locale_metadata_t *m = (hclib_hip_locale_metadata_t *)gpus[k]->metadata;
        assert(m && m->device == k);
    }
    assert(hclib_get_num_locales_of_type(l2) == 12 && hclib_get_num_locales_of_type(l3) == 2);

    /* worker 0: pop = steal = L2_0_0, L3_0, sysmem */
    hclib_locale_t *closest = hclib_get_closest_locale();
    assert(strcmp(closest->lbl, "L2_0_0") == 0 && (int)closest->type == l2);
    assert(hclib_get_master_place() == closest);
    assert(strcmp(hclib_get_central_place()->lbl, "sysmem") == 0);
    hclib_locale_t **priv = hclib_get_thread_private_locales();
    assert(priv[0] == closest);
    free(priv);

    /* breadth-first over the reachability edges */
    assert(hclib_get_closest_locale_of_type(closest, gpu) == by_label("GPU0"));
    assert(hclib_get_closest_locale_of_type(by_label("L2_1_3"), l3) == by_label("L3_1"));
    assert(hclib_get_closest_locale_of_type(by_label("GPU1"), ic) == by_label("Interconnect"));
    int types[2] = {l3, gpu};
    assert(hclib_get_closest_locale_of_types(by_label("L2_1_5"), types, 2) == by_label("L3_1"));
    assert(hclib_get_closest_locale_of_type(closest, 12345) == NULL);

    /* the graph object and every declared worker's paths */
    int nworkers = 0;
    hclib_locality_graph *g = NULL;
    hclib_worker_paths *paths = NULL;
    generate_locality_info(&nworkers, &g, &paths);
    assert(nworkers == 12 && g->n_locales == 18);
    assert(g->edges[0 * 18 + 15] && g->edges[15 * 18 + 0] && !g->edges[15 * 18 + 16]);
    assert(paths[7].pop_path->path_length == 3);
    assert(strcmp(paths[7].pop_path->locales[0]->lbl, "L2_1_1") == 0);
    assert(strcmp(paths[7].steal_path->locales[1]->lbl, "L3_1") == 0);
    print_locality_graph(g);
    print_worker_paths(paths, 2);

    /* memory at a system-memory locale of the file */
    int *p = (int *)hclib_future_wait(hclib_allocate_at(64 * sizeof(int), by_label("sysmem")));
    assert(p);
    hclib_future_wait(hclib_memset_at(p, 0, 64 * sizeof(int), by_label("sysmem")));
    assert(p[63] == 0);
    hclib_free_at(p, by_label("sysmem"));

    if (use_gpu) {
        /* memory at the file's GPU0 locale: the hip module's callbacks */
        void (*counts)(unsigned long long *) =
            (void (*)(unsigned long long *))dlsym(RTLD_DEFAULT, "hclib_hip_module_counts");
        assert(counts);
        unsigned long long c0[6], c1[6];
        counts(c0);
        assert(c0[5] == 2); /* the module populated both GPU locales' metadata */
        hclib_locale_t *g0 = by_label("GPU0"), *host = by_label("sysmem");
        const size_t N = 1 << 16;
        unsigned char *d = (unsigned char *)hclib_future_wait(hclib_allocate_at(N, g0));
        assert(d);
        hclib_future_wait(hclib_memset_at(d, 0x3c, N, g0));
        unsigned char *h = (unsigned char *)malloc(N);
        hclib_future_wait(hclib_async_copy(host, h, g0, d, N, NULL, 0));
        for (size_t i = 0; i < N; ++i) assert(h[i] == 0x3c);
        hclib_free_at(d, g0);
        free(h);
        counts(c1);
        assert(c1[0] == c0[0] + 1 && c1[3] == c0[3] + 1 && c1[4] == c0[4] + 1 && c1[2] == c0[2] + 1);
        printf("hip module callbacks: alloc %llu, memset %llu, copy %llu, free %llu\n", c1[0], c1[3], c1[4], c1[2]);
    }
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "nointerconnect") == 0) with_interconnect = 0;
    if (argc > 1 && strcmp(argv[1], "nohip") == 0) with_hip = 0;
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) use_gpu = 1;
    const char *deps[] = {"hip"};
    hclib_launch(entrypoint, NULL, deps, with_hip ? 1 : 0);
    printf("Check results: OK\n");
    return 0;
}
