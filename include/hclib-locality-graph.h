/*
 * hclib-locality-graph.h — locales and the locality graph (MI355X build).
 *
 * Same types and prototypes as the reference's inc/hclib-locality-graph.h:
 *   hclib_locale_t            :56-67 (programs index hclib_get_all_locales()
 *                             as an array, test/c/memory/allocate.c:42-47)
 *   hclib_locality_graph / _path / hclib_worker_paths   :69-84
 *   locale queries            :100-121
 *   hclib_add_known_locale_type (unsigned)              :123
 *
 * The graph of this build is the host's system memory ("sysmem") plus the
 * GPU locales (type "GPU"), either the process's bound GPU (default) or the
 * GPU locales a locality file names (HCLIB_LOCALITY_FILE, the reference's
 * JSON format, src/hclib-locality-graph.c:372-573). Modules add locale types
 * (modules/system adds L1/L2/L3/sysmem) before the graph is built.
 */
#ifndef _HCLIB_LOCALITY_GRAPH_H
#define _HCLIB_LOCALITY_GRAPH_H

#include "hclib-rt.h"

struct _hclib_deque_t;
struct _hclib_task_t;

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _hclib_locale_t {
    int id;
    unsigned type;
    const char *lbl;
    const char *special_type;
    void *metadata;
    void (**idle_funcs)(void);
    unsigned n_idle_funcs;
    int reachable;

    struct _hclib_deque_t *deques;
} hclib_locale_t;

typedef struct _hclib_locality_graph {
    hclib_locale_t *locales;
    unsigned n_locales;
    unsigned *edges; /* n_locales x n_locales adjacency (1 = connected) */
} hclib_locality_graph;

typedef struct _hclib_locality_path {
    hclib_locale_t **locales;
    unsigned path_length;
} hclib_locality_path;

typedef struct _hclib_worker_paths {
    hclib_locality_path *pop_path;
    hclib_locality_path *steal_path;
    int last_successful_steal_locale;
} hclib_worker_paths;

/* src/hclib-locality-graph.c:372-573: parse a locality file (the reference's
 * JSON: "declarations", "reachability", "pop_paths", "steal_paths") into a
 * graph and per-worker paths; exits with a message on a malformed file */
void load_locality_info(const char *filename, int *nworkers_out, hclib_locality_graph **graph_out,
                        hclib_worker_paths **worker_paths_out);
/* src/hclib-locality-graph.c:581-643: the default graph of this build */
void generate_locality_info(int *nworkers_out, hclib_locality_graph **graph_out,
                            hclib_worker_paths **worker_paths_out);
void print_locality_graph(hclib_locality_graph *graph);
void print_worker_paths(hclib_worker_paths *worker_paths, int nworkers);

void hclib_locale_mark_special(hclib_locale_t *locale, const char *special_type);

int hclib_get_num_locales(void);
hclib_locale_t *hclib_get_closest_locale(void);
hclib_locale_t **hclib_get_thread_private_locales(void);
hclib_locale_t *hclib_get_master_place(void);
hclib_locale_t *hclib_get_central_place(void);
hclib_locale_t *hclib_get_all_locales(void);
hclib_locale_t *hclib_get_closest_locale_of_types(hclib_locale_t *locale, int *locale_types,
                                                  int n_locale_types);
hclib_locale_t *hclib_get_closest_locale_of_type(hclib_locale_t *locale, int locale_type);
hclib_locale_t **hclib_get_all_locales_of_type(int type, int *out_count);
int hclib_get_num_locales_of_type(int locale_type);

unsigned hclib_add_known_locale_type(const char *lbl);

/* inc/hclib-locality-graph.h:102-105 (src/hclib-locality-graph.c:760-829):
 * tasks queued at a locale (here: ready host tasks placed there — the host
 * control thread is this build's one host worker; device tasks live in the
 * megakernel's queues only while a launch runs), and per-locale idle
 * functions, run for every locale of a worker's steal path on request */
unsigned locale_num_tasks(hclib_locale_t *locale);
void locale_run_idle_tasks(hclib_worker_state *ws);
void locale_register_idle_task(hclib_locale_t *locale, void (*fp)(void));

#ifdef __cplusplus
}
#endif

#endif
