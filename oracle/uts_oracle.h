/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the UTS tree generator that HClib's UTS workload uses
 * (reference: test/uts/uts.c, test/uts/rng/brg_sha1.c, test/uts/UTS.cpp).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code; the product (hclib_amd/) never links or calls it.
 *
 * Parity pin: validated against the reference's own uts.c + brg_sha1.c
 * compiled from /root/reference by oracle/Makefile into oracle/_ref/ (see
 * tests/test_oracle.py) and against the published goldens in
 * test/uts/sample_trees.sh:17-43 (committed as tests/golden/uts_goldens.json).
 */
#ifndef HCLIB_ORACLE_UTS_H
#define HCLIB_ORACLE_UTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Tree / shape enums: test/uts/uts.h:72-73 */
enum { ORA_BIN = 0, ORA_GEO = 1, ORA_HYBRID = 2, ORA_BALANCED = 3 };
enum { ORA_LINEAR = 0, ORA_EXPDEC = 1, ORA_CYCLIC = 2, ORA_FIXED = 3 };

/* Tree parameters with the defaults of test/uts/uts.c:57-103 and the T1
 * defaults uts_parseParams installs (uts.c:366-375). */
typedef struct {
    int type;          /* -t */
    int shape_fn;      /* -a */
    int gen_mx;        /* -d */
    int root_id;       /* -r */
    int non_leaf_bf;   /* -m */
    int compute_gran;  /* -g */
    double b_0;        /* -b */
    double non_leaf_prob; /* -q */
    double shift_depth;   /* -f */
} ora_uts_params_t;

typedef struct {
    uint64_t nodes;
    uint64_t leaves;
    uint64_t max_depth;
} ora_uts_result_t;

/* Default params (T1, uts.c:366-375). */
void ora_uts_default_params(ora_uts_params_t *p);

/* SHA-1 single-block compression from the standard IV over 16 big-endian
 * words (brg_sha1.c:187-239 sha1_compile + sha1_begin IV :241-249). */
void ora_sha1_block(const uint32_t w[16], uint32_t h[5]);

/* RNG state is kept as the 5 big-endian digest words; byte k of the
 * reference's uint8 state[20] is (st[k/4] >> (24 - 8*(k%4))) & 0xff. */
void ora_rng_init(uint32_t st[5], int seed);                          /* brg_sha1.c:49-66 */
void ora_rng_spawn(const uint32_t parent[5], uint32_t child[5], int i); /* brg_sha1.c:68-83 */
int  ora_rng_rand(const uint32_t st[5]);                              /* brg_sha1.c:85-95 */

/* uts_numChildren (uts.c:225-274), incl. _bin (162-168) and _geo (171-222),
 * evaluated with libm exactly as the reference does. */
int ora_uts_num_children(const ora_uts_params_t *p, int node_type, int height,
                         const uint32_t st[5]);
int ora_uts_child_type(const ora_uts_params_t *p, int height); /* uts.c:277-294 */

/* Serial depth-first search over the whole tree (the per-worker stack walk
 * of UTS.cpp:154-232, one worker). Counts nodes at pop, leaves when
 * numChildren <= 0, depth = max height (UTS.cpp:161, 205-206, 383-402).
 * level_hist (optional, may be NULL) receives nodes per depth for depths
 * < max_levels. Returns 0 on success. */
int ora_uts_serial(const ora_uts_params_t *p, ora_uts_result_t *out,
                   uint64_t *level_hist, int max_levels);

/* Serial walk of the subtrees rooted at the children [first, last) of the
 * root only (used for multi-rank sharding checks). The root itself is
 * counted iff count_root != 0. */
int ora_uts_serial_root_range(const ora_uts_params_t *p, int first, int last,
                              int count_root, ora_uts_result_t *out);

#ifdef __cplusplus
}
#endif
#endif
