/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see uts_oracle.h).
 *
 * Restatement of the UTS 2.1 tree generator used by HClib's UTS workload.
 * Each function cites the reference lines it follows.
 */
#include "uts_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORA_MAXNUMCHILDREN 100 /* test/uts/uts.h:31 */

void ora_uts_default_params(ora_uts_params_t *p) {
    /* uts.c:57-103 defaults, overridden by the T1 defaults of uts.c:366-375 */
    p->type = ORA_GEO;
    p->shape_fn = ORA_FIXED;
    p->gen_mx = 10;
    p->b_0 = 4.0;
    p->root_id = 19;
    p->non_leaf_bf = 4;
    p->non_leaf_prob = 15.0 / 64.0;
    p->shift_depth = 0.5;
    p->compute_gran = 1;
}

static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* brg_sha1.c:241-249 (IV) and :187-239 (80 rounds over a 16-word rolling
 * schedule, ch/parity/maj as brg_sha1.c:160-164, round constants K). */
#define ORA_R(i, f, k)                                                            \
    do {                                                                          \
        uint32_t wi;                                                              \
        if ((i) < 16) wi = w[(i)];                                                \
        else {                                                                    \
            wi = rotl(w[((i) + 13) & 15] ^ w[((i) + 8) & 15] ^ w[((i) + 2) & 15] ^ \
                      w[(i) & 15], 1);                                            \
            w[(i) & 15] = wi;                                                     \
        }                                                                         \
        uint32_t t = rotl(a, 5) + (f) + e + (k) + wi;                             \
        e = d; d = c; c = rotl(b, 30); b = a; a = t;                              \
    } while (0)
#define ORA_CH (d ^ (b & (c ^ d)))
#define ORA_PAR (b ^ c ^ d)
#define ORA_MAJ ((b & c) | (d & (b ^ c)))

void ora_sha1_block(const uint32_t win[16], uint32_t h[5]) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = win[i];
    uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u,
             e = 0xc3d2e1f0u;
#pragma GCC unroll 80
    for (int i = 0; i < 20; i++) ORA_R(i, ORA_CH, 0x5a827999u);
#pragma GCC unroll 80
    for (int i = 20; i < 40; i++) ORA_R(i, ORA_PAR, 0x6ed9eba1u);
#pragma GCC unroll 80
    for (int i = 40; i < 60; i++) ORA_R(i, ORA_MAJ, 0x8f1bbcdcu);
#pragma GCC unroll 80
    for (int i = 60; i < 80; i++) ORA_R(i, ORA_PAR, 0xca62c1d6u);
    h[0] = 0x67452301u + a;
    h[1] = 0xefcdab89u + b;
    h[2] = 0x98badcfeu + c;
    h[3] = 0x10325476u + d;
    h[4] = 0xc3d2e1f0u + e;
}

/* rng_init, brg_sha1.c:49-66: SHA1(16 zero bytes || seed big-endian).
 * 20-byte message -> one block: words 0..4 = data, word 5 = 0x80 pad,
 * word 15 = bit length 160 (sha1_end, brg_sha1.c:283-325). */
void ora_rng_init(uint32_t st[5], int seed) {
    uint32_t w[16] = {0};
    w[4] = (uint32_t)seed;
    w[5] = 0x80000000u;
    w[15] = 160;
    ora_sha1_block(w, st);
}

/* rng_spawn, brg_sha1.c:68-83: SHA1(parent[20] || spawnnumber big-endian).
 * 24-byte message -> one block, bit length 192. */
void ora_rng_spawn(const uint32_t parent[5], uint32_t child[5], int i) {
    uint32_t w[16] = {0};
    for (int k = 0; k < 5; k++) w[k] = parent[k];
    w[5] = (uint32_t)i;
    w[6] = 0x80000000u;
    w[15] = 192;
    ora_sha1_block(w, child);
}

/* rng_rand, brg_sha1.c:85-95: bytes 16..19 big-endian, & POS_MASK. */
int ora_rng_rand(const uint32_t st[5]) { return (int)(st[4] & 0x7fffffffu); }

/* rng_toProb, uts.c:143-148 */
static double to_prob(int n) { return (n < 0) ? 0.0 : ((double)n) / 2147483648.0; }

/* uts_numChildren_bin, uts.c:162-168 */
static int num_children_bin(const ora_uts_params_t *p, const uint32_t st[5]) {
    int v = ora_rng_rand(st);
    double d = to_prob(v);
    return (d < p->non_leaf_prob) ? p->non_leaf_bf : 0;
}

/* uts_numChildren_geo, uts.c:171-222 */
static int num_children_geo(const ora_uts_params_t *p, int depth, const uint32_t st[5]) {
    double b_i = p->b_0;
    if (depth > 0) {
        switch (p->shape_fn) {
        case ORA_EXPDEC:
            b_i = p->b_0 * pow((double)depth, -log(p->b_0) / log((double)p->gen_mx));
            break;
        case ORA_CYCLIC:
            if (depth > 5 * p->gen_mx) { b_i = 0.0; break; }
            b_i = pow(p->b_0, sin(2.0 * 3.141592653589793 * (double)depth / (double)p->gen_mx));
            break;
        case ORA_FIXED:
            b_i = (depth < p->gen_mx) ? p->b_0 : 0;
            break;
        case ORA_LINEAR:
        default:
            b_i = p->b_0 * (1.0 - (double)depth / (double)p->gen_mx);
            break;
        }
    }
    double prob = 1.0 / (1.0 + b_i);
    int h = ora_rng_rand(st);
    double u = to_prob(h);
    double x = floor(log(1 - u) / log(1 - prob));
    /* (int) of a NaN is undefined in C; x86-64 cvttsd2si yields INT_MIN,
     * which the caller then treats as a leaf (numChildren <= 0). */
    if (x != x) return (int)0x80000000u;
    return (int)x;
}

/* uts_numChildren, uts.c:225-274 */
int ora_uts_num_children(const ora_uts_params_t *p, int node_type, int height,
                         const uint32_t st[5]) {
    int nc = 0;
    switch (p->type) {
    case ORA_BIN:
        nc = (height == 0) ? (int)floor(p->b_0) : num_children_bin(p, st);
        break;
    case ORA_GEO:
        nc = num_children_geo(p, height, st);
        break;
    case ORA_HYBRID:
        nc = (height < p->shift_depth * p->gen_mx) ? num_children_geo(p, height, st)
                                                  : num_children_bin(p, st);
        break;
    case ORA_BALANCED:
        if (height < p->gen_mx) nc = (int)p->b_0;
        break;
    default:
        return 0;
    }
    if (height == 0 && node_type == ORA_BIN) {
        int root_bf = (int)ceil(p->b_0);
        if (nc > root_bf) nc = root_bf;
    } else if (p->type != ORA_BALANCED) {
        if (nc > ORA_MAXNUMCHILDREN) nc = ORA_MAXNUMCHILDREN;
    }
    return nc;
}

/* uts_childType, uts.c:277-294 */
int ora_uts_child_type(const ora_uts_params_t *p, int height) {
    switch (p->type) {
    case ORA_HYBRID:
        return (height < p->shift_depth * p->gen_mx) ? ORA_GEO : ORA_BIN;
    default:
        return p->type;
    }
}

typedef struct {
    uint32_t st[5];
    int height;
    int type;
} ora_node_t;

typedef struct {
    ora_node_t *v;
    size_t n, cap;
} ora_stack_t;

static int stack_push(ora_stack_t *s, const ora_node_t *x) {
    if (s->n == s->cap) {
        size_t nc = s->cap ? s->cap * 2 : 4096;
        ora_node_t *nv = (ora_node_t *)realloc(s->v, nc * sizeof(ora_node_t));
        if (!nv) return -1;
        s->v = nv;
        s->cap = nc;
    }
    s->v[s->n++] = *x;
    return 0;
}

/* genChildren + ss_get_work loop (UTS.cpp:154-232, 383-402) on one worker. */
static int dfs(const ora_uts_params_t *p, ora_stack_t *s, ora_uts_result_t *out,
               uint64_t *hist, int max_levels) {
    while (s->n) {
        ora_node_t parent = s->v[--s->n];
        out->nodes++;
        if (hist && parent.height < max_levels) hist[parent.height]++;
        if ((uint64_t)parent.height > out->max_depth) out->max_depth = parent.height;
        int nc = ora_uts_num_children(p, parent.type, parent.height, parent.st);
        int ct = ora_uts_child_type(p, parent.height);
        if (nc > 0) {
            for (int i = 0; i < nc; i++) {
                ora_node_t child;
                child.type = ct;
                child.height = parent.height + 1;
                for (int g = 0; g < p->compute_gran; g++) ora_rng_spawn(parent.st, child.st, i);
                if (stack_push(s, &child)) return -1;
            }
        } else {
            out->leaves++;
        }
    }
    return 0;
}

int ora_uts_serial(const ora_uts_params_t *p, ora_uts_result_t *out, uint64_t *hist,
                   int max_levels) {
    ora_stack_t s = {0};
    ora_node_t root;
    memset(out, 0, sizeof(*out));
    if (hist) memset(hist, 0, sizeof(uint64_t) * (size_t)max_levels);
    /* uts_initRoot, uts.c:151-159 */
    root.type = p->type;
    root.height = 0;
    ora_rng_init(root.st, p->root_id);
    if (stack_push(&s, &root)) return -1;
    int rc = dfs(p, &s, out, hist, max_levels);
    free(s.v);
    return rc;
}

int ora_uts_serial_root_range(const ora_uts_params_t *p, int first, int last, int count_root,
                              ora_uts_result_t *out) {
    ora_stack_t s = {0};
    ora_node_t root;
    memset(out, 0, sizeof(*out));
    root.type = p->type;
    root.height = 0;
    ora_rng_init(root.st, p->root_id);
    int nc = ora_uts_num_children(p, root.type, 0, root.st);
    if (count_root) {
        out->nodes = 1;
        if (nc <= 0) out->leaves = 1;
    }
    int ct = ora_uts_child_type(p, 0);
    for (int i = first; i < last && i < nc; i++) {
        ora_node_t child;
        child.type = ct;
        child.height = 1;
        ora_rng_spawn(root.st, child.st, i);
        if (stack_push(&s, &child)) return -1;
    }
    int rc = dfs(p, &s, out, NULL, 0);
    free(s.v);
    return rc;
}
