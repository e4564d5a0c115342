/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Harness linked with the reference's OWN UTS sources, compiled in place
 * from /root/reference/test/uts/uts.c and test/uts/rng/brg_sha1.c by
 * oracle/Makefile (output: oracle/_ref/libref_uts.so, git-ignored). The
 * reference's uts.c expects the implementation hooks impl_* that UTS.cpp
 * defines (UTS.cpp:258-301); they are provided here. The walk below is the
 * one-worker form of UTS.cpp's genChildren/ss_get_work loop (154-232,
 * 383-402), using the reference's uts_initRoot / uts_numChildren /
 * uts_childType / rng_spawn and its argv parser uts_parseParams.
 *
 * Used only to pin oracle/uts_oracle.c (tests/test_oracle.py) and to make
 * golden fixtures (scripts/gen_golden.py); never shipped or measured.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "uts.h"

char *impl_getName(void) { return "oracle ref harness (serial)"; }
int impl_paramsToStr(char *strBuf, int ind) { return ind; }
int impl_parseParam(char *param, char *value) { (void)param; (void)value; return 1; }
void impl_helpMessage(void) {}
void impl_abort(int err) { exit(err); }

typedef struct {
    Node *v;
    size_t n, cap;
} ref_stack_t;

static void push(ref_stack_t *s, const Node *x) {
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 4096;
        s->v = (Node *)realloc(s->v, s->cap * sizeof(Node));
        if (!s->v) exit(3);
    }
    s->v[s->n++] = *x;
}

/* Parse a UTS argument vector with the reference parser, then walk the tree.
 * argv[0] is a program name. Outputs nodes/leaves/max-height and an
 * optional per-depth histogram. */
int ref_uts_run(int argc, char **argv, unsigned long long *nodes, unsigned long long *leaves,
                unsigned long long *depth, unsigned long long *hist, int max_levels) {
    verbose = 0;
    uts_parseParams(argc, argv);
    ref_stack_t s = {0};
    Node root;
    memset(&root, 0, sizeof(root));
    uts_initRoot(&root, type);
    push(&s, &root);
    unsigned long long nn = 0, nl = 0, md = 0;
    if (hist) memset(hist, 0, sizeof(unsigned long long) * (size_t)max_levels);
    while (s.n) {
        Node parent = s.v[--s.n];
        nn++;
        if (hist && parent.height < max_levels) hist[parent.height]++;
        if ((unsigned long long)parent.height > md) md = parent.height;
        int nc = uts_numChildren(&parent);
        int ct = uts_childType(&parent);
        if (nc > 0) {
            for (int i = 0; i < nc; i++) {
                Node child;
                memset(&child, 0, sizeof(child));
                child.type = ct;
                child.height = parent.height + 1;
                for (int j = 0; j < computeGranularity; j++)
                    rng_spawn(parent.state.state, child.state.state, i);
                push(&s, &child);
            }
        } else {
            nl++;
        }
    }
    free(s.v);
    *nodes = nn;
    *leaves = nl;
    *depth = md;
    return 0;
}

void ref_rng_init(int seed, unsigned char out[20]) { rng_init(out, seed); }

void ref_rng_spawn(const unsigned char parent[20], int i, unsigned char out[20]) {
    rng_spawn((RNG_state *)parent, out, i);
}

int ref_rng_rand(const unsigned char st[20]) { return rng_rand((RNG_state *)st); }

/* uts_numChildren for an explicit node, after ref_uts_set_params. */
int ref_uts_num_children(int node_type, int height, const unsigned char st[20]) {
    Node n;
    memset(&n, 0, sizeof(n));
    n.type = node_type;
    n.height = height;
    memcpy(n.state.state, st, 20);
    return uts_numChildren(&n);
}

void ref_uts_set_params(int argc, char **argv) {
    verbose = 0;
    uts_parseParams(argc, argv);
}
