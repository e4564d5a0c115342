/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
 *
 * CPU restatements of the remaining HClib hot-path workloads:
 *   - Smith-Waterman tiled DAG (test/smithwaterman/smith_waterman.cpp)
 *   - fib_iter (test/fib/fib.c:38-46)
 *   - forasync 1-D FLAT / RECURSIVE iteration sets (src/hclib.c:110-120,
 *     158-190, 316-351, 452-464)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* smith_waterman.cpp:6-9, 36-43 (GAP=-1, TRANSITION=-2, TRANSVERSION=-4, MATCH=2) */
static const signed char ora_sw_matrix[5][5] = {
    {-1, -1, -1, -1, -1},
    {-1, 2, -4, -2, -4},
    {-1, -4, 2, -4, -2},
    {-1, -2, -4, 2, -4},
    {-1, -4, -2, -4, 2},
};

/* clear_whitespaces_do_mapping + char_mapping, smith_waterman.cpp:13-59:
 * keep only A/C/G/T and map them to 1..4. Returns the mapped length. */
size_t ora_sw_map(const char *in, size_t n, signed char *out) {
    size_t k = 0;
    for (size_t i = 0; i < n; i++) {
        switch (in[i]) {
        case 'A': out[k++] = 1; break;
        case 'C': out[k++] = 2; break;
        case 'G': out[k++] = 3; break;
        case 'T': out[k++] = 4; break;
        default: break;
        }
    }
    return k;
}

/* The tiled DAG of smith_waterman.cpp:119-232 computes the single global
 * alignment matrix over the first (n1/tw)*tw x (n2/th)*th characters:
 * boundary row H[0][c] = -c, column H[r][0] = -r (the pre-put promises of
 * :141-165), interior H[r][c] = max(max(H[r][c-1]-1, H[r-1][c]-1),
 * H[r-1][c-1] + M[s2][s1]) (:201-210). The score is the bottom-right cell
 * (:239). This walks it row by row with O(width) memory.
 * last_row (optional, width+1 ints) receives H[rows][0..width];
 * last_col (optional, rows+1 ints) receives H[0..rows][width]. */
int ora_sw_score(const signed char *s1, size_t n1, const signed char *s2, size_t n2, int tw,
                 int th, int *last_row, int *last_col) {
    size_t ntw = n1 / (size_t)tw, nth = n2 / (size_t)th;
    size_t W = ntw * (size_t)tw, R = nth * (size_t)th;
    int *row = (int *)malloc((W + 1) * sizeof(int));
    if (!row) return 0;
    for (size_t c = 0; c <= W; c++) row[c] = -(int)c;
    if (last_col) last_col[0] = row[W];
    for (size_t r = 1; r <= R; r++) {
        int diag = row[0];
        row[0] = -(int)r;
        int left = row[0];
        const signed char *m = ora_sw_matrix[s2[r - 1]];
        for (size_t c = 1; c <= W; c++) {
            int up = row[c];
            int d = diag + m[s1[c - 1]];
            int l = left - 1;
            int u = up - 1;
            int lt = (l > u) ? l : u;
            int v = (lt > d) ? lt : d;
            row[c] = v;
            diag = up;
            left = v;
        }
        if (last_col) last_col[r] = row[W];
    }
    int score = row[W];
    if (last_row) memcpy(last_row, row, (W + 1) * sizeof(int));
    free(row);
    return score;
}

/* fib_iter, test/fib/fib.c:38-46 */
long ora_fib_iter(int n) {
    int i, x, y;
    for (i = 0, x = 1, y = 0; i <= n; i++) {
        int t = x;
        x = y;
        y += t;
    }
    return x;
}

/* forasync1D_runner (src/hclib.c:110-120): for i = low; i < high; i += stride */
static void run_tile(int low, int high, int stride, int base, int32_t *counts, int ncounts) {
    for (int i = low; i < high; i += stride) {
        long k = (long)i - base;
        if (k >= 0 && k < ncounts) counts[k]++;
    }
}

static void recursive(int low, int high, int stride, int tile, int base, int32_t *counts,
                      int ncounts) {
    /* forasync1D_recursive, src/hclib.c:158-190 */
    while ((high - low) > tile) {
        int mid = (high + low) / 2;
        recursive(mid, high, stride, tile, base, counts, ncounts);
        high = mid;
    }
    run_tile(low, high, stride, base, counts, ncounts);
}

/* Count how often each index in [base, base+ncounts) is visited by
 * hclib_forasync(dim=1) with the given domain and mode (0 FLAT, 1 RECURSIVE),
 * after the tile==-1 -> ceil((high-low)/nworkers) rule of src/hclib.c:452-464.
 * Returns the tile actually used. */
int ora_forasync1d_counts(int low, int high, int stride, int tile, int mode, int nworkers,
                          int base, int32_t *counts, int ncounts) {
    if (tile == -1) tile = ((high - low) + nworkers - 1) / nworkers;
    memset(counts, 0, sizeof(int32_t) * (size_t)ncounts);
    if (mode == 1) {
        recursive(low, high, stride, tile, base, counts, ncounts);
    } else {
        /* forasync1D_flat, src/hclib.c:316-351 (nb_chunks ignores low) */
        int nb_chunks = high / tile;
        int size = tile * nb_chunks;
        int low0;
        for (low0 = low; low0 < size; low0 += tile) run_tile(low0, low0 + tile, stride, base, counts, ncounts);
        if (size < high) run_tile(low0, high, stride, base, counts, ncounts);
    }
    return tile;
}
