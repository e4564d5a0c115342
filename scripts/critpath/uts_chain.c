/* Diagnostic (not product, not oracle): find one deepest root-to-leaf chain
 * of a BIN UTS tree (test/uts/uts.c BIN rules: the root has floor(b_0)
 * children, every other node m children when rand < q * 2^31) and write the
 * child index of each chain node within its parent, for the chain-stamp
 * build of the UTS kernel (HCLIB_HIP_UTS_TRACE=2, scripts/critpath/).
 *
 *   gcc -O2 -o uts_chain uts_chain.c && ./uts_chain out.bin [b0 q m r]
 *
 * out.bin: uint32 {D, k_1, ..., k_D}: chain node d is child k_d of node d-1.
 * SHA-1 is FIPS 180-4's block function; a node's child i is
 * SHA1(parent digest || i big-endian) (brg_sha1.c:68-83 rng_spawn). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void block(const uint32_t m[16], uint32_t out[5]) {
    uint32_t w[80];
    for (int t = 0; t < 16; ++t) w[t] = m[t];
    for (int t = 16; t < 80; ++t) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    const uint32_t iv[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    uint32_t a = iv[0], b = iv[1], c = iv[2], d = iv[3], e = iv[4];
    for (int t = 0; t < 80; ++t) {
        uint32_t f, k;
        if (t < 20) { f = (b & c) | (~b & d); k = 0x5a827999u; }
        else if (t < 40) { f = b ^ c ^ d; k = 0x6ed9eba1u; }
        else if (t < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdcu; }
        else { f = b ^ c ^ d; k = 0xca62c1d6u; }
        const uint32_t tmp = rol(a, 5) + f + e + k + w[t];
        e = d; d = c; c = rol(b, 30); b = a; a = tmp;
    }
    out[0] = iv[0] + a; out[1] = iv[1] + b; out[2] = iv[2] + c; out[3] = iv[3] + d; out[4] = iv[4] + e;
}

static void spawn(const uint32_t p[5], uint32_t i, uint32_t c[5]) {
    uint32_t m[16] = {0};
    memcpy(m, p, 20);
    m[5] = i; m[6] = 0x80000000u; m[15] = 192;
    block(m, c);
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s out.bin [b0 q m r]\n", argv[0]); return 2; }
    const double b0 = argc > 2 ? atof(argv[2]) : 2000.0, q = argc > 3 ? atof(argv[3]) : 0.200014;
    const int m = argc > 4 ? atoi(argv[4]) : 5, r = argc > 5 ? atoi(argv[5]) : 7;
    /* rand < q * 2^31 with rand = digest word 4 & 0x7fffffff (to_prob(rand) < q) */
    const uint32_t thr = (uint32_t)(q * 2147483648.0) + ((double)(uint32_t)(q * 2147483648.0) < q * 2147483648.0);
    enum { MAXD = 1 << 20 };
    uint32_t (*st)[5] = malloc(sizeof(uint32_t[5]) * MAXD);
    uint32_t *next = malloc(4 * MAXD), *nc = malloc(4 * MAXD), *best = malloc(4 * MAXD);
    {
        uint32_t msg[16] = {0};
        msg[4] = (uint32_t)r; msg[5] = 0x80000000u; msg[15] = 160;
        block(msg, st[0]);
    }
    nc[0] = (uint32_t)b0; next[0] = 0;
    long long nodes = 1, deepest_leaves = 0;
    int d = 0, maxd = 0;
    while (d >= 0) {
        if (next[d] == nc[d]) { --d; continue; }
        const uint32_t k = next[d]++;
        spawn(st[d], k, st[d + 1]);
        ++d; ++nodes;
        if (d + 1 >= MAXD) { fprintf(stderr, "too deep\n"); return 1; }
        nc[d] = ((st[d][4] & 0x7fffffffu) < thr) ? (uint32_t)m : 0u;
        next[d] = 0;
        if (d > maxd) { maxd = d; deepest_leaves = 0; for (int i = 1; i <= d; ++i) best[i] = next[i - 1] - 1; }
        if (d == maxd && nc[d] == 0) ++deepest_leaves;
    }
    best[0] = (uint32_t)maxd;
    FILE *f = fopen(argv[1], "wb");
    fwrite(best, 4, (size_t)maxd + 1, f);
    fclose(f);
    printf("{\"nodes\": %lld, \"max_depth\": %d, \"deepest_leaves\": %lld}\n", nodes, maxd, deepest_leaves);
    return 0;
}
