/* Locales and memory operations through include/hclib.h
 * (src/hclib-mem.c:23-241, inc/hclib.h:130-150): hclib_allocate_at /
 * reallocate_at / memset_at / free_at / async_copy as futures at a locale,
 * with the host ("sysmem") callbacks, and — with argument "gpu" — the GPU
 * locale's hipMalloc / hipMemsetAsync / hipMemcpyAsync callbacks
 * (the MI355X counterpart of modules/cuda/src/hclib_cuda.cpp:69-174),
 * including a copy whose source is a future
 * (HCLIB_ASYNC_COPY_USE_FUTURE_AS_SRC, src/hclib-mem.c:227-233).
 * Prints "Check results: OK". */
#define _GNU_SOURCE /* RTLD_DEFAULT */
#include <assert.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hclib.h"

static int use_gpu = 0;

static void *wait_ptr(hclib_future_t *f) { return hclib_future_wait(f); }

static void body(void *arg) {
    (void)arg;
    hclib_locale_t *host = hclib_get_locale(0);
    assert(host && hclib_get_closest_locale() == host);
    assert(strcmp(hclib_get_locale_type_name(hclib_get_locale_type(host)), "sysmem") == 0);
    assert(hclib_add_known_locale_type("sysmem") == hclib_get_locale_type(host));

    /* host locale */
    unsigned char *p = (unsigned char *)wait_ptr(hclib_allocate_at(1024, host));
    assert(p);
    hclib_future_wait(hclib_memset_at(p, 7, 1024, host));
    for (int i = 0; i < 1024; ++i) assert(p[i] == 7);
    p = (unsigned char *)wait_ptr(hclib_reallocate_at(p, 4096, host));
    for (int i = 0; i < 1024; ++i) assert(p[i] == 7);
    unsigned char *q = (unsigned char *)malloc(4096);
    memset(q, 0, 4096);
    hclib_future_wait(hclib_async_copy(host, q, host, p, 1024, NULL, 0));
    for (int i = 0; i < 1024; ++i) assert(q[i] == 7);
    hclib_free_at(p, host);

    if (use_gpu) {
        /* every GPU-locale operation below runs the hip plug-in module's
         * registered callbacks (libhclib_hip.so, loaded through deps) */
        void (*counts)(unsigned long long *) =
            (void (*)(unsigned long long *))dlsym(RTLD_DEFAULT, "hclib_hip_module_counts");
        assert(counts);
        unsigned long long c0[6], c1[6];
        counts(c0);
        int n = 0;
        hclib_locale_t **gpus = hclib_get_all_locales_of_type(hclib_add_known_locale_type("GPU"), &n);
        assert(n >= 1 && gpus[0] == hclib_get_locale(1));
        hclib_locale_t *g = gpus[0];
        free(gpus);
        const size_t N = 1 << 20;
        void *d = wait_ptr(hclib_allocate_at(N, g));
        assert(d);
        hclib_future_wait(hclib_memset_at(d, 0x5a, N, g));
        unsigned char *h = (unsigned char *)malloc(N);
        hclib_future_wait(hclib_async_copy(host, h, g, d, N, NULL, 0));
        for (size_t i = 0; i < N; ++i) assert(h[i] == 0x5a);
        /* host -> GPU -> host round trip, the second copy awaiting the first */
        unsigned char *h2 = (unsigned char *)malloc(N);
        for (size_t i = 0; i < N; ++i) h[i] = (unsigned char)(i * 7 + 3);
        hclib_future_t *up = hclib_async_copy(g, d, host, h, N, NULL, 0);
        hclib_future_wait(hclib_async_copy(host, h2, g, d, N, &up, 1));
        assert(memcmp(h, h2, N) == 0);
        /* reallocate keeps the prefix */
        d = wait_ptr(hclib_reallocate_at(d, 2 * N, g));
        memset(h2, 0, N);
        hclib_future_wait(hclib_async_copy(host, h2, g, d, N, NULL, 0));
        assert(memcmp(h, h2, N) == 0);
        /* the source of a copy given as a future (its value is the pointer) */
        hclib_promise_t *src = hclib_promise_create();
        hclib_future_t *sf = hclib_get_future_for_promise(src);
        memset(h2, 0, N);
        hclib_future_t *c = hclib_async_copy(host, h2, g, HCLIB_ASYNC_COPY_USE_FUTURE_AS_SRC, 4096, &sf, 1);
        hclib_promise_put(src, d);
        hclib_future_wait(c);
        assert(memcmp(h, h2, 4096) == 0);
        hclib_free_at(d, g);
        free(h);
        free(h2);
        counts(c1);
        /* 1 alloc, 1 realloc, 1 free, 1 memset, 5 copies */
        assert(c1[0] - c0[0] == 1 && c1[1] - c0[1] == 1 && c1[2] - c0[2] == 1 && c1[3] - c0[3] == 1 &&
               c1[4] - c0[4] == 5);
        printf("hip module callbacks: alloc %llu, realloc %llu, free %llu, memset %llu, copy %llu\n", c1[0], c1[1],
               c1[2], c1[3], c1[4]);
    }
    free(q);
}

int main(int argc, char **argv) {
    use_gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    const char *deps[] = {"system", "hip"};
    hclib_launch(body, NULL, deps, use_gpu ? 2 : 1);
    printf("Check results: OK\n");
    return 0;
}
