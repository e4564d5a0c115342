// system_module.cpp — a third-party module, loaded from `deps`, on this build.
//
// The test harness compiles the reference's own modules/system/src/
// hclib_system.cpp, unmodified, against include/ into libhclib_system.so
// (tests/test_modules.py) and runs this program with HCLIB_MODULE_PATH
// pointing at it. hclib_launch(deps = {"system"}) must dlopen it
// (src/hclib-runtime.c:294-317), run its pre-init (locale types L1/L2/L3/
// sysmem) before the graph is built and its post-init (memory callbacks)
// after, so that:
//   * the default graph gains worker 0's private L1 locale ("L10") at the
//     front of its pop path (src/hclib-locality-graph.c:608-637);
//   * allocations at system memory go through the module's allocation_func,
//     whose first-touch memset leaves byte 0 = 42 (hclib_system.cpp:8-16);
//   * hclib::get_closest_cpu_locale() (defined by the module) finds L10.
#include <assert.h>
#include <string.h>

#include <iostream>

#include "hclib_cpp.h"

namespace hclib {
hclib::locale_t *get_closest_cpu_locale();  // modules/system/inc/hclib_system.h
}

int main() {
    const char *deps[] = {"system"};
    hclib::launch(deps, 1, [] {
        int n = 0;
        bool have[4] = {false, false, false, false};
        const char *want[4] = {"L1", "L2", "L3", "sysmem"};
        for (int t = 0; hclib_get_locale_type_name(t); ++t)
            for (int k = 0; k < 4; ++k) have[k] |= strcmp(hclib_get_locale_type_name(t), want[k]) == 0;
        for (int k = 0; k < 4; ++k) assert(have[k]);

        hclib::locale_t *closest = hclib::get_closest_locale();
        assert(strcmp(closest->lbl, "L10") == 0);
        assert(strcmp(hclib_get_locale_type_name(closest->type), "L1") == 0);
        assert(hclib::get_closest_cpu_locale() == closest);
        hclib_locale_t **priv = hclib_get_thread_private_locales();
        assert(priv[0] == closest);
        free(priv);
        // one host worker: its private L1 is also on every (its only) path
        assert(hclib_get_central_place() == closest);
        hclib_locale_t *sys = hclib_get_locale(0);
        assert(strcmp(sys->lbl, "sysmem") == 0);
        (void)n;

        // the module's allocation_func touches byte 0 with 42
        for (hclib::locale_t *l : {closest, sys}) {
            char *p = (char *)hclib::allocate_at(4096, l)->wait();
            assert(p && p[0] == 42);
            memset(p, 7, 4096);
            char *q = (char *)hclib::reallocate_at(p, 8192, l)->wait();
            assert(q && q[4095] == 7);
            hclib::memset_at(q, 3, 8192, l)->wait();
            assert(q[8191] == 3);
            char *r = (char *)hclib::allocate_at(8192, l)->wait();
            hclib::async_copy(l, r, l, q, 8192)->wait();
            assert(r[0] == 3 && r[8191] == 3);
            hclib::free_at(q, l);
            hclib::free_at(r, l);
        }
    });
    std::cout << "Check results: OK" << std::endl;
    return 0;
}
