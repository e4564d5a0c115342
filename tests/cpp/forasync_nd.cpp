// hclib::forasync{1,2,3}D over host lambdas, FLAT and RECURSIVE, through
// include/hclib_cpp.h. Every index must be visited exactly as often as the
// reference's tiling visits it: restated here independently of the header
// by direct recursion over the reference's task structure
// (forasync1D_flat / _recursive / _runner, src/hclib.c:110-190, 316-351;
// 2-D/3-D: every index exactly once, src/hclib.c:353-416). Checks follow
// test/cpp/forasync{1D,2D,3D}{Ch,Rec}.cpp (assert ran[i] == -1; ran[i] = i).
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hclib_cpp.h"

// reference tiling, as visit counts over [0, ext)
static void ref_runner(int low, int high, int stride, std::vector<int> &cnt) {
    for (int i = low; i < high; i += stride) cnt[i]++;
}
static void ref_recursive(int low, int high, int stride, int tile, std::vector<int> &cnt) {
    if ((high - low) > tile) {
        int mid = (high + low) / 2;
        ref_recursive(mid, high, stride, tile, cnt);  // the spawned upper half
        ref_recursive(low, mid, stride, tile, cnt);
    } else {
        ref_runner(low, high, stride, cnt);
    }
}
static void ref_flat1d(int low, int high, int stride, int tile, std::vector<int> &cnt) {
    int nb_chunks = high / tile, size = tile * nb_chunks, low0;
    for (low0 = low; low0 < size; low0 += tile) ref_runner(low0, low0 + tile, stride, cnt);
    if (size < high) ref_runner(low0, high, stride, cnt);
}
static void check1d(int low, int high, int nchunks, int stride, int mode) {
    const int ext = high + 256;
    std::vector<int> want(ext, 0), got(ext, 0);
    hclib::loop_domain_1d dom(low, high, nchunks, stride);
    const int tile = dom.get_internal()->tile;
    if (mode == FORASYNC_MODE_RECURSIVE) ref_recursive(low, high, stride, tile, want);
    else ref_flat1d(low, high, stride, tile, want);
    int *g = got.data();
    hclib::forasync1D(&dom, [=](int i) { g[i]++; }, false, mode);
    assert(memcmp(want.data(), got.data(), ext * sizeof(int)) == 0);
}

int main() {
    const char *deps[] = {"system"};
    hclib::launch(deps, 1, [&]() {
        // 1-D, FLAT and RECURSIVE, including the FLAT low != 0 overrun quirk
        // (domain {10, 100, 1, 33} runs indices 10..108)
        const int cases[][4] = {{0, 1000, 7, 1}, {0, 1024, 8, 1}, {10, 100, 3, 1}, {5, 777, 13, 3}, {0, 1, 4, 1}};
        for (auto &c : cases)
            for (int mode : {FORASYNC_MODE_FLAT, FORASYNC_MODE_RECURSIVE}) check1d(c[0], c[1], c[2], c[3], mode);
        {
            std::vector<int> got(256, 0);
            int *g = got.data();
            hclib::loop_domain_1d dom(10, 100, 3, 1);
            dom.get_internal()->tile = 33;
            hclib::forasync1D(&dom, [=](int i) { g[i]++; }, false, FORASYNC_MODE_FLAT);
            for (int i = 0; i < 256; ++i) assert(got[i] == ((i >= 10 && i <= 108) ? 1 : 0));
        }
        // 2-D (test/cpp/forasync2DRec.cpp / 2DCh.cpp shape, smaller)
        for (int mode : {FORASYNC_MODE_FLAT, FORASYNC_MODE_RECURSIVE}) {
            const int H1 = 96, H2 = 40;
            int *ran = (int *)malloc(H1 * H2 * sizeof(int));
            for (int i = 0; i < H1 * H2; ++i) ran[i] = -1;
            hclib::loop_domain_2d dom(H1, H2);
            dom.get_internal()[0].tile = 11;
            dom.get_internal()[1].tile = 7;
            hclib::forasync2D(&dom, [=](int a, int b) {
                assert(ran[a * H2 + b] == -1);
                ran[a * H2 + b] = a * H2 + b;
            }, false, mode);
            for (int i = 0; i < H1 * H2; ++i) assert(ran[i] == i);
            free(ran);
        }
        // 3-D with explicit tiles (test/cpp/forasync3DCh.cpp shape, smaller)
        for (int mode : {FORASYNC_MODE_FLAT, FORASYNC_MODE_RECURSIVE}) {
            const int H1 = 12, H2 = 10, H3 = 9;
            int *ran = (int *)malloc(H1 * H2 * H3 * sizeof(int));
            for (int i = 0; i < H1 * H2 * H3; ++i) ran[i] = -1;
            hclib::loop_domain_3d dom(0, H1, 5, 0, H2, 3, 0, H3, 4);
            hclib::forasync3D(&dom, [=](int a, int b, int c) {
                const int k = (a * H2 + b) * H3 + c;
                assert(ran[k] == -1);
                ran[k] = k;
            }, false, mode);
            for (int i = 0; i < H1 * H2 * H3; ++i) assert(ran[i] == i);
            free(ran);
        }
        // forasync1D_future (test/cpp/promise/future3.cpp shape)
        {
            const int H = 256;
            int *ran = new int[H];
            for (int i = 0; i < H; ++i) ran[i] = -1;
            hclib::loop_domain_1d dom(0, H, 16);
            hclib::future_t<void> *ev = hclib::forasync1D_future(&dom, [=](int i) {
                assert(ran[i] == -1);
                ran[i] = i;
            });
            ev->wait();
            for (int i = 0; i < H; ++i) assert(ran[i] == i);
            delete[] ran;
        }
    });
    printf("Check results: OK\n");
    return 0;
}
