// promise_t / future_t / async_await / async_future / nonblocking_finish over
// host lambdas through include/hclib_cpp.h. Restates the checks of the
// reference's test/cpp/nested_finish_async_await.cpp (rounds of tiles, each
// awaiting its neighbours' futures), test/cpp/promise/asyncAwait0Vector.cpp
// (a chain of asyncs each awaiting the previous promise, built back to
// front), test/cpp/promise/future0Int.cpp (values by value) and
// async_future(_await) (inc/hclib-async.h:356-545).
#include <assert.h>
#include <stdio.h>

#include <vector>

#include "hclib_cpp.h"

int main() {
    const char *deps[] = {"system"};
    int order_ok = 1, chain_out = -1, fut_sum = 0, nb_ran = 0, rounds_done = 0;
    hclib::launch(deps, 1, [&]() {
        // nested_finish_async_await: n_rounds x n_tiles promises
        const int n_rounds = 20, n_tiles = 5;
        auto tile = new hclib::promise_t<void *> **[n_rounds + 1];
        for (int t = 0; t <= n_rounds; ++t) {
            tile[t] = new hclib::promise_t<void *> *[n_tiles];
            for (int j = 0; j < n_tiles; ++j) tile[t][j] = new hclib::promise_t<void *>();
        }
        for (int j = 0; j < n_tiles; ++j) tile[0][j]->put(nullptr);
        int *done = &rounds_done;
        hclib::finish([=]() {
            for (int t = 0; t < n_rounds; ++t)
                for (int j = 0; j < n_tiles; ++j) {
                    const int l = (n_tiles + j - 1) % n_tiles, r = (j + 1) % n_tiles;
                    hclib::async_await([=]() {
                        hclib::finish([=]() {
                            hclib::async_await([=]() {
                                tile[t + 1][j]->put(nullptr);
                                if (j == 0) (*done)++;
                            }, tile[t][l]->get_future());
                        });
                    }, tile[t][l]->get_future(), tile[t][r]->get_future());
                }
        });
        for (int j = 0; j < n_tiles; ++j) assert(tile[n_rounds][j]->get_future()->test());

        // asyncAwait0Vector: chain built back to front, started by promise 0
        const int n = 10;
        hclib::promise_t<int *> **plist = new hclib::promise_t<int *> *[n + 1];
        for (int i = 0; i <= n; ++i) plist[i] = new hclib::promise_t<int *>();
        int *ok = &order_ok;
        hclib::finish([=]() {
            for (int index = n; index >= 1; index--) {
                std::vector<hclib_future_t *> fv;
                fv.push_back(plist[index - 1]->get_future());
                hclib::async_await([=]() {
                    int *input = plist[index - 1]->get_future()->get();
                    if (*input != index - 1) *ok = 0;
                    plist[index]->put(new int(index));
                }, fv);
            }
            plist[0]->put(new int(0));
        });
        chain_out = *plist[n]->get_future()->get();
        for (int i = 0; i <= n; ++i) {
            delete plist[i]->future().get();
            delete plist[i];
        }
        delete[] plist;

        // values by value, async_future and async_future_await
        hclib::promise_t<int> pi;
        hclib::future_t<int> *a = hclib::async_future([]() { return 20; });
        hclib::future_t<int> *b = hclib::async_future_await([a]() { return a->get() + 1; }, a);
        hclib::async([&pi]() { pi.put(21); });
        int *fs = &fut_sum;
        hclib::finish([=, &pi]() {
            hclib::async_await([=, &pi]() { *fs = b->get() + pi.get_future()->get(); },
                               b, pi.get_future());
        });
        hclib::future_t<void> *v = hclib::async_future([]() {});
        v->wait();

        // nonblocking_finish: the future is put when the scope drains
        int *nr = &nb_ran;
        hclib::future_t<void> *ev = hclib::nonblocking_finish([=]() {
            for (int i = 0; i < 8; ++i) hclib::async([=]() { (*nr)++; });
        });
        ev->wait();
    });
    printf("Check results: ");
    assert(rounds_done == 20);
    assert(order_ok == 1 && chain_out == 10);
    assert(fut_sum == 42);
    assert(nb_ran == 8);
    printf("OK\n");
    return 0;
}
