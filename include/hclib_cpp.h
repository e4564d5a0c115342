/*
 * hclib_cpp.h — HClib's C++ API (namespace hclib) over the MI355X build's
 * C API (include/hclib.h).
 *
 * Same names, signatures and semantics as the reference's header-only C++
 * layer, so test/cpp-style programs compile unchanged:
 *
 *   this header                                 reference
 *   ------------------------------------------  ------------------------------------
 *   hclib::launch(deps, n, f) / (nw, deps, n, f) inc/hclib_cpp.h:29-47
 *   hclib::async / async_at / async_nb(_at)     inc/hclib-async.h:161-246
 *   hclib::async_await(_at) (1-4 futures, vec)  inc/hclib-async.h:247-355
 *   hclib::async_future(_await)                 inc/hclib-async.h:356-545
 *   hclib::finish / nonblocking_finish          inc/hclib-async.h:550-566
 *   hclib::promise_t<T> / future_t<T>           inc/hclib_promise.h:42-121,
 *                                               inc/hclib_future.h:10-75
 *   hclib::loop_domain_{1,2,3}d, forasync{1,2,3}D(_nb, _future)
 *                                               inc/hclib-forasync.h:55-660
 *   get_num_workers / get_current_worker / get_closest_locale
 *                                               inc/hclib_cpp.h:49-60
 *
 * Lambdas are copied to the heap and run through one C trampoline per
 * lambda type, as the reference's lambda_wrapper does
 * (inc/hclib-async.h:64-150). Host lambdas run on the host control thread
 * (it executes host tasks help-first inside end_finish and
 * future_wait). GPU work is reached through device task kinds and loop
 * bodies (hclib.h) or, from HIP code, through hclib_hip_cpp.h (device
 * lambdas for forasync, user-defined device task kinds).
 */
#ifndef HCLIB_CPP_H_
#define HCLIB_CPP_H_

#include <stdio.h>
#include <stdlib.h>

#include <functional>
#include <type_traits>
#include <utility>
#include <vector>

#include "hclib.h"
#include "hclib_forasync_sets.h"

namespace hclib {

typedef hclib_locale_t locale_t;

// ------------------------------------------------------------ futures
// Trivial wrappers over hclib_future_t (inc/hclib_future.h:10-75): a
// future_t<T>* is a hclib_future_t* and back.
template <typename T>
struct future_t : public hclib_future_t {
    static_assert(sizeof(T) <= sizeof(void *), "future_t value type larger than a pointer");
    T get() {
        union { void *vp; T val; } u;
        u.vp = hclib_future_get(this);
        return u.val;
    }
    T wait() {
        union { void *vp; T val; } u;
        u.vp = hclib_future_wait(this);
        return u.val;
    }
    bool test() { return hclib_future_is_satisfied(this) != 0; }
};
template <typename T>
struct future_t<T *> : public hclib_future_t {
    T *get() { return static_cast<T *>(hclib_future_get(this)); }
    T *wait() { return static_cast<T *>(hclib_future_wait(this)); }
    bool test() { return hclib_future_is_satisfied(this) != 0; }
};
template <typename T>
struct future_t<T &> : public hclib_future_t {
    T &get() { return *static_cast<T *>(hclib_future_get(this)); }
    T &wait() { return *static_cast<T *>(hclib_future_wait(this)); }
    bool test() { return hclib_future_is_satisfied(this) != 0; }
};
template <>
struct future_t<void> : public hclib_future_t {
    void get() {}
    void wait() { hclib_future_wait(this); }
    bool test() { return hclib_future_is_satisfied(this) != 0; }
};
static_assert(sizeof(future_t<void *>) == sizeof(hclib_future_t), "future_t wraps hclib_future_t");

// ------------------------------------------------------------ promises
// inc/hclib_promise.h:42-121: values of at most pointer size travel in the
// promise's void* datum.
template <typename T>
struct promise_t : public hclib_promise_t {
    static_assert(sizeof(T) <= sizeof(void *), "promise_t value type larger than a pointer");
    static_assert(std::is_trivially_copyable<T>::value, "promise_t value type must be trivially copyable");
    promise_t() { hclib_promise_init(this); }
    void put(T datum) {
        union { void *vp; T val; } u;
        u.vp = nullptr;
        u.val = datum;
        hclib_promise_put(this, u.vp);
    }
    future_t<T> *get_future() {
        return static_cast<future_t<T> *>(&static_cast<hclib_promise_t *>(this)->future);
    }
    future_t<T> &future() { return *get_future(); }
};
template <typename T>
struct promise_t<T *> : public hclib_promise_t {
    promise_t() { hclib_promise_init(this); }
    void put(T *datum) { hclib_promise_put(this, (void *)datum); }
    future_t<T *> *get_future() {
        return static_cast<future_t<T *> *>(&static_cast<hclib_promise_t *>(this)->future);
    }
    future_t<T *> &future() { return *get_future(); }
};
template <typename T>
struct promise_t<T &> : public hclib_promise_t {
    promise_t() { hclib_promise_init(this); }
    void put(T &datum) { hclib_promise_put(this, (void *)&datum); }
    future_t<T &> *get_future() {
        return static_cast<future_t<T &> *>(&static_cast<hclib_promise_t *>(this)->future);
    }
    future_t<T &> &future() { return *get_future(); }
};
template <>
struct promise_t<void> : public hclib_promise_t {
    promise_t() { hclib_promise_init(this); }
    void put() { hclib_promise_put(this, nullptr); }
    future_t<void> *get_future() {
        return static_cast<future_t<void> *>(&static_cast<hclib_promise_t *>(this)->future);
    }
    future_t<void> &future() { return *get_future(); }
};

// ------------------------------------------------------------- lambdas
namespace detail {

// lambda_wrapper + call_lambda, inc/hclib-async.h:64-98
template <typename U>
void call_and_delete(void *p) {
    U *f = static_cast<U *>(p);
    (*f)();
    delete f;
}

template <typename T>
inline void spawn(T &&lambda, hclib_future_t **futures, int nfutures, hclib_locale_t *locale) {
    typedef typename std::remove_cv<typename std::remove_reference<T>::type>::type U;
    U *heap = new U(std::forward<T>(lambda));
    hclib_async(call_and_delete<U>, heap, futures, nfutures, locale);
}

}  // namespace detail

// ----------------------------------------------------------- lifecycle
inline void init(const char **deps, int ndeps, const int instrument) { hclib_init(deps, ndeps, instrument); }
inline void finalize(const int instrument) { hclib_finalize(instrument); }

template <typename T>
inline void launch(const char **deps, int ndeps, T &&lambda) {
    typedef typename std::remove_cv<typename std::remove_reference<T>::type>::type U;
    hclib_launch(detail::call_and_delete<U>, new U(std::forward<T>(lambda)), deps, ndeps);
}

template <typename T>
inline void launch(const int nworkers, const char **deps, int ndeps, T &&lambda) {
    char buf[32];
    snprintf(buf, sizeof(buf), "%d", nworkers);
    setenv("HCLIB_WORKERS", buf, 1);  // inc/hclib_cpp.h:38-46
    launch(deps, ndeps, std::forward<T>(lambda));
}

inline int get_current_worker() { return hclib_get_current_worker(); }
// inc/hclib_cpp.h:49-58 (src/hclib_cpp.cpp)
inline hclib_worker_state *current_ws() { return ::current_ws(); }
inline locale_t **get_thread_private_locales() { return hclib_get_thread_private_locales(); }
inline locale_t *get_master_place() { return hclib_get_master_place(); }
inline int get_num_workers() { return hclib_get_num_workers(); }
inline locale_t *get_closest_locale() { return hclib_get_closest_locale(); }
// inc/hclib_cpp.h:53-57
inline int get_num_locales() { return hclib_get_num_locales(); }
inline locale_t *get_all_locales() { return hclib_get_all_locales(); }
inline locale_t **get_all_locales_of_type(int type, int *out_count) {
    return hclib_get_all_locales_of_type(type, out_count);
}
// inc/hclib-async.h:564-571
inline void yield() { hclib_yield(NULL); }
inline void yield_at(locale_t *locale) { hclib_yield(locale); }
inline unsigned long long current_time_ns() { return hclib_current_time_ns(); }

// --------------------------------------------------------------- async
template <typename T>
inline void async(T &&lambda) { detail::spawn(std::forward<T>(lambda), nullptr, 0, nullptr); }
template <typename T>
inline void async_at(T &&lambda, hclib_locale_t *locale) {
    detail::spawn(std::forward<T>(lambda), nullptr, 0, locale);
}
// a non-blocking async never blocks, so it is a plain async here
// (inc/hclib-async.h:175-246)
template <typename T>
inline void async_nb(T &&lambda) { async(std::forward<T>(lambda)); }
template <typename T>
inline void async_nb_at(T &&lambda, hclib_locale_t *locale) { async_at(std::forward<T>(lambda), locale); }

template <typename T>
inline void async_await_at(T &&lambda, hclib_future_t *f, hclib_locale_t *locale) {
    hclib_future_t *fs[1] = {f};
    detail::spawn(std::forward<T>(lambda), f ? fs : nullptr, f ? 1 : 0, locale);
}
template <typename T>
inline void async_await(T &&lambda, hclib_future_t *f) { async_await_at(std::forward<T>(lambda), f, nullptr); }
template <typename T>
inline void async_await(T &&lambda, hclib_future_t *f1, hclib_future_t *f2) {
    hclib_future_t *fs[2] = {f1, f2};
    detail::spawn(std::forward<T>(lambda), fs, 2, nullptr);
}
template <typename T>
inline void async_await(T &&lambda, hclib_future_t *f1, hclib_future_t *f2, hclib_future_t *f3) {
    hclib_future_t *fs[3] = {f1, f2, f3};
    detail::spawn(std::forward<T>(lambda), fs, 3, nullptr);
}
template <typename T>
inline void async_await(T &&lambda, hclib_future_t *f1, hclib_future_t *f2, hclib_future_t *f3,
                        hclib_future_t *f4) {
    hclib_future_t *fs[4] = {f1, f2, f3, f4};
    detail::spawn(std::forward<T>(lambda), fs, 4, nullptr);
}
template <typename T>
inline void async_await(T &&lambda, std::vector<hclib_future_t *> &futures) {
    detail::spawn(std::forward<T>(lambda), futures.data(), (int)futures.size(), nullptr);
}
template <typename T>
inline void async_await(T &&lambda, std::vector<hclib_future_t *> &&futures) {
    detail::spawn(std::forward<T>(lambda), futures.data(), (int)futures.size(), nullptr);
}
template <typename T>
inline void async_await(T &&lambda, std::vector<hclib_future_t *> *futures) {
    detail::spawn(std::forward<T>(lambda), futures->data(), (int)futures->size(), nullptr);
}
template <typename T>
inline void async_nb_await(T &&lambda, hclib_future_t *f) { async_await(std::forward<T>(lambda), f); }
template <typename T>
inline void async_nb_await(T &&lambda, std::vector<hclib_future_t *> &futures) {
    async_await(std::forward<T>(lambda), futures);
}

// async_future: run the lambda, put its result into a fresh promise
// (inc/hclib-async.h:356-440; a void lambda puts nullptr)
namespace detail {
template <typename R>
struct future_putter {
    template <typename F>
    static void run(promise_t<R> *p, F &f) { p->put(f()); }
};
template <>
struct future_putter<void> {
    template <typename F>
    static void run(promise_t<void> *p, F &f) {
        f();
        p->put();
    }
};
template <typename T>
inline auto async_future_helper(T &&lambda, hclib_future_t **futures, int n, hclib_locale_t *locale)
    -> future_t<decltype(lambda())> * {
    typedef decltype(lambda()) R;
    typedef typename std::remove_cv<typename std::remove_reference<T>::type>::type U;
    promise_t<R> *p = new promise_t<R>();
    U f(std::forward<T>(lambda));
    spawn([p, f]() mutable { future_putter<R>::run(p, f); }, futures, n, locale);
    return p->get_future();
}
}  // namespace detail

template <typename T>
inline auto async_future(T &&lambda) -> future_t<decltype(lambda())> * {
    return detail::async_future_helper(std::forward<T>(lambda), nullptr, 0, nullptr);
}
template <typename T>
inline auto async_future_at(T &&lambda, hclib_locale_t *locale) -> future_t<decltype(lambda())> * {
    return detail::async_future_helper(std::forward<T>(lambda), nullptr, 0, locale);
}
template <typename T>
inline auto async_future_await(T &&lambda, hclib_future_t *f) -> future_t<decltype(lambda())> * {
    hclib_future_t *fs[1] = {f};
    return detail::async_future_helper(std::forward<T>(lambda), f ? fs : nullptr, f ? 1 : 0, nullptr);
}
template <typename T>
inline auto async_future_await(T &&lambda, std::vector<hclib_future_t *> &futures)
    -> future_t<decltype(lambda())> * {
    return detail::async_future_helper(std::forward<T>(lambda), futures.data(), (int)futures.size(),
                                       nullptr);
}

// inc/hclib-async.h:515-547
template <typename T>
inline auto async_future_await_at(T &&lambda, hclib_future_t *f, hclib_locale_t *locale)
    -> future_t<decltype(lambda())> * {
    hclib_future_t *fs[1] = {f};
    return detail::async_future_helper(std::forward<T>(lambda), f ? fs : nullptr, f ? 1 : 0, locale);
}
template <typename T>
inline auto async_future_await_at(T &&lambda, std::vector<hclib_future_t *> &futures, hclib_locale_t *locale)
    -> future_t<decltype(lambda())> * {
    return detail::async_future_helper(std::forward<T>(lambda), futures.data(), (int)futures.size(), locale);
}
template <typename T>
inline auto async_future_await_at(T &&lambda, std::vector<hclib_future_t *> &&futures, hclib_locale_t *locale)
    -> future_t<decltype(lambda())> * {
    return detail::async_future_helper(std::forward<T>(lambda), futures.data(), (int)futures.size(), locale);
}

// ------------------------------------------------------ memory at locales
// inc/hclib_cpp.h:58-80 (src/hclib-mem.c behind them)
inline future_t<void *> *allocate_at(size_t nbytes, locale_t *locale) {
    return static_cast<future_t<void *> *>(hclib_allocate_at(nbytes, locale));
}
inline future_t<void *> *reallocate_at(void *ptr, size_t nbytes, locale_t *locale) {
    return static_cast<future_t<void *> *>(hclib_reallocate_at(ptr, nbytes, locale));
}
inline void free_at(void *ptr, locale_t *locale) { hclib_free_at(ptr, locale); }
inline future_t<void *> *memset_at(void *ptr, int pattern, size_t nbytes, locale_t *locale) {
    return static_cast<future_t<void *> *>(hclib_memset_at(ptr, pattern, nbytes, locale));
}
inline future_t<void *> *async_copy(locale_t *dst_locale, void *dst, locale_t *src_locale, void *src,
                                    size_t nbytes) {
    return static_cast<future_t<void *> *>(hclib_async_copy(dst_locale, dst, src_locale, src, nbytes, NULL, 0));
}
inline future_t<void *> *async_copy_await(locale_t *dst_locale, void *dst, locale_t *src_locale, void *src,
                                          size_t nbytes, hclib_future_t *future) {
    return static_cast<future_t<void *> *>(
        hclib_async_copy(dst_locale, dst, src_locale, src, nbytes, future ? &future : NULL, future ? 1 : 0));
}

// -------------------------------------------------------------- finish
inline void finish(std::function<void()> &&lambda) {  // inc/hclib-async.h:550-554
    hclib_start_finish();
    lambda();
    hclib_end_finish();
}

inline future_t<void> *nonblocking_finish(std::function<void()> &&lambda) {  // :556-566
    hclib_start_finish();
    lambda();
    promise_t<void> *event = new promise_t<void>();
    hclib_end_finish_nonblocking_helper(event);
    return event->get_future();
}

// ------------------------------------------------------------- forasync
inline int default_tile_size(const int n, const int nchunks) { return (n + nchunks - 1) / nchunks; }

class loop_domain_1d {  // inc/hclib-forasync.h:60-85
    hclib_loop_domain_t loop;

public:
    loop_domain_1d(int N) : loop{0, N, 1, default_tile_size(N, hclib_get_num_workers())} {}
    loop_domain_1d(int low, int high)
        : loop{low, high, 1, default_tile_size(high - low, hclib_get_num_workers())} {}
    loop_domain_1d(int low, int high, int nchunks)
        : loop{low, high, 1, default_tile_size(high - low, nchunks)} {}
    loop_domain_1d(int low, int high, int nchunks, int stride)
        : loop{low, high, stride, default_tile_size(high - low, nchunks)} {}
    hclib_loop_domain_t *get_internal() { return &loop; }
};

class loop_domain_2d {  // inc/hclib-forasync.h:87-112
    hclib_loop_domain_t loop[2];

public:
    loop_domain_2d(int N1, int N2) : loop_domain_2d(0, N1, 0, N2) {}
    loop_domain_2d(int low1, int high1, int low2, int high2) {
        loop[0] = {low1, high1, 1, default_tile_size(high1 - low1, hclib_get_num_workers())};
        loop[1] = {low2, high2, 1, default_tile_size(high2 - low2, hclib_get_num_workers())};
    }
    hclib_loop_domain_t *get_internal() { return loop; }
};

class loop_domain_3d {  // inc/hclib-forasync.h:114-148
    hclib_loop_domain_t loop[3];

public:
    loop_domain_3d(int N1, int N2, int N3) : loop_domain_3d(0, N1, 0, N2, 0, N3) {}
    loop_domain_3d(int low1, int high1, int low2, int high2, int low3, int high3) {
        const int nw = hclib_get_num_workers();
        loop[0] = {low1, high1, 1, default_tile_size(high1 - low1, nw)};
        loop[1] = {low2, high2, 1, default_tile_size(high2 - low2, nw)};
        loop[2] = {low3, high3, 1, default_tile_size(high3 - low3, nw)};
    }
    loop_domain_3d(int low1, int high1, int tile1, int low2, int high2, int tile2, int low3, int high3,
                   int tile3) {
        loop[0] = {low1, high1, 1, tile1};
        loop[1] = {low2, high2, 1, tile2};
        loop[2] = {low3, high3, 1, tile3};
    }
    hclib_loop_domain_t *get_internal() { return loop; }
};

namespace detail {

inline std::vector<hclib_sets::Run> dim_runs(hclib_loop_domain_t *d, int ndim, int mode) {
    hclib_sets::resolve_tile(&d->tile, d->low, d->high, hclib_get_num_workers());
    const hclib_sets::Domain dd{d->low, d->high, d->stride, d->tile};
    return hclib_sets::runs(dd, ndim, mode);
}

template <typename B>
inline void tile_task(B &&body, hclib_future_t *future) {
    if (future) async_await(std::forward<B>(body), future);
    else async(std::forward<B>(body));
}

// One host task per run of reference tiles; each runs its indices in order
// like forasync{1,2,3}D_runner (src/hclib.c:110-156).
template <typename T>
inline void tasks1(hclib_loop_domain_t *loop, T lambda, int mode, hclib_future_t *future) {
    for (const hclib_sets::Run a : dim_runs(&loop[0], 1, mode))
        tile_task([=]() {
            for (int i = 0, x = a.first; i < a.count; ++i, x += a.stride) lambda(x);
        }, future);
}
template <typename T>
inline void tasks2(hclib_loop_domain_t *loop, T lambda, int mode, hclib_future_t *future) {
    const std::vector<hclib_sets::Run> r0 = dim_runs(&loop[0], 2, mode), r1 = dim_runs(&loop[1], 2, mode);
    for (const hclib_sets::Run a : r0)
        for (const hclib_sets::Run b : r1)
            tile_task([=]() {
                for (int i = 0, x = a.first; i < a.count; ++i, x += a.stride)
                    for (int j = 0, y = b.first; j < b.count; ++j, y += b.stride) lambda(x, y);
            }, future);
}
template <typename T>
inline void tasks3(hclib_loop_domain_t *loop, T lambda, int mode, hclib_future_t *future) {
    const std::vector<hclib_sets::Run> r0 = dim_runs(&loop[0], 3, mode), r1 = dim_runs(&loop[1], 3, mode),
                                       r2 = dim_runs(&loop[2], 3, mode);
    for (const hclib_sets::Run a : r0)
        for (const hclib_sets::Run b : r1)
            for (const hclib_sets::Run c : r2)
                tile_task([=]() {
                    for (int i = 0, x = a.first; i < a.count; ++i, x += a.stride)
                        for (int j = 0, y = b.first; j < b.count; ++j, y += b.stride)
                            for (int k = 0, z = c.first; k < c.count; ++k, z += c.stride) lambda(x, y, z);
                }, future);
}

}  // namespace detail

template <typename T>
inline void forasync1D_seq(loop_domain_1d *loop, T lambda) {
    const hclib_loop_domain_t *d = loop->get_internal();
    for (int i = d->low; i < d->high; i += d->stride) lambda(i);
}
template <typename T>
inline void forasync1D_nb(loop_domain_1d *loop, T lambda, bool force_seq = false,
                          int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    if (force_seq) return forasync1D_seq(loop, lambda);
    detail::tasks1(loop->get_internal(), lambda, mode, future);
}
template <typename T>
inline void forasync1D(loop_domain_1d *loop, T lambda, bool force_seq = false,
                       int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    if (force_seq) return forasync1D_seq(loop, lambda);
    finish([&]() { forasync1D_nb(loop, lambda, false, mode, future); });
}
template <typename T>
inline future_t<void> *forasync1D_future(loop_domain_1d *loop, T lambda, bool force_seq = false,
                                         int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    return nonblocking_finish([&]() { forasync1D_nb(loop, lambda, force_seq, mode, future); });
}

template <typename T>
inline void forasync2D_seq(loop_domain_2d *loop, T lambda) {
    const hclib_loop_domain_t *d = loop->get_internal();
    for (int i = d[0].low; i < d[0].high; i += d[0].stride)
        for (int j = d[1].low; j < d[1].high; j += d[1].stride) lambda(i, j);
}
template <typename T>
inline void forasync2D_nb(loop_domain_2d *loop, T lambda, bool force_seq = false,
                          int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    if (force_seq) return forasync2D_seq(loop, lambda);
    detail::tasks2(loop->get_internal(), lambda, mode, future);
}
template <typename T>
inline void forasync2D(loop_domain_2d *loop, T lambda, bool force_seq = false,
                       int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    if (force_seq) return forasync2D_seq(loop, lambda);
    finish([&]() { forasync2D_nb(loop, lambda, false, mode, future); });
}
template <typename T>
inline future_t<void> *forasync2D_future(loop_domain_2d *loop, T lambda, bool force_seq = false,
                                         int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    return nonblocking_finish([&]() { forasync2D_nb(loop, lambda, force_seq, mode, future); });
}

template <typename T>
inline void forasync3D_seq(loop_domain_3d *loop, T lambda) {
    const hclib_loop_domain_t *d = loop->get_internal();
    for (int i = d[0].low; i < d[0].high; i += d[0].stride)
        for (int j = d[1].low; j < d[1].high; j += d[1].stride)
            for (int k = d[2].low; k < d[2].high; k += d[2].stride) lambda(i, j, k);
}
template <typename T>
inline void forasync3D_nb(loop_domain_3d *loop, T lambda, bool force_seq = false,
                          int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    if (force_seq) return forasync3D_seq(loop, lambda);
    detail::tasks3(loop->get_internal(), lambda, mode, future);
}
template <typename T>
inline void forasync3D(loop_domain_3d *loop, T lambda, bool force_seq = false,
                       int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    if (force_seq) return forasync3D_seq(loop, lambda);
    finish([&]() { forasync3D_nb(loop, lambda, false, mode, future); });
}
template <typename T>
inline future_t<void> *forasync3D_future(loop_domain_3d *loop, T lambda, bool force_seq = false,
                                         int mode = FORASYNC_MODE_RECURSIVE, hclib_future_t *future = NULL) {
    return nonblocking_finish([&]() { forasync3D_nb(loop, lambda, force_seq, mode, future); });
}

}  // namespace hclib

#endif  // HCLIB_CPP_H_
