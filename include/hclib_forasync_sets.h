/*
 * hclib_forasync_sets.h — the exact iteration sets of hclib_forasync.
 *
 * The reference tiles a forasync into tasks and runs each tile with
 * `for (i = low; i < high; i += stride) fn(i)` (forasync1D_runner,
 * src/hclib.c:110-120). This header describes the union of those tiles, per
 * dimension, as runs {first, count, stride} in index order, so that a launch
 * (or the host C++ layer) can sweep exactly the reference's iterations:
 *
 *   mode       dim   reference                           rule
 *   ---------  ----  ----------------------------------  -----------------------------
 *   FLAT       1     forasync1D_flat, src/hclib.c:316-351 chunks counted from 0:
 *                                                        nb_chunks = high / tile, so
 *                                                        with low != 0 the last full
 *                                                        chunk can overrun `high`
 *                                                        (kept)
 *   FLAT       2, 3  forasync2D/3D_flat, src/hclib.c:353-416  tiles [low, min(low+tile, high))
 *   RECURSIVE  any   forasync{1,2,3}D_recursive,          bisection at (high+low)/2 until
 *                    src/hclib.c:158-314                  high-low <= tile
 *
 * tile == -1 means "auto": ceil((high-low)/nworkers), written back into the
 * caller's domain (src/hclib.c:452-461). Host-only, header-only C++.
 */
#ifndef HCLIB_FORASYNC_SETS_H_
#define HCLIB_FORASYNC_SETS_H_

#include <stdint.h>

#include <vector>

namespace hclib_sets {

struct Run {
    int first;
    int count;
    int stride;
    int pad;
};

struct Domain {  // hclib_loop_domain_t (inc/hclib-task.h:53-58)
    int low, high, stride, tile;
};

inline void add_run(std::vector<Run> &v, int lo, int hi, int stride) {
    if (hi <= lo) return;
    const int cnt = (int)(((int64_t)hi - lo + stride - 1) / stride);
    if (!v.empty() && stride == 1 && v.back().stride == 1 && v.back().first + v.back().count == lo) {
        v.back().count += cnt;  // contiguous unit-stride tiles merge
        return;
    }
    v.push_back(Run{lo, cnt, stride, 0});
}

// forasync1D_flat, src/hclib.c:316-351
inline void flat1d(const Domain &d, std::vector<Run> &v) {
    const int nb_chunks = d.high / d.tile;
    const int size = d.tile * nb_chunks;
    int low0;
    for (low0 = d.low; low0 < size; low0 += d.tile) add_run(v, low0, low0 + d.tile, d.stride);
    if (size < d.high) add_run(v, low0, d.high, d.stride);
}

// per-dimension tiles of forasync2D/3D_flat, src/hclib.c:353-416
inline void flat_nd(const Domain &d, std::vector<Run> &v) {
    for (int low0 = d.low; low0 < d.high; low0 += d.tile) {
        const int high0 = (low0 + d.tile) > d.high ? d.high : (low0 + d.tile);
        add_run(v, low0, high0, d.stride);
    }
}

// forasync{1,2,3}D_recursive, src/hclib.c:158-314 (leaves in index order)
inline void recursive(int low, int high, const Domain &d, std::vector<Run> &v) {
    if ((high - low) > d.tile) {
        const int mid = (high + low) / 2;
        recursive(low, mid, d, v);
        recursive(mid, high, d, v);
    } else {
        add_run(v, low, high, d.stride);
    }
}

// The runs of dimension `dim` (0-based) of a `ndim`-D forasync in `mode`
// (0 FLAT, 1 RECURSIVE). The domain's tile must already be resolved (>= 1).
inline std::vector<Run> runs(const Domain &d, int ndim, int mode) {
    std::vector<Run> v;
    if (mode == 1) recursive(d.low, d.high, d, v);
    else if (ndim == 1) flat1d(d, v);
    else flat_nd(d, v);
    return v;
}

// Resolve tile == -1 (auto) like src/hclib.c:455-461; tiles < 1 become 1.
inline void resolve_tile(int *tile, int low, int high, int nworkers) {
    if (*tile == -1) *tile = ((high - low) + nworkers - 1) / nworkers;
    if (*tile < 1) *tile = 1;
}

inline int64_t count(const std::vector<Run> &v) {
    int64_t n = 0;
    for (const Run &r : v) n += r.count;
    return n;
}

}  // namespace hclib_sets

#endif  // HCLIB_FORASYNC_SETS_H_
