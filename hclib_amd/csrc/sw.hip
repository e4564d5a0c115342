// sw.hip — the Smith-Waterman tile DAG (test/smithwaterman/smith_waterman.cpp)
// with device-side dependency counters.
//
// Reference: every tile is an async_await on three futures (:227-229); each
// completed tile puts three promises (bottom_right, right_column,
// bottom_row, :212-226) and hclib_promise_put walks the waiter lists
// (src/hclib-promise.c:203-245) to make dependants runnable.
// Here: a tile's three futures are one dependency counter (boundary
// promises are pre-satisfied, :141-165, so border tiles start lower); a
// finished tile publishes its bottom row / right column / corner with
// write-through stores, releases, then decrements each dependant's counter;
// the decrement that reaches zero appends the dependant to a ready list.
// Persistent waves take tickets on the ready list in order (one agent
// atomic) — every ticket below the tile count is eventually filled because
// the DAG is acyclic, so the wait is bounded and deadlock-free.
//
// In-tile DP: one wave per tile; lane L owns RP consecutive rows of a
// 64*RP-row band and sweeps the columns skewed by L (anti-diagonal
// pipeline): at step s it computes column s-L, receiving the cell above from
// lane L-1 through a one-lane DPP shift. Bands are chained through LDS.
#include <string.h>

#include <vector>

#include "hx_module.h"

namespace hx {

constexpr uint32_t kEmpty = 0xffffffffu;
constexpr int kSwRP = 4;  // rows per lane per band -> 256-row bands

struct SwCtx {
    const int8_t *s1;  // coded 1..4
    const int8_t *s2;
    int tw, th, ntw, nth;
    int *bottom;       // [tiles][tw]
    int *right;        // [tiles][th]
    int *corner;       // [tiles]
    uint32_t *deps;    // [tiles]
    uint32_t *ready;   // [tiles] ticket-ordered ready list (kEmpty = not yet)
    uint32_t *ready_tail;
    uint32_t *ready_head;
    uint32_t *err;
    unsigned long long *stats;  // [0] tiles, [1] releases
    uint32_t spin_ms;
};

// alignment_score_matrix (smith_waterman.cpp:36-43) row for s2 code a, plus
// 2 (see the G transform below), packed as four signed bytes for s1 = 1..4:
// A: 4 -2 0 -2 | C: -2 4 -2 0 | G: 0 -2 4 -2 | T: -2 0 -2 4
__device__ __forceinline__ uint32_t sw_row2(int a) {
    return a == 1 ? 0xfe00fe04u : a == 2 ? 0x00fe04feu : a == 3 ? 0xfe04fe00u : 0x04fe00feu;
}

__device__ __forceinline__ int shift_up1(int v) {
    // lane L receives lane L-1's value in one DPP move (GFX9 wave_shr:1);
    // lane 0 receives 0 and reads its input from LDS instead
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}

// One tile task. The DP runs on G = H + row + col (matrix indices): with the
// unit gap penalty, H = max(H_left - 1, H_up - 1, H_diag + M) becomes
// G = max3(G_left, G_up, G_diag + M + 2) — one dependent max3 per cell.
// Inputs are converted to G when loaded, outputs back to H when stored, so
// the promises' data (bottom row, right column, corner) are the reference's.
__device__ void sw_tile(const SwCtx &c, uint32_t t, int *lds_top, int *lds_bot, int8_t *lds_s1) {
    const int lane = lane_id();
    const int i = (int)(t / (uint32_t)c.ntw) + 1;  // tile row (1-based)
    const int j = (int)(t % (uint32_t)c.ntw) + 1;  // tile col
    const int tw = c.tw, th = c.th;
    const int R0 = (i - 1) * th + 1, C0 = (j - 1) * tw + 1;  // matrix index of cell (0,0)
    const uint32_t tup = t - (uint32_t)c.ntw, tleft = t - 1, tdiag = t - (uint32_t)c.ntw - 1;
    // s1 segment of this tile column
    for (int q = lane; q < tw; q += 64) lds_s1[q] = c.s1[(size_t)(j - 1) * tw + q];
    // top row = matrix row R0-1, columns C0-1 .. C0-1+tw: corner + above tile's bottom row
    if (lane == 0) {
        int h = (i == 1) ? -((j - 1) * tw) : (j == 1 ? -((i - 1) * th) : ld_agent(&c.corner[tdiag]));
        if (i == 1 && j == 1) h = 0;
        lds_top[0] = h + (R0 - 1) + (C0 - 1);
    }
    for (int q = lane; q < tw; q += 64) {
        const int h = (i == 1) ? -((j - 1) * tw + q + 1) : ld_agent(&c.bottom[(size_t)tup * tw + q]);
        lds_top[q + 1] = h + (R0 - 1) + (C0 + q);
    }
    __syncthreads();
    for (int r0 = 0; r0 < th; r0 += 64 * kSwRP) {
        const int rfirst = r0 + lane * kSwRP;
        int left[kSwRP];
        uint32_t mrow[kSwRP];
        int nvalid = 0;
#pragma unroll
        for (int q = 0; q < kSwRP; ++q) {
            const int r = rfirst + q;
            if (r < th) {
                ++nvalid;
                const int h = (j == 1) ? -((i - 1) * th + r + 1) : ld_agent(&c.right[(size_t)tleft * th + r]);
                left[q] = h + (R0 + r) + (C0 - 1);
                mrow[q] = sw_row2(c.s2[(size_t)(i - 1) * th + r]);
            } else {
                left[q] = 0;
                mrow[q] = 0;
            }
        }
        // G at (rfirst-1, column 0): the left boundary one row up (corner for row 0)
        int up_prev;
        if (rfirst == 0) up_prev = lds_top[0];
        else if (j == 1) up_prev = -((i - 1) * th + rfirst) + (R0 + rfirst - 1) + (C0 - 1);
        else up_prev = (rfirst - 1 < th)
                           ? ld_agent(&c.right[(size_t)tleft * th + rfirst - 1]) + (R0 + rfirst - 1) + (C0 - 1)
                           : 0;
        const int band_rows = (th - r0) < 64 * kSwRP ? (th - r0) : 64 * kSwRP;
        const int last_lane = (band_rows - 1) / kSwRP;
        const int last_q = (band_rows - 1) % kSwRP;
        if (lane == last_lane) lds_bot[0] = left[last_q];  // G[band last row][0]
        int out = 0;
        const int steps = tw + 63;
        // LDS operands of step s are loaded during step s-1 (latency hidden)
        int c0 = -lane < 0 ? 0 : -lane;
        int b_cur = lds_s1[c0], top_cur = lds_top[c0 + 1];
        // one anti-diagonal step of this lane's kSwRP rows
        auto cell_rows = [&](int up) {
            int diag = up_prev;
            up_prev = up;
            const int sh = (b_cur << 3) - 8;  // byte of the s1 code in the packed score row
#pragma unroll
            for (int q = 0; q < kSwRP; ++q) {
                const int d = diag + __builtin_amdgcn_sbfe((int)mrow[q], sh, 8);
                const int a = left[q] > up ? left[q] : up;
                const int h = a > d ? a : d;
                diag = left[q];
                left[q] = h;
                up = h;
            }
            return up;
        };
        auto masked_step = [&](int s) {
            const int recv = shift_up1(out);
            const int cidx = s - lane;  // 0-based column
            int cn = cidx + 1;
            cn = cn < 0 ? 0 : (cn >= tw ? tw - 1 : cn);
            const int b_nxt = lds_s1[cn];
            const int top_nxt = lds_top[cn + 1];
            if (cidx >= 0 && cidx < tw && nvalid > 0) {
                out = cell_rows((lane == 0) ? top_cur : recv);
                if (lane == last_lane) lds_bot[cidx + 1] = left[last_q];
            }
            b_cur = b_nxt;
            top_cur = top_nxt;
        };
        int s = 0;
        if (band_rows == 64 * kSwRP && tw > 64) {
            // ramp-in, a branch-free steady state in which every lane is on a
            // valid column (s-63 .. s), then ramp-out
            for (; s < 63; ++s) masked_step(s);
            const int dummy = tw + 2 + lane;  // lds_bot has 64 spare words past tw+1
            for (; s < tw; ++s) {
                const int recv = shift_up1(out);
                const int cidx = s - lane;
                const int cn = cidx + 1 < tw ? cidx + 1 : tw - 1;
                const int b_nxt = lds_s1[cn];
                const int top_nxt = lds_top[cn + 1];
                out = cell_rows(lane == 0 ? top_cur : recv);
                // lane 63 owns the band's last row; the others hit a private dummy word
                lds_bot[(lane == 63) ? cidx + 1 : dummy] = out;
                b_cur = b_nxt;
                top_cur = top_nxt;
            }
        }
        for (; s < steps; ++s) masked_step(s);
        // the right column H[row][tw] is each lane's final `left`
#pragma unroll
        for (int q = 0; q < kSwRP; ++q)
            if (q < nvalid)
                st_agent(&c.right[(size_t)t * th + rfirst + q],
                         left[q] - (R0 + rfirst + q) - (C0 + tw - 1));
        __syncthreads();
        // the band's bottom row becomes the next band's top row (both in G)
        for (int q = lane; q <= tw; q += 64) lds_top[q] = lds_bot[q];
        __syncthreads();
    }
    const int Rb = R0 + th - 1;  // matrix row of the tile's bottom row
    for (int q = lane; q < tw; q += 64)
        st_agent(&c.bottom[(size_t)t * tw + q], lds_top[q + 1] - Rb - (C0 + q));
    if (lane == 0) st_agent(&c.corner[t], lds_top[tw] - Rb - (C0 + tw - 1));
}

__global__ __launch_bounds__(64) void k_sw(SwCtx c) {
    extern __shared__ __attribute__((aligned(16))) int sw_lds[];
    int *lds_top = sw_lds;
    int *lds_bot = sw_lds + ((c.tw + 1 + 3) & ~3);
    int8_t *lds_s1 = (int8_t *)(lds_bot + ((c.tw + 1 + 3) & ~3) + 68);  // + 64 dummy words
    const int lane = lane_id();
    const uint32_t ntiles = (uint32_t)(c.ntw * c.nth);
    unsigned long long ntile = 0, nrel = 0, cyc_tile = 0, cyc_rel = 0;
    while (true) {
        uint32_t ticket = 0;
        if (lane == 0) ticket = add_agent(c.ready_head, 1u);
        ticket = __shfl(ticket, 0, 64);
        if (ticket >= ntiles) break;
        uint32_t t = kEmpty;
        if (lane == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while ((t = ld_agent(&c.ready[ticket])) == kEmpty) {
                if (ld_agent(c.err)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * c.spin_ms) {
                    dev_error(c.err, kErrSpinTimeout);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        t = __shfl(t, 0, 64);
        if (t == kEmpty) break;
        // inputs are read with sc1 loads only: no L1 invalidate needed
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        sw_tile(c, t, lds_top, lds_bot, lds_s1);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        cyc_tile += t1 - t0;
        ++ntile;
        // every output word was stored write-through (sc1); drain them before
        // the counters that publish the tile (MI355X_MICROARCH.md, Valid forms:
        // sc1 payload + drained counter; consumers read with sc1 loads)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            const int i = (int)(t / (uint32_t)c.ntw), j = (int)(t % (uint32_t)c.ntw);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t succ = k == 0 ? t + 1 : (k == 1 ? t + (uint32_t)c.ntw : t + (uint32_t)c.ntw + 1);
                const bool ok = k == 0 ? (j + 1 < c.ntw) : (k == 1 ? (i + 1 < c.nth) : (j + 1 < c.ntw && i + 1 < c.nth));
                if (!ok) continue;
                ++nrel;
                const uint32_t old = add_agent(&c.deps[succ], (uint32_t)-1);
                if (old == 1) {
                    const uint32_t pos = add_agent(c.ready_tail, 1u);
                    st_agent(&c.ready[pos], succ);
                }
            }
        }
        __syncthreads();
        cyc_rel += __builtin_amdgcn_s_memtime() - t1;
    }
    if (lane == 0) {
        add_agent(&c.stats[0], ntile);
        add_agent(&c.stats[1], nrel);
        add_agent(&c.stats[2], cyc_tile);
        add_agent(&c.stats[3], cyc_rel);
    }
}

__global__ void k_sw_init(uint32_t *deps, uint32_t *ready, int ntw, int nth) {
    const uint32_t n = (uint32_t)(ntw * nth);
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const int i = (int)(t / ntw), j = (int)(t % ntw);
        deps[t] = (uint32_t)((i > 0) + (j > 0) + (i > 0 && j > 0));
        ready[t] = (t == 0) ? 0u : kEmpty;
    }
}

}  // namespace hx

using namespace hx;

extern "C" int hclib_hip_sw(const int8_t *s1, size_t n1, const int8_t *s2, size_t n2, int tw,
                            int th, int *score, hclib_hip_sw_result_t *result) {
    if (!s1 || !s2 || !score || tw < 1 || th < 1 || tw > 16384) {
        set_error("hclib_hip_sw: invalid arguments (1 <= tw <= 16384, th >= 1)");
        return HCLIB_HIP_EINVAL;
    }
    const size_t ntw = n1 / (size_t)tw, nth = n2 / (size_t)th;
    if (ntw == 0 || nth == 0 || ntw * nth > 0x7fffffffull) {
        set_error("hclib_hip_sw: empty or oversized tile grid");
        return HCLIB_HIP_EINVAL;
    }
    for (size_t k = 0; k < ntw * (size_t)tw; ++k)
        if (s1[k] < 1 || s1[k] > 4) { set_error("hclib_hip_sw: s1 must be coded 1..4"); return HCLIB_HIP_EINVAL; }
    for (size_t k = 0; k < nth * (size_t)th; ++k)
        if (s2[k] < 1 || s2[k] > 4) { set_error("hclib_hip_sw: s2 must be coded 1..4"); return HCLIB_HIP_EINVAL; }
    HX_TRY(ensure_device());
    Module &m = mod();
    const size_t nt = ntw * nth;
    const size_t b_s1 = ntw * tw, b_s2 = nth * th;
    const size_t b_bot = nt * tw * 4, b_right = nt * th * 4, b_c = nt * 4, b_dep = nt * 4,
                 b_ready = nt * 4;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t total = al(b_s1) + al(b_s2) + al(b_bot) + al(b_right) + al(b_c) + al(b_dep) +
                         al(b_ready) + 1024;
    char *d = nullptr;
    if (hipMalloc((void **)&d, total) != hipSuccess) {
        set_error("hclib_hip_sw: hipMalloc(%zu) failed", total);
        return HCLIB_HIP_ENOMEM;
    }
    SwCtx c;
    size_t off = 0;
    c.s1 = (const int8_t *)(d + off); off += al(b_s1);
    c.s2 = (const int8_t *)(d + off); off += al(b_s2);
    c.bottom = (int *)(d + off); off += al(b_bot);
    c.right = (int *)(d + off); off += al(b_right);
    c.corner = (int *)(d + off); off += al(b_c);
    c.deps = (uint32_t *)(d + off); off += al(b_dep);
    c.ready = (uint32_t *)(d + off); off += al(b_ready);
    uint32_t *misc = (uint32_t *)(d + off);
    c.ready_tail = misc;
    c.ready_head = misc + 64;
    c.err = misc + 128;
    c.stats = (unsigned long long *)(misc + 192);
    c.tw = tw;
    c.th = th;
    c.ntw = (int)ntw;
    c.nth = (int)nth;
    c.spin_ms = (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    int rc = HCLIB_HIP_OK;
    auto fail = [&](int r) { (void)hipFree(d); return r; };
    if ((rc = hip_check(hipMemcpyAsync((void *)c.s1, s1, b_s1, hipMemcpyHostToDevice, m.stream), "copy s1"))) return fail(rc);
    if ((rc = hip_check(hipMemcpyAsync((void *)c.s2, s2, b_s2, hipMemcpyHostToDevice, m.stream), "copy s2"))) return fail(rc);
    if ((rc = hip_check(hipMemsetAsync(misc, 0, 1024, m.stream), "memset"))) return fail(rc);
    {
        uint32_t one = 1;  // tile 0 already sits at ready[0]
        if ((rc = hip_check(hipMemcpyAsync(c.ready_tail, &one, 4, hipMemcpyHostToDevice, m.stream), "tail"))) return fail(rc);
    }
    hipLaunchKernelGGL(k_sw_init, dim3(1024), dim3(256), 0, m.stream, c.deps, c.ready, c.ntw, c.nth);
    const size_t lds = 2 * (size_t)(((tw + 1 + 3) & ~3) * 4) + 68 * 4 + (size_t)tw + 16;
    if (lds > 160 * 1024) return fail((set_error("hclib_hip_sw: tile width too large for LDS"), HCLIB_HIP_EINVAL));
    int per_cu = (int)((160 * 1024) / lds);
    int wpc = env_int("HCLIB_HIP_SW_WAVES_PER_CU", 2);
    if (wpc > per_cu) wpc = per_cu;
    if (wpc < 1) wpc = 1;
    const int grid = m.num_cus * wpc;
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void *)k_sw, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if ((rc = hip_check(hipEventRecord(m.ev0, m.stream), "event"))) return fail(rc);
    hipLaunchKernelGGL(k_sw, dim3(grid), dim3(64), lds, m.stream, c);
    if ((rc = hip_check(hipGetLastError(), "k_sw launch"))) return fail(rc);
    if ((rc = hip_check(hipEventRecord(m.ev1, m.stream), "event"))) return fail(rc);
    uint32_t herr = 0;
    unsigned long long st[4] = {0, 0, 0, 0};
    int corner = 0;
    if ((rc = hip_check(hipStreamSynchronize(m.stream), "k_sw"))) return fail(rc);
    (void)hipMemcpy(&herr, c.err, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(st, c.stats, 32, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&corner, c.corner + (nt - 1), 4, hipMemcpyDeviceToHost);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, m.ev0, m.ev1);
    (void)hipFree(d);
    if (herr) {
        set_error("hclib_hip_sw: device error %u", herr);
        return HCLIB_HIP_EDEVICE;
    }
    if (st[0] != nt) {
        set_error("hclib_hip_sw: executed %llu of %zu tiles", st[0], nt);
        return HCLIB_HIP_EDEVICE;
    }
    *score = corner;  // bottom_row[tw-1] of the last tile == its corner (:239)
    if (result) {
        result->tiles = st[0];
        result->releases = st[1];
        result->kernel_ms = ms;
        result->cells_per_s = (double)nt * tw * th / (ms * 1e-3);
        result->tile_us = st[0] ? (double)st[2] / st[0] / 2400.0 : 0.0;
        result->release_us = st[0] ? (double)st[3] / st[0] / 2400.0 : 0.0;
    }
    return HCLIB_HIP_OK;
}
