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
#include <stdio.h>
#include <string.h>

#include <vector>

#include "hx_module.h"
#include "../../include/hclib_hip/hx_dag.h"

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
    // row-pipelined schedule: a tile's bottom row is published as 8-byte
    // {tag = 1, H} granules — the data is the promise (R2 hand-off)
    unsigned long long *gbot;  // [tiles][tw]
    // column band (multi-GPU sharding by tile columns; the whole grid is
    // j0 = 0, j1 = ntw, i0 = 0, i1 = nth): tile columns [j0, j1), tile rows
    // [i0, i1) of this launch. left_in = H of matrix column j0*tw, rows
    // 1..nth*th (the left band's right column; null when j0 == 0);
    // right_out receives H of matrix column j1*tw (null: not wanted)
    int j0, j1, i0, i1;
    int progressive;  // row schedule: chunked bottom-row hand-off
    const int *left_in;  // [nth*th]
    int *right_out;      // [nth*th]
    // the packed DAG body's outputs as tagged granules {1 << 32 | H}
    // (bottom rows in gbot [tiles][tw]; right columns [tiles][th]; corners [tiles])
    unsigned long long *gright, *gcorner;
    int form;            // multi-wave bands: 100 * rows per lane + 10 * skew + hand-off steps / 16
    int bh;              // multi-wave band height (64 * rows per lane)
    // diagnostic build (HX_STAMPS): the DAG's per-task trace (hx_dag.h
    // kDagTraceWords), where tile tasks stamp their waves' phases; else null
    unsigned long long *dtrace;
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
// Diagnostic build (-DHX_STAMPS=1, `python -m hclib_amd.build --variant stamps`):
// per-phase cycles of a tile into SwCtx::stats[4..9]; compiled out otherwise.
#ifndef HX_STAMPS
#define HX_STAMPS 0
#endif
__device__ __forceinline__ unsigned long long sw_stamp() {
#if HX_STAMPS
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
#else
    return 0;
#endif
}

// ROWS = false: the three futures came through device dependency counters and
// the inputs are global arrays (queue schedule). ROWS = true: the owning wave
// keeps the left neighbour's right column in LDS (lds_left, H values) and the
// top row is the up neighbour's granules, swept until every tag is set;
// `corner` carries H at (R0-1, C0-1) in and the up tile's bottom-right out.
template <bool ROWS, bool PROG = false>
__device__ bool sw_tile(const SwCtx &c, uint32_t t, int *lds_top, int *lds_bot, int8_t *lds_s1,
                        const int *lds_left, int *lds_right, int &corner, unsigned long long *ph) {
    unsigned long long ts = sw_stamp();
    auto phase = [&](int k) {
        if (HX_STAMPS) {
            const unsigned long long now = sw_stamp();
            ph[k] += now - ts;
            ts = now;
        }
    };
    const int lane = lane_id();
    const int i = (int)(t / (uint32_t)c.ntw) + 1;  // tile row (1-based)
    const int j = (int)(t % (uint32_t)c.ntw) + 1;  // tile col
    const int tw = c.tw, th = c.th;
    const int R0 = (i - 1) * th + 1, C0 = (j - 1) * tw + 1;  // matrix index of cell (0,0)
    const uint32_t tup = t - (uint32_t)c.ntw, tleft = t - 1, tdiag = t - (uint32_t)c.ntw - 1;
    // progressive bottom-row hand-off (row schedule, one 256-row band, whole
    // 64-column chunks): the tile publishes each chunk of its bottom row as
    // soon as its last lane has computed it, and the tile below starts after
    // the first chunk instead of the whole row (HCLIB_HIP_SW_PROGRESSIVE=0
    // publishes at the end, as before)
    const bool prog_out = ROWS && PROG && th == 64 * kSwRP && (tw & 63) == 0;
    const bool prog = prog_out && i > 1;
    // s1 segment of this tile column
    for (int q = lane; q < tw; q += 64) lds_s1[q] = c.s1[(size_t)(j - 1) * tw + q];
    // v_perm selectors of the 4x4-blocked band: byte k of word b = s1 code - 1
    // of column 4b+k (codes 1..4 -> 0..3, so no byte borrows)
    uint32_t *lds_sel = (uint32_t *)(lds_s1 + ((tw + 3) & ~3));
    if ((tw & 3) == 0)
        for (int b = lane; b < (tw >> 2); b += 64)
            lds_sel[b] = ((const uint32_t *)(c.s1 + (size_t)(j - 1) * tw))[b] - 0x01010101u;
    // top row = matrix row R0-1, columns C0-1 .. C0-1+tw: corner + above tile's bottom row
    if (ROWS) {
        if (lane == 0) lds_top[0] = corner + (R0 - 1) + (C0 - 1);
        if (i == 1) {
            for (int q = lane; q < tw; q += 64) lds_top[q + 1] = -((j - 1) * tw + q + 1) + (R0 - 1) + (C0 + q);
            corner = -(j * tw);  // bottom_right of boundary tile (0, j), smith_waterman.cpp:151
        } else {
            // sweep the up tile's granules until every tag is set (bounded);
            // progressive: only the first 64-column chunk, the rest is
            // fetched inside the step loop as the up tile publishes it
            const unsigned long long *g = c.gbot + (size_t)tup * tw;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            const int qend = prog ? 64 : tw;
            bool all = false;
            while (!all) {
                bool ok = true;
                for (int q = lane; q < qend; q += 64) {
                    const unsigned long long x = ld_agent(&g[q]);
                    if ((x >> 32) != 1ull) ok = false;
                    else lds_top[q + 1] = (int)(uint32_t)x + (R0 - 1) + (C0 + q);
                }
                all = __all(ok);
                if (!all) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * c.spin_ms) {
                        if (lane == 0) dev_error(c.err, kErrSpinTimeout);
                        return false;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            // the next tile's diagonal corner: the up tile's bottom-right
            if (!prog || tw == 64) corner = (int)(uint32_t)ld_agent(&g[tw - 1]);
        }
    } else {
        if (lane == 0) {
            int h = (i == 1) ? -((j - 1) * tw) : (j == 1 ? -((i - 1) * th) : ld_agent(&c.corner[tdiag]));
            if (i == 1 && j == 1) h = 0;
            lds_top[0] = h + (R0 - 1) + (C0 - 1);
        }
        for (int q = lane; q < tw; q += 64) {
            const int h = (i == 1) ? -((j - 1) * tw + q + 1) : ld_agent(&c.bottom[(size_t)tup * tw + q]);
            lds_top[q + 1] = h + (R0 - 1) + (C0 + q);
        }
    }
    __syncthreads();
    for (int r0 = 0; r0 < th; r0 += 64 * kSwRP) {
        phase(0);
        const int rfirst = r0 + lane * kSwRP;
        int left[kSwRP];
        uint32_t mrow[kSwRP];
        int nvalid = 0;
#pragma unroll
        for (int q = 0; q < kSwRP; ++q) {
            const int r = rfirst + q;
            if (r < th) {
                ++nvalid;
                const int h = (j == 1) ? -((i - 1) * th + r + 1)
                                       : (ROWS ? lds_left[r] : ld_agent(&c.right[(size_t)tleft * th + r]));
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
                           ? (ROWS ? lds_left[rfirst - 1] : ld_agent(&c.right[(size_t)tleft * th + rfirst - 1])) +
                                 (R0 + rfirst - 1) + (C0 - 1)
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
        auto cell_rows_sh = [&](int up, int sh) {  // sh: bit offset of the s1 code's score byte
            int diag = up_prev;
            up_prev = up;
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
        auto cell_rows = [&](int up) { return cell_rows_sh(up, (b_cur << 3) - 8); };
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
        phase(1);
        if (band_rows == 64 * kSwRP && (tw & 3) == 0) {
            // 4x4-blocked wavefront: at step st lane L computes its 4 rows x
            // the 4 columns of block st-L (16 cells). The cells above come
            // from lane L-1's previous step (4 DPP wave shifts whose `old`
            // operand is lane 0's top row, so lane 0 needs no select); the
            // score bytes of a row for 4 columns are one v_perm of the packed
            // score row by the block's selector. One DPP latency per 16
            // cells, no LDS round trip in the dependency chain.
            const int nblocks = tw >> 2, nsteps = nblocks + 63;
            int o0 = 0, o1 = 0, o2 = 0, o3 = 0;  // row-3 outputs of this lane's last block
            // the block's selector and top values are loaded one step ahead
            // (their LDS latency hides behind a step's arithmetic)
            auto clampb = [&](int b) { return b < 0 ? 0 : (b >= nblocks ? nblocks - 1 : b); };
            int cbn = clampb(-lane);
            uint32_t sel_n = lds_sel[cbn];
            int t0n = lds_top[4 * cbn + 1], t1n = lds_top[4 * cbn + 2], t2n = lds_top[4 * cbn + 3],
                t3n = lds_top[4 * cbn + 4];
            unsigned long long pf = 0;  // prefetched granule of the up tile (progressive)
            // one anti-diagonal step of the 4x4-blocked band
            auto step = [&](const int st) {
                const int blk = st - lane;
                const bool valid = blk >= 0 && blk < nblocks;
                const uint32_t sel = sel_n;
                const int u0 = __builtin_amdgcn_update_dpp(t0n, o0, 0x138, 0xf, 0xf, false);
                const int u1 = __builtin_amdgcn_update_dpp(t1n, o1, 0x138, 0xf, 0xf, false);
                const int u2 = __builtin_amdgcn_update_dpp(t2n, o2, 0x138, 0xf, 0xf, false);
                const int u3 = __builtin_amdgcn_update_dpp(t3n, o3, 0x138, 0xf, 0xf, false);
                cbn = clampb(blk + 1);
                sel_n = lds_sel[cbn];
                t0n = lds_top[4 * cbn + 1];
                t1n = lds_top[4 * cbn + 2];
                t2n = lds_top[4 * cbn + 3];
                t3n = lds_top[4 * cbn + 4];
                if (valid) {
                    uint32_t pm[kSwRP];
#pragma unroll
                    for (int q = 0; q < kSwRP; ++q) pm[q] = __builtin_amdgcn_perm(0u, mrow[q], sel);
                    const int uu[4] = {u0, u1, u2, u3};
                    int ov[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        int diag = jj == 0 ? up_prev : uu[jj - 1];
                        int up = uu[jj];
#pragma unroll
                        for (int q = 0; q < kSwRP; ++q) {
                            const int d = diag + (int)(int8_t)(pm[q] >> (8 * jj));
                            const int a = left[q] > up ? left[q] : up;
                            const int h = a > d ? a : d;
                            diag = left[q];
                            left[q] = h;
                            up = h;
                        }
                        ov[jj] = up;
                    }
                    up_prev = u3;
                    o0 = ov[0];
                    o1 = ov[1];
                    o2 = ov[2];
                    o3 = ov[3];
                    if (lane == 63) {  // the band's last row
                        int *bp = &lds_bot[4 * blk + 1];
                        bp[0] = o0;
                        bp[1] = o1;
                        bp[2] = o2;
                        bp[3] = o3;
                    }
                }
            };
            if (!prog_out) {
                for (int st = 0; st < nsteps; ++st) step(st);
            } else {
                // progressive: the hand-off work sits between 16-step runs,
                // after every step st = 16m + 14 (chunk k is published after
                // step 16k + 78 and the up tile's chunk k is needed from step
                // 16k - 1 on), so the step loop itself stays free of it
                if (prog) pf = ld_agent(&c.gbot[(size_t)tup * tw + 64 + lane]);  // chunk 1
                for (int base = -1; base < nsteps; base += 16) {
                    const int lo = base < 0 ? 0 : base, hi = (base + 16) < nsteps ? base + 16 : nsteps;
                    for (int st = lo; st < hi; ++st) step(st);
                    const int st = hi - 1;  // = 16m + 14 (nsteps = 16n + 15)
                    const int pk = st - 78;
                    if (pk >= 0) {
                        const int q = 4 * pk + lane;  // chunk pk/16 of this tile's bottom row
                        st_agent(&c.gbot[(size_t)t * tw + q],
                                 (1ull << 32) | (unsigned long long)(uint32_t)(lds_bot[q + 1] - (R0 + th - 1) - (C0 + q)));
                    }
                    const int kc = st + 2;  // 16k: the up tile's chunk k is due
                    if (prog && (kc >> 4) < nblocks / 16) {
                        const int q = 4 * kc + lane;
                        const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
                        while (!__all((pf >> 32) == 1ull)) {
                            if (__builtin_amdgcn_s_memrealtime() - w0 > 100000ull * c.spin_ms) {
                                if (lane == 0) dev_error(c.err, kErrSpinTimeout);
                                return false;
                            }
                            pf = ld_agent(&c.gbot[(size_t)tup * tw + q]);
                        }
                        lds_top[q + 1] = (int)(uint32_t)pf + (R0 - 1) + (C0 + q);
                        if (q + 64 - lane == tw)  // last chunk: the next tile's corner
                            corner = (int)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pf, 63);
                        else  // prefetch the next chunk, due 16 steps later
                            pf = ld_agent(&c.gbot[(size_t)tup * tw + q + 64]);
                    }
                }
            }
            s = steps;
        } else if (band_rows == 64 * kSwRP && tw > 64) {
            // ramp-in, a branch-free steady state in which every lane is on a
            // valid column (s-63 .. s), then ramp-out
            for (; s < 63; ++s) masked_step(s);
            phase(2);
            // Register pipeline, no LDS round trip per step: lane L's s1 code
            // for column s-L is lane L-1's from step s-1 (one DPP shift), as
            // is the cell above; lane 0 takes the new column's code and top
            // value from a 64-column chunk (readlane + lane-0 select), and lane
            // 63's bottom-row outputs collect in a chunk stored once per 64
            // steps. LDS is touched three times per 64 columns.
            int shv = lane <= 62 ? (((int)lds_s1[62 - lane]) << 3) - 8 : 0;  // column 62-L
            for (int s0 = 63; s0 < tw; s0 += 64) {
                const int nblk = (tw - s0) < 64 ? (tw - s0) : 64;
                const int cc = s0 + lane;
                const int csh = cc < tw ? (((int)lds_s1[cc]) << 3) - 8 : 0;
                const int ctop = cc < tw ? lds_top[cc + 1] : 0;
                int botc = 0;
                for (int k = 0; k < nblk; ++k) {
                    const int up_in = shift_up1(out), sh_in = shift_up1(shv);
                    const int top_k = __builtin_amdgcn_readlane(ctop, k), sh_k = __builtin_amdgcn_readlane(csh, k);
                    const int recv = lane == 0 ? top_k : up_in;
                    shv = lane == 0 ? sh_k : sh_in;
                    out = cell_rows_sh(recv, shv);
                    const int b63 = __builtin_amdgcn_readlane(out, 63);
                    botc = lane == k ? b63 : botc;
                }
                // lane 63 computed columns s0-63 .. s0-63+nblk-1 (the band's last row)
                if (lane < nblk) lds_bot[s0 - 63 + lane + 1] = botc;
                s = s0 + nblk;
            }
            // masked_step's operands for step s (column s-L)
            const int cn = (s - lane) < tw ? (s - lane) : tw - 1;
            b_cur = lds_s1[cn];
            top_cur = lds_top[cn + 1];
        }
        phase(3);
        for (; s < steps; ++s) masked_step(s);
        phase(4);
        // the right column H[row][tw] is each lane's final `left`; in the
        // row schedule it stays in LDS for the same wave's next tile
#pragma unroll
        for (int q = 0; q < kSwRP; ++q)
            if (q < nvalid) {
                const int hv = left[q] - (R0 + rfirst + q) - (C0 + tw - 1);
                if (ROWS) lds_right[rfirst + q] = hv;
                else st_agent(&c.right[(size_t)t * th + rfirst + q], hv);
            }
        __syncthreads();
        // the band's bottom row becomes the next band's top row (both in G)
        for (int q = lane; q <= tw; q += 64) lds_top[q] = lds_bot[q];
        __syncthreads();
    }
    const int Rb = R0 + th - 1;  // matrix row of the tile's bottom row
    if (ROWS && !prog_out) {
        // publish: one 8-byte sc1 granule per value (tag 1 = put), drained
        for (int q = lane; q < tw; q += 64)
            st_agent(&c.gbot[(size_t)t * tw + q],
                     (1ull << 32) | (unsigned long long)(uint32_t)(lds_top[q + 1] - Rb - (C0 + q)));
    } else if (!ROWS) {
        for (int q = lane; q < tw; q += 64)
            st_agent(&c.bottom[(size_t)t * tw + q], lds_top[q + 1] - Rb - (C0 + q));
        if (lane == 0) st_agent(&c.corner[t], lds_top[tw] - Rb - (C0 + tw - 1));
    }
    phase(5);
    return true;
}

__global__ __launch_bounds__(64) void k_sw(SwCtx c) {
    extern __shared__ __attribute__((aligned(16))) int sw_lds[];
    int *lds_top = sw_lds;
    int *lds_bot = sw_lds + ((c.tw + 1 + 3) & ~3);
    int8_t *lds_s1 = (int8_t *)(lds_bot + ((c.tw + 1 + 3) & ~3) + 68);  // + 64 dummy words
    const int lane = lane_id();
    const uint32_t ntiles = (uint32_t)(c.ntw * c.nth);
    unsigned long long ntile = 0, nrel = 0, cyc_tile = 0, cyc_rel = 0;
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
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
        int corner_unused = 0;
        sw_tile<false>(c, t, lds_top, lds_bot, lds_s1, nullptr, nullptr, corner_unused, ph);
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
        if (HX_STAMPS)
            for (int k = 0; k < 6; ++k) add_agent(&c.stats[4 + k], ph[k]);
    }
}

// Row schedule ("owner computes"): wave w owns tile rows w, w + W, ... and
// runs each left to right. Tile (i, j)'s three futures: the left one is the
// wave's own previous tile (program order; its right column stays in LDS),
// the up one is the up tile's published granules (swept, R2 hand-off), the
// diagonal one is implied (the up row's owner finished (i-1, j-1) before
// (i-1, j)). Every wave is resident (grid <= CUs) and rows complete in
// order, so each wait ends.
template <bool PROG>
__global__ __launch_bounds__(64) void k_sw_rows(SwCtx c) {
    extern __shared__ __attribute__((aligned(16))) int sw_lds[];
    int *lds_top = sw_lds;
    int *lds_bot = sw_lds + ((c.tw + 1 + 3) & ~3);
    int *lds_left = lds_bot + ((c.tw + 1 + 3) & ~3) + 68;  // + 64 dummy words
    int *lds_right = lds_left + ((c.th + 3) & ~3);             // swapped per tile
    int8_t *lds_s1 = (int8_t *)(lds_right + ((c.th + 3) & ~3));
    const int lane = lane_id();
    unsigned long long ntile = 0, cyc_tile = 0, cyc_wait = 0;
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
    bool ok = true;
    for (int i = c.i0 + (int)blockIdx.x; i < c.i1 && ok; i += gridDim.x) {
        // H(R0-1, C0-1) of tile (i, j0): the boundary column, or for a band
        // the left band's right column one row above the tile
        int corner = (i == 0) ? -(c.j0 * c.tw) : -(i * c.th);
        if (c.j0 > 0) {
            if (i > 0) corner = ld_agent(&c.left_in[(size_t)i * c.th - 1]);
            for (int r = lane; r < c.th; r += 64) lds_left[r] = ld_agent(&c.left_in[(size_t)i * c.th + r]);
            __syncthreads();
        }
        for (int j = c.j0; j < c.j1 && ok; ++j) {
            const uint32_t t = (uint32_t)(i * c.ntw + j);
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            ok = sw_tile<true, PROG>(c, t, lds_top, lds_bot, lds_s1, lds_left, lds_right, corner, ph);
            vm_drain();  // every granule of this tile is out before the next one is computed
            int *tmp = lds_left;  // this tile's right column is the next tile's left
            lds_left = lds_right;
            lds_right = tmp;
            cyc_tile += __builtin_amdgcn_s_memtime() - t0;
            ++ntile;
        }
        // the band's right column (now in lds_left) goes to the right band
        if (ok && c.right_out)
            for (int r = lane; r < c.th; r += 64) c.right_out[(size_t)i * c.th + r] = lds_left[r];
    }
    if (lane == 0) {
        add_agent(&c.stats[0], ntile);
        add_agent(&c.stats[2], cyc_tile);
        add_agent(&c.stats[3], cyc_wait);
        if (HX_STAMPS)
            for (int k = 0; k < 6; ++k) add_agent(&c.stats[4 + k], ph[k]);
    }
}

// ----------------------------------------------- multi-wave tile rows
// Tile row as a workgroup of NW = th / 64 waves: wave w owns the 64 matrix
// rows 64w .. 64w + 63 of the tile row (one row per lane) and sweeps the
// band's columns left to right in ONE continuous anti-diagonal pipeline —
// tile boundaries inside the row are only where granules are published, so
// no wave pays a ramp per tile. Lane L computes column s - L at step s; the
// cell above comes from lane L-1 by one DPP wave shift, lane 0's from the
// wave above through an LDS ring (ring w + 1 = wave w's bottom row, written
// by its lane 63 every step). Wave 0's ring is filled from the up tile row's
// granules (or the boundary row); wave NW-1 publishes its ring as the tile
// row's granules. Hand-offs every kSwSub steps: prod[w] = columns of ring w
// written, cons[w] = columns of ring w read, so wave w + 1 runs 64 + kSwSub
// steps behind wave w. NW waves run on the CU's 4 SIMDs at once instead of
// one wave per tile row.
constexpr int kSwRing = 512;  // columns per inter-wave ring (+1 wrap slot)
constexpr int kSwRingStride = kSwRing + 4;
constexpr int kSwSub = 16;    // steps per hand-off
// dummy ring slots per compute wave (its lanes 0..62 write there every step
// while lane 63 writes the out ring; lane stride 1: neighbours' two-dword
// writes overlap, which measured no slower than stride 2)
constexpr int kSwDummy = 128;

__host__ __device__ inline size_t sw_band_lds_bytes(int nw) {
    return (size_t)(nw + 1) * kSwRingStride * 4  // rings
           + (size_t)nw * kSwDummy * 4            // per-wave dummy slots (lanes 0..62's ring writes)
           + (size_t)nw * 2048                    // per-wave code rings: 4 byte-shifted copies, double-mapped
           + 2 * 64 * 4;                          // prod / cons words
}

// the multi-wave kernel's shape: bands of bh = 64 or 128 rows, 1..14 compute
// waves per tile row (+ the ingress and egress waves)
inline bool sw_band_ok(int th, int bh) { return th % bh == 0 && th / bh >= 1 && th / bh <= 14; }
// HCLIB_HIP_SW_FORM (default `def`), kept to a valid form for th: two rows
// per lane need th % 128 == 0, else one row per lane with the same hand-off
inline int sw_pick_form(int th, int def) {
    int form = env_int("HCLIB_HIP_SW_FORM", def);
    if (form != 11 && form != 12 && form != 14 && form != 21 && form != 22 && form != 211 && form != 212 &&
        form != 214 && form != 411 && form != 412 && form != 414)
        form = def;
    if (form > 400 && th % 256 != 0) form -= 200;
    if (form > 200 && th % 128 != 0) form -= 200;
    return form;
}
inline int sw_form_bh(int form) { return 64 * (form > 100 ? form / 100 : 1); }
// tile rows per workgroup (HCLIB_HIP_SW_ROWS_PER_WG, default 1): more share
// the CU's SIMDs between more waves and measured slower (scripts/probe_sw.py)
inline int sw_band_rows_per_wg(int th, int bh) {
    const int bpt = th / bh, most = 14 / bpt;
    int k = env_int("HCLIB_HIP_SW_ROWS_PER_WG", 1);
    return k < 1 ? 1 : (k > most ? most : k);
}

// Flags between the waves of a workgroup. The LDS performs one wave's DS
// operations in issue order, so a flag stored after the ring data is seen
// after that data by any wave that reads the flag first and the data next;
// only the compiler must keep the program order (no memory fence needed,
// and none that would also wait for the wave's global loads and stores).
// (The casts keep these DS operations: a volatile or atomic access through
// a generic pointer becomes a FLAT one, which waits for the wave's global
// memory traffic as well.)
typedef __attribute__((address_space(3))) int lds_i32;
__device__ __forceinline__ int lds_flag_ld(const int *p) {
    asm volatile("" ::: "memory");
    const int v = __hip_atomic_load((const lds_i32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    return __builtin_amdgcn_readfirstlane(v);  // wave-uniform: scalar branches
}
__device__ __forceinline__ void lds_flag_st(int *p, int v) {
    asm volatile("" ::: "memory");
    __hip_atomic_store((lds_i32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}

// K steps of one wave's band from step s with skew S: lane L computes
// column s - S L at step s, so the cell above (lane L-1's, one column
// back... the same column) was computed S steps earlier. With S = 2 the DPP
// shift that brings it over leaves the step's dependency chain (it moves a
// value one step old), so a step costs one dependent max3 instead of a
// max3 and a DPP; the price is a band ramp of 126 steps instead of 63.
// top4 = ring slots of columns s .. s + K - 1 (lane-uniform, 16-byte
// aligned), code4 = this lane's aligned code words for columns s - S lane ..
// (4 codes each), wb = this lane's write slot for step s (lane 63: the out
// ring's slot of column s - 63 S; other lanes: their dummy slots). G-space
// cells (see sw_tile). left = h one step back, o2 = h two steps back (S = 2).
// Operands of 4 steps are read two groups ahead, in program order before the
// previous group's ring writes.
// SHIFT (64-step hand-offs): lane 63's outputs are not written to the ring
// step by step (one LDS store per step, issued by every lane — measured 14-16
// cycles of a lone wave's step, scripts/ubench/ub_swstep.hip) but shifted into
// `acc` by one DPP per step (wave_shl:1, lane 63 taking the new value), so
// after the 64 steps lane j holds step j's output and one store per chunk
// writes them all (sw_band_row).
template <bool MASK, int S, int K, bool SHIFT = false>
__device__ __forceinline__ void sw_band_sub(int s, int ncols, const int *top4, const uint32_t *code4, int *wb,
                                            uint32_t mrow, int &left, int &diag, int &o2, int &acc) {
    constexpr int G = K / 4;
    const int lane = lane_id();
    int4 tn = *(const int4 *)top4, tn2 = *(const int4 *)(top4 + 4);
    uint32_t cn = code4[0], cn2 = code4[1];
#pragma unroll
    for (int m = 0; m < G; ++m) {
        const int4 tc = tn;
        const uint32_t cc = cn;
        tn = tn2;
        cn = cn2;
        if (m + 2 < G) {
            tn2 = *(const int4 *)(top4 + 4 * (m + 2));
            cn2 = code4[m + 2];
        }
        // score bytes of the 4 columns (s2 row fixed per lane)
        const uint32_t sc = __builtin_amdgcn_perm(0u, mrow, cc);
        const int tv[4] = {tc.x, tc.y, tc.z, tc.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 4 * m + j;
            const int up = __builtin_amdgcn_update_dpp(tv[j], S == 1 ? left : o2, 0x138, 0xf, 0xf, false);
            const int d = diag + (int)(int8_t)(sc >> (8 * j));
            const int a = left > up ? left : up;
            int h = a > d ? a : d;
            if (MASK) {
                const bool v = (unsigned)(s + k - S * lane) < (unsigned)ncols;
                h = v ? h : left;
                diag = v ? up : diag;
            } else {
                diag = up;
            }
            if (S == 2) o2 = left;
            left = h;
            if (SHIFT) acc = __builtin_amdgcn_update_dpp(h, acc, 0x130, 0xf, 0xf, false);
            else wb[k] = h;
        }
    }
}

// The same K steps with R = 2 or 4 rows per lane (skew 1): lane L owns rows
// R L .. R L + R - 1 of a 64 R-row band; the cell above the lane's first row
// comes from lane L-1's last row, each other row's from the row before it in
// the same column. One DPP shift and one ring write serve R cells, and a
// 256-row tile needs 4 / R waves, so fewer hand-off lags are paid.
template <bool MASK, int K, int R, bool SHIFT = false>
__device__ __forceinline__ void sw_band_subR(int s, int ncols, const int *top4, const uint32_t *code4, int *wb,
                                             const uint32_t (&mrow)[R], int (&lr)[R], int &diag, int &acc) {
    constexpr int G = K / 4;
    const int lane = lane_id();
    int4 tn = *(const int4 *)top4, tn2 = *(const int4 *)(top4 + 4);
    uint32_t cn = code4[0], cn2 = code4[1];
#pragma unroll
    for (int m = 0; m < G; ++m) {
        const int4 tc = tn;
        const uint32_t cc = cn;
        tn = tn2;
        cn = cn2;
        if (m + 2 < G) {
            tn2 = *(const int4 *)(top4 + 4 * (m + 2));
            cn2 = code4[m + 2];
        }
        uint32_t sc[R];
#pragma unroll
        for (int q = 0; q < R; ++q) sc[q] = __builtin_amdgcn_perm(0u, mrow[q], cc);
        const int tv[4] = {tc.x, tc.y, tc.z, tc.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 4 * m + j;
            const int up0 = __builtin_amdgcn_update_dpp(tv[j], lr[R - 1], 0x138, 0xf, 0xf, false);
            const bool v = !MASK || (unsigned)(s + k - lane) < (unsigned)ncols;
            int up = up0, dg = diag;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int d = dg + (int)(int8_t)(sc[q] >> (8 * j));
                const int a = lr[q] > up ? lr[q] : up;
                int h = a > d ? a : d;
                if (MASK) h = v ? h : lr[q];
                dg = lr[q];
                lr[q] = h;
                up = h;
            }
            diag = MASK ? (v ? up0 : diag) : up0;
            if (SHIFT) acc = __builtin_amdgcn_update_dpp(lr[R - 1], acc, 0x130, 0xf, 0xf, false);
            else wb[k] = lr[R - 1];
        }
    }
}

// Wait for an LDS flag. The device error word and the clock are looked at
// only every 64 polls: a global load here would wait for all of the wave's
// outstanding global memory operations.
__device__ bool sw_band_spin(const SwCtx &c, const int *flag, int want, unsigned long long t0) {
    want = __builtin_amdgcn_readfirstlane(want);
    for (uint32_t n = 1; lds_flag_ld(flag) < want; ++n) {
        __builtin_amdgcn_s_sleep(1);
        if ((n & 63) == 0) {
            if (ld_agent(c.err)) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * c.spin_ms) {
                if (lane_id() == 0) dev_error(c.err, kErrSpinTimeout);
                return false;
            }
        }
    }
    return true;
}

// One wave's band of tile row i over the band's columns (matrix columns
// C0 + 1 .. C0 + ncols, C0 = j0 * tw). Returns false on a device error.
// Diagnostic build only (HX_STAMPS): ph[0] compute, [1] waiting for the
// top row, [2] waiting for ring space, [3] staging + publishing (cycles).
// What one workgroup's bands compute: rows R0 + 1 .. R0 + 64 nb (nb bands)
// over columns C0 + 1 .. C0 + ncols, from a top row, a left column and a
// corner, to a bottom row and a right column. The row schedule hands top and
// bottom rows between workgroups as tagged granules (polled); a tile task of
// the promise DAG reads and writes the reference's plain arrays (its inputs
// are complete before it runs).
struct SwBand {
    int R0, C0, ncols, nb, bh;  // nb bands of bh = 64 R rows
    const int *leftcol;  // H(R0 + 1 + k, C0), k < 64 nb; null when C0 == 0
    int corner_h;        // H(R0, C0)
    int *rightcol;       // H(R0 + 1 + k, C0 + ncols) out, or null
    const unsigned long long *gin;  // top row as tagged granules, or
    const int *hin;                 // as plain H; both null: the boundary row (R0 == 0)
    unsigned long long *gout;       // bottom row as tagged granules, or
    int *hout;                      // as plain H, with
    int *corner_out;                //   its last value here (may be null)
    // DAG tile tasks: the left column / the next corner through LDS when the
    // workgroup ran the left neighbour itself (null / false otherwise)
    bool left_lds;       // leftcol points to LDS (plain loads)
    int *rightcol_lds;   // also keep the right column here
    int *corner_lds;     // H(R0, C0 + ncols): the right neighbour's corner
    int *corner_out_lds = nullptr;  // the bottom row's last value, also here
    // diagnostic (HX_DAG_TRACE builds): the tile task's trace record, where
    // waves 0 / 1 stamp their loop start ([12] / [15]); null otherwise
    unsigned long long *trec = nullptr;
};

// The workgroup's ingress wave: moves the top row into ring 0 and publishes
// prod[0], so that no compute wave ever waits on a global load. Granules are
// polled 128 columns per round trip (two loads per lane in flight) and the
// longest ready prefix is published.
__device__ bool sw_band_ingress(const SwCtx &c, const SwBand &B, int *ring0, int *prod, int *cons) {
    const int lane = lane_id();
    const int ncols = B.ncols;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int next = 0;
    for (uint32_t n = 1; next < ncols; ++n) {
        if (next + 128 - kSwRing > 0 && !sw_band_spin(c, &cons[0], next + 128 - kSwRing, t0)) return false;
        const int x0 = next + lane, x1 = x0 + 64;
        const int xa = x0 < ncols ? x0 : ncols - 1, xb = x1 < ncols ? x1 : ncols - 1;
        const int ga = B.R0 + (B.C0 + x0 + 1), gb = B.R0 + (B.C0 + x1 + 1);  // H -> G
        int m;
        if (B.gin) {
            // every other poll reads through this XCD's L2 (an sc0 load): the
            // up workgroup normally runs on the same XCD (see k_sw_band_rows),
            // whose L2 holds its write-through stores at once; the agent-scope
            // polls in between keep the hand-off correct on any placement
            unsigned long long a, b;
            if (n & 1) {
                a = __hip_atomic_load(&B.gin[xa], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                b = __hip_atomic_load(&B.gin[xb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                a = ld_agent(&B.gin[xa]);
                b = ld_agent(&B.gin[xb]);
            }
            const bool ra = (a >> 32) == 1ull || x0 >= ncols, rb = (b >> 32) == 1ull || x1 >= ncols;
            const unsigned long long ba = __ballot(ra), bb = __ballot(rb);
            m = ~ba ? __builtin_ctzll(~ba) : (~bb ? 64 + __builtin_ctzll(~bb) : 128);
            if (lane < m) ring0[x0 & (kSwRing - 1)] = (int)(uint32_t)a + ga;
            if (lane + 64 < m) ring0[x1 & (kSwRing - 1)] = (int)(uint32_t)b + gb;
        } else {
            // complete inputs (a DAG tile's) or the boundary row, H(0, c) = -c:
            // 256 columns per round trip (four loads per lane in flight)
            const int x2 = x0 + 128, x3 = x0 + 192;
            const int xc = x2 < ncols ? x2 : ncols - 1, xd = x3 < ncols ? x3 : ncols - 1;
            int ha = 0, hb = 0, hc = 0, hd = 0;
            if (B.hin) {
                ha = ld_agent(&B.hin[xa]);
                hb = ld_agent(&B.hin[xb]);
                if (next + 128 < ncols) {
                    hc = ld_agent(&B.hin[xc]);
                    hd = ld_agent(&B.hin[xd]);
                }
            }
            const bool four = next + 128 < ncols && next + 256 - kSwRing <= lds_flag_ld(&cons[0]);
            if (B.corner_lds) {  // H(R0, C0 + ncols): the top row's last value
                const int lx = ncols - 1 - next;
                const int hl = !B.hin ? -(B.C0 + ncols) : (lx == lane ? ha : lx == lane + 64 ? hb : lx == lane + 128 ? hc : hd);
                if (lx >= 0 && lx < 256 && (lx & 63) == lane) *B.corner_lds = hl;
            }
            ring0[x0 & (kSwRing - 1)] = B.hin ? ha + ga : 0;
            ring0[x1 & (kSwRing - 1)] = B.hin ? hb + gb : 0;
            if (four) {
                ring0[x2 & (kSwRing - 1)] = B.hin ? hc + B.R0 + (B.C0 + x2 + 1) : 0;
                ring0[x3 & (kSwRing - 1)] = B.hin ? hd + B.R0 + (B.C0 + x3 + 1) : 0;
            }
            m = four ? 256 : 128;
        }
        if (m > 0) {
            next = next + m < ncols ? next + m : ncols;
            if (lane == 0) lds_flag_st(&prod[0], next);
        } else {
            __builtin_amdgcn_s_sleep(2);
            if ((n & 255) == 0) {
                if (ld_agent(c.err)) return false;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * c.spin_ms) {
                    if (lane == 0) dev_error(c.err, kErrSpinTimeout);
                    return false;
                }
            }
        }
    }
    return true;
}

// The workgroup's egress wave: stores the last band's bottom row (ring nb)
// as granules or plain H, up to 64 columns per batch, and publishes
// cons[nb]; the compute waves issue no global stores but the right column.
__device__ bool sw_band_egress(const SwCtx &c, const SwBand &B, int *ring, int *prod, int *cons) {
    const int lane = lane_id();
    const int ncols = B.ncols, nb = B.nb, Rb = B.R0 + B.bh * nb;  // matrix row of the bottom row
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int next = 0;
    while (next < ncols) {
        const int want = next + kSwSub < ncols ? next + kSwSub : ncols;
        if (!sw_band_spin(c, &prod[nb], want, t0)) return false;
        int avail = lds_flag_ld(&prod[nb]);
        avail = avail < next + 64 ? avail : next + 64;
        const int x = next + lane;
        if (x < avail) {
            const int h = ring[x & (kSwRing - 1)] - Rb - (B.C0 + x + 1);
            if (B.gout) st_agent(&B.gout[x], (1ull << 32) | (unsigned long long)(uint32_t)h);
            else st_agent(&B.hout[x], h);
            if (B.corner_out && x == ncols - 1) st_agent(B.corner_out, h);
            if (B.corner_out_lds && x == ncols - 1) *B.corner_out_lds = h;
        }
        next = avail;
        if (lane == 0) lds_flag_st(&cons[nb], next);
    }
    return true;
}

// One wave's band (band w of the workgroup's nb) over the band's columns,
// skew S, hand-offs every K steps. Returns false on a device error.
// Diagnostic build only (HX_STAMPS): ph[0] compute, [1] waiting for the top
// row, [2] waiting for ring space + staging codes, [3] publishing (cycles).
template <int S, int K, int R>
__device__ bool sw_band_row(const SwCtx &c, const SwBand &B, int w, int *rings, int *dummy, uint8_t *code_rings,
                            int *prod, int *cons, unsigned long long *ph, bool stamp_first) {
    static_assert(R == 1 || S == 1, "several rows per lane only with skew 1");
    constexpr int D = 63 * S;        // lane 63's lag in steps
    constexpr int CR = S == 1 ? 128 : 256;  // code ring columns (needs D + 64)
    unsigned long long ts = sw_stamp();
    auto phase = [&](int k) {
        if (HX_STAMPS) {
            const unsigned long long now = sw_stamp();
            ph[k] += now - ts;
            ts = now;
        }
    };
    const int lane = lane_id();
    const int C0 = B.C0, ncols = B.ncols;
    int *ring_in = rings + (size_t)w * kSwRingStride, *ring_out = ring_in + kSwRingStride;
    uint8_t *cr = code_rings + w * 2048;
    const int r = B.R0 + w * 64 * R + R * lane + 1;  // this lane's (first) matrix row
    const uint32_t mrow = sw_row2(c.s2[r - 1]);
    // G at (r, C0) and (r - 1, C0): the band's left column
    auto left_h = [&](int row) {
        return C0 == 0 ? -row
                       : (row == B.R0 ? B.corner_h
                                      : (B.left_lds ? B.leftcol[row - B.R0 - 1] : ld_agent(&B.leftcol[row - B.R0 - 1])));
    };
    int left = left_h(r) + r + C0;
    int diag = left_h(r - 1) + (r - 1) + C0;
    int o2 = left;
    // R > 1: the lane's rows r .. r + R - 1 (lr[0] is `left`'s role)
    uint32_t mr[R];
    int lr[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        mr[q] = sw_row2(c.s2[r - 1 + q]);
        lr[q] = left_h(r + q) + (r + q) + C0;
    }
    int *wbase = lane == 63 ? ring_out : dummy + w * kSwDummy + lane;
    const int8_t *s1 = c.s1 + C0;
    // s1 code (1..4) of column x; loads clamped to the band, never predicated,
    // so that nothing waits for them before their use
    auto code_at = [&](int x) { return s1[x < ncols ? x : ncols - 1]; };
    // copy o holds column x's code - 1 at byte (x + o) mod CR (and + CR), so
    // lane L reads aligned words from copy (S L) mod 4
    auto stage_codes = [&](int x, int code) {
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            const int q = (x + o) & (CR - 1);
            cr[o * 2 * CR + q] = (uint8_t)(code - 1);
            cr[o * 2 * CR + q + CR] = (uint8_t)(code - 1);
        }
    };
    stage_codes(lane, code_at(lane));
    const int cofs = (S * lane) & 3;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    // (SHIFT, lane 63's outputs gathered by DPP and stored once per 64-step
    // chunk: the one-tile-row sweep 57 -> 55 cycles per step, but the DAG
    // 8.12 -> 8.55 ms, profiles/r03/sw_shift_ab.log; not built)
    constexpr bool kShift = false;
    int acc = 0;
    // (trace builds: the loop start only — a stamp inside the loop, an SMEM
    // read, waits for every LDS operation in flight and slows the sweep)
    if (HX_DAG_TRACE && B.trec && lane == 0 && w < 2) B.trec[w == 0 ? 12 : 15] = __builtin_amdgcn_s_memrealtime();
    for (int s0 = 0; ok && s0 < ncols + D; s0 += 64) {
        const int slot = s0 & (kSwRing - 1);
        // ring_out's slots for columns s0 - D .. s0 + 63 - D are free
        if (s0 + 64 - D - kSwRing > 0 && !sw_band_spin(c, &cons[w + 1], s0 + 64 - D - kSwRing, t0)) {
            ok = false;
            break;
        }
        // the next chunk's codes (staged after this chunk's last read)
        const int craw = code_at(s0 + 64 + lane);
        const uint32_t *cb = (const uint32_t *)(cr + cofs * 2 * CR + ((s0 - S * lane + cofs) & (CR - 1)));
        int *wb = wbase + (lane == 63 ? ((s0 - D) & (kSwRing - 1)) : 0);
        const bool full = s0 >= D && s0 + 64 <= ncols;
        phase(s0 == 0 ? 4 : 2);
#pragma unroll
        for (int q = 0; q < 64 / K; ++q) {
            const int s = s0 + q * K;
            // this hand-off's top row: columns s .. s + K - 1 of ring_in
            if (!sw_band_spin(c, &prod[w], s + K < ncols ? s + K : ncols, t0)) {
                ok = false;
                break;
            }
            if (HX_STAMPS && s == 0 && w == 0 && lane == 0 && stamp_first) {
                // first input of the tile row (global clock): rows' start spacing
                const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                if (B.R0 == c.i0 * c.th) st_agent(&c.stats[27], now);
                if (B.R0 + B.bh * B.nb == c.i1 * c.th) st_agent(&c.stats[26], now);
            }
            phase(1);
            if (R > 1) {
                if (full)
                    sw_band_subR<false, K, R, kShift>(s, ncols, ring_in + slot + q * K, cb + q * (K / 4), wb + q * K,
                                                      mr, lr, diag, acc);
                else
                    sw_band_subR<true, K, R, kShift>(s, ncols, ring_in + slot + q * K, cb + q * (K / 4), wb + q * K,
                                                     mr, lr, diag, acc);
            } else if (full) {
                sw_band_sub<false, S, K, kShift>(s, ncols, ring_in + slot + q * K, cb + q * (K / 4), wb + q * K, mrow,
                                                 left, diag, o2, acc);
            } else {
                sw_band_sub<true, S, K, kShift>(s, ncols, ring_in + slot + q * K, cb + q * (K / 4), wb + q * K, mrow,
                                                left, diag, o2, acc);
            }
            if (kShift) {
                // the chunk's 64 outputs of lane 63 (columns s0 - D .. s0 + 63
                // - D), one per lane: the slots the per-step stores filled
                ring_out[((s0 - D) & (kSwRing - 1)) + lane] = acc;
            }
            phase(0);
            // lane 63's last S columns of the chunk may have gone past the
            // ring's end (wrap slots): they are also stored at their own slots
            if (q == 64 / K - 1 && lane == 63) {
                ring_out[(s0 + 63 - D) & (kSwRing - 1)] = R > 1 ? lr[R - 1] : left;
                if (S == 2) ring_out[(s0 + 62 - D) & (kSwRing - 1)] = o2;
            }
            // publish: ring_out holds columns < s + K - D, ring_in's columns
            // < s + K are read
            if (lane == 0) {
                const int pc = s + K - D;
                lds_flag_st(&prod[w + 1], pc < 0 ? 0 : (pc < ncols ? pc : ncols));
                lds_flag_st(&cons[w], s + K);
            }
            phase(3);
        }
        stage_codes(s0 + 64 + lane, craw);
    }
    if (HX_STAMPS && stamp_first && w == B.nb - 1 && lane == 0 && B.R0 + B.bh * B.nb == c.i1 * c.th)
        st_agent(&c.stats[28], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (ok && B.rightcol) {
        if (R == 1) st_agent(&B.rightcol[r - B.R0 - 1], left - r - (C0 + ncols));
#pragma unroll
        for (int q = 0; R > 1 && q < R; ++q) st_agent(&B.rightcol[r - B.R0 - 1 + q], lr[q] - (r + q) - (C0 + ncols));
    }
    if (ok && B.rightcol_lds) {
        if (R == 1) B.rightcol_lds[r - B.R0 - 1] = left - r - (C0 + ncols);
#pragma unroll
        for (int q = 0; R > 1 && q < R; ++q) B.rightcol_lds[r - B.R0 - 1 + q] = lr[q] - (r + q) - (C0 + ncols);
    }
    return ok;
}

// the (rows per lane, skew, hand-off) forms: HCLIB_HIP_SW_FORM =
// 100 R + 10 S + K / 16 (sw_pick_form keeps to the valid ones)
__device__ __forceinline__ bool sw_band_row_any(int form, const SwCtx &c, const SwBand &B, int w, int *rings,
                                                int *dummy, uint8_t *code_rings, int *prod, int *cons,
                                                unsigned long long *ph, bool stamp_first) {
    switch (form) {
        case 11: return sw_band_row<1, 16, 1>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 12: return sw_band_row<1, 32, 1>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 14: return sw_band_row<1, 64, 1>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 21: return sw_band_row<2, 16, 1>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 22: return sw_band_row<2, 32, 1>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 211: return sw_band_row<1, 16, 2>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 212: return sw_band_row<1, 32, 2>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 411: return sw_band_row<1, 16, 4>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 412: return sw_band_row<1, 32, 4>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        case 214: return sw_band_row<1, 64, 2>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
        default: return sw_band_row<1, 64, 4>(c, B, w, rings, dummy, code_rings, prod, cons, ph, stamp_first);
    }
}

// A workgroup runs k consecutive tile rows (k * th / 64 compute waves, then
// the ingress and the egress wave): only every k-th tile row boundary
// crosses workgroups through global memory.
__global__ __launch_bounds__(1024) void k_sw_band_rows(SwCtx c) {
    extern __shared__ __attribute__((aligned(16))) int sw_lds[];
    const int nwave = (int)(blockDim.x >> 6) - 2, w = (int)(threadIdx.x >> 6);
    const int bpt = c.th / c.bh, k = nwave / bpt;
    int *rings = sw_lds;
    int *dummy = rings + (size_t)(nwave + 1) * kSwRingStride;
    uint8_t *code_rings = (uint8_t *)(dummy + nwave * kSwDummy);
    int *prod = (int *)(code_rings + nwave * 2048), *cons = prod + 64;
    const size_t gstride = (size_t)c.ntw * c.tw;  // granules per tile row
    bool ok = true;
    unsigned long long ntile = 0;
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
    // blocks of k tile rows; with the grid a multiple of the 8 XCDs, block
    // positions are dealt so that consecutive blocks run on one XCD (the
    // dispatcher places workgroup b on XCD b mod 8 — for speed only: every
    // hand-off is correct on any placement). Each workgroup takes its blocks
    // in increasing order and all are resident, so every wait ends.
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    const int p0 = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
    for (int i = c.i0 + p0 * k; i < c.i1; i += G * k) {
        const int kk = k < c.i1 - i ? k : c.i1 - i;  // tile rows of this block
        SwBand B;
        B.R0 = i * c.th;
        B.C0 = c.j0 * c.tw;
        B.ncols = (c.j1 - c.j0) * c.tw;
        B.nb = kk * bpt;
        B.bh = c.bh;
        B.leftcol = c.j0 > 0 ? c.left_in + B.R0 : nullptr;
        B.corner_h = B.R0 == 0 ? -B.C0 : (c.j0 == 0 ? -B.R0 : (c.j0 > 0 ? ld_agent(&c.left_in[B.R0 - 1]) : 0));
        B.rightcol = c.right_out ? c.right_out + B.R0 : nullptr;
        B.gin = i > 0 ? c.gbot + (size_t)(i - 1) * gstride + B.C0 : nullptr;
        B.hin = nullptr;
        B.gout = c.gbot + (size_t)(i + kk - 1) * gstride + B.C0;
        B.hout = nullptr;
        B.corner_out = nullptr;
        B.left_lds = false;
        B.rightcol_lds = nullptr;
        B.corner_lds = nullptr;
        if (threadIdx.x < 128) prod[threadIdx.x] = 0;  // prod[0..63], cons[0..63]
        __syncthreads();
        if (w == nwave)
            ok = sw_band_ingress(c, B, rings, prod, cons);
        else if (w == nwave + 1)
            ok = sw_band_egress(c, B, rings + (size_t)B.nb * kSwRingStride, prod, cons);
        else if (w < B.nb)
            ok = sw_band_row_any(c.form, c, B, w, rings, dummy, code_rings, prod, cons, ph, true);
        vm_drain();
        if (__syncthreads_or(!ok)) break;  // every wave leaves together
        ntile += (unsigned long long)(c.j1 - c.j0) * kk;
    }
    if (threadIdx.x == 0) add_agent(&c.stats[0], ntile);
    if (HX_STAMPS && lane_id() == 0 && w < 4)  // per compute wave (first four)
        for (int q = 0; q < 6 && w < 3; ++q) add_agent(&c.stats[4 + 6 * w + q], ph[q]);
}

// The generic device promise DAG (include/hclib_hip/hx_dag.h) driving the
// reference's tile program as written: every tile is an async_await on three
// futures (left tile's right column, up tile's bottom row, diagonal tile's
// corner, smith_waterman.cpp:227-229) and puts three promises when done
// (:212-226). The boundary promises the reference puts before the loop
// (:141-165) are simply not awaited.
struct SwDagKind {
    using Ctx = SwCtx;
    __device__ static void run(const SwCtx &c, DagWave &w, uint32_t t, const uint32_t *) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        int *lds_top = sw_lds;
        int *lds_bot = sw_lds + ((c.tw + 1 + 3) & ~3);
        int8_t *lds_s1 = (int8_t *)(lds_bot + ((c.tw + 1 + 3) & ~3) + 68);
        unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
        int corner_unused = 0;
        __syncthreads();
        sw_tile<false>(c, t, lds_top, lds_bot, lds_s1, nullptr, nullptr, corner_unused, ph);
        // right column, bottom row, corner (:212-226): one release for all three
        const uint32_t ps[3] = {3u * t + 0u, 3u * t + 1u, 3u * t + 2u};
        const unsigned long long ds[3] = {0ull, 0ull, (unsigned long long)(uint32_t)ld_agent(&c.corner[t])};
        dag_put_n<3>(w, ps, ds);
    }
};

__global__ __launch_bounds__(64) void k_sw_dag(SwCtx c, DagView v) {
    run_dag_worker<SwDagKind>(c, v);
}

// The same tile program with every tile task run by a workgroup: th / 64
// compute waves (one 64-row band each, chained through LDS rings as in the
// row schedule) plus the ingress wave (the up tile's bottom row into ring 0)
// and the egress wave (the bottom row and corner out); the tile's three
// promises are put by wave 0 once every wave's stores are drained.
struct SwDagWgKind {
    using Ctx = SwCtx;
    // every tile input from another task (top row, left column, corner) is
    // read with ld_agent and written with st_agent: no fences needed
    static constexpr bool kSc1Payload = true;
    __device__ static bool run_group(const SwCtx &c, uint32_t t, const uint32_t *, int wave) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        const int nw = c.th / c.bh;
        int *rings = sw_lds;
        int *dummy = rings + (size_t)(nw + 1) * kSwRingStride;
        uint8_t *code_rings = (uint8_t *)(dummy + nw * kSwDummy);
        int *prod = (int *)(code_rings + nw * 2048), *cons = prod + 64;
        // the workgroup's last tile: its right column (two buffers by tile
        // parity) and its right neighbour's corner, for a row successor
        int *last = cons + 64, *corner_keep = last + 1, *right_keep = last + 4;  // [2][th]
        const int i = (int)(t / (uint32_t)c.ntw), j = (int)(t % (uint32_t)c.ntw);
        // `last` (the workgroup's previous tile) and the zeroed prod / cons
        // flags were written by after_body before the DAG's slot barrier:
        // the body starts without a barrier of its own
        const bool from_lds = j > 0 && *last == (int)t - 1;
        SwBand B;
        B.R0 = i * c.th;
        B.C0 = j * c.tw;
        B.ncols = c.tw;
        B.nb = nw;
        B.bh = c.bh;
        B.left_lds = from_lds;
        B.leftcol = j == 0 ? nullptr : (from_lds ? right_keep + ((t - 1) & 1) * c.th : c.right + (size_t)(t - 1) * c.th);
        B.corner_h = B.R0 == 0 ? -B.C0
                               : (j == 0 ? -B.R0 : (from_lds ? corner_keep[(t - 1) & 1]
                                                             : ld_agent(&c.corner[t - (uint32_t)c.ntw - 1])));
        B.rightcol_lds = right_keep + (t & 1) * c.th;
        B.corner_lds = corner_keep + (t & 1);
        B.rightcol = c.right + (size_t)t * c.th;
        B.gin = nullptr;
        B.hin = i > 0 ? c.bottom + (size_t)(t - (uint32_t)c.ntw) * c.tw : nullptr;
        B.gout = nullptr;
        B.hout = c.bottom + (size_t)t * c.tw;
        B.corner_out = c.corner + t;
        B.corner_out_lds = last + 3;  // the corner promise's datum (datums())
        B.trec = HX_DAG_TRACE && c.dtrace ? c.dtrace + (size_t)t * kDagTraceWords : nullptr;
        unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
        // trace words 8.. (stamps build): [8] ingress done, [9] egress done,
        // [10 + w] compute wave w done
        auto tstamp = [&](int k) {
            if (HX_DAG_TRACE && c.dtrace && lane_id() == 0)
                c.dtrace[(size_t)t * kDagTraceWords + k] = __builtin_amdgcn_s_memrealtime();
        };
        if (wave == nw) {
            const bool r = sw_band_ingress(c, B, rings, prod, cons);
            tstamp(8);
            return r;
        }
        if (wave == nw + 1) {
            const bool r = sw_band_egress(c, B, rings + (size_t)nw * kSwRingStride, prod, cons);
            tstamp(9);
            return r;
        }
        const bool ok = sw_band_row_any(c.form, c, B, wave, rings, dummy, code_rings, prod, cons, ph, false);
        if (wave < 6) tstamp(10 + wave);
        if (HX_STAMPS && lane_id() == 0 && wave < 4)
            for (int q = 0; q < 6 && wave < 3; ++q) add_agent(&c.stats[4 + 6 * wave + q], ph[q]);
        return ok;
    }
    // between tiles (every wave done with this one): the hand-off flags back
    // to 0 and this tile recorded as the workgroup's last, for the next body
    __device__ static void after_body(const SwCtx &c, uint32_t t) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        int *prod = flags_of(c), *last = prod + 128;
        if (threadIdx.x < 128) prod[threadIdx.x] = 0;  // prod[0..63], cons[0..63]
        if (threadIdx.x == 0) *last = (int)t;
    }
    __device__ static int *flags_of(const SwCtx &c) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        const int nw = c.th / c.bh;
        return (int *)((uint8_t *)(sw_lds + (size_t)(nw + 1) * kSwRingStride + nw * kSwDummy) + nw * 2048);
    }
    // right column, bottom row, corner (:212-226): run_dag_group's split put
    // (waiters prefetched while the tile runs, one release for all three)
    static constexpr int kPutN = 3;
    __device__ static void promises(const SwCtx &, uint32_t t, uint32_t (&p)[3]) {
        p[0] = 3u * t + 0u;
        p[1] = 3u * t + 1u;
        p[2] = 3u * t + 2u;
    }
    __device__ static void datums(const SwCtx &c, uint32_t t, unsigned long long (&d)[3]) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        const int nw = c.th / c.bh;
        const int *last = (const int *)((const uint8_t *)(sw_lds + (size_t)(nw + 1) * kSwRingStride + nw * kSwDummy) +
                                        nw * 2048) + 128;
        (void)t;
        d[0] = 0ull;
        d[1] = 0ull;
        d[2] = (unsigned long long)(uint32_t)last[3];  // the egress wave's copy of c.corner[t]
    }
};

__global__ __launch_bounds__(1024) void k_sw_dag_wg(SwCtx c, DagView v) {
    extern __shared__ __attribute__((aligned(16))) int sw_lds[];
    __shared__ uint32_t task_slot;
    const int nw = c.th / c.bh;
    int *prod = (int *)((uint8_t *)(sw_lds + (size_t)(nw + 1) * kSwRingStride + nw * kSwDummy) + nw * 2048);
    int *last = prod + 128;
    if (threadIdx.x < 128) prod[threadIdx.x] = 0;  // prod / cons (after_body resets them between tiles)
    if (threadIdx.x == 0) *last = -2;  // no tile yet (run_dag_group's first barrier orders these)
    run_dag_group<SwDagWgKind>(c, v, &task_slot);
}

// ------------------------------------------------ packed-half tile bodies
// A 256-row tile in ONE wave, two cells per VALU operation (gfx950
// v_pk_maximum3_f16 / v_pk_add_f16). Inside a tile the G values (G = H + row
// + col, see sw_tile) are kept relative to the tile's corner,
// v = G - G(R0, C0). G never decreases along a row or a column and grows by
// at most 4 per diagonal step, so 0 <= v <= 4 max(di, dj) <= 2048 for tiles
// of at most 256 x 512 cells (and v - 2 >= -2 for a diagonal plus score):
// integers every f16 holds exactly, so the packed max/add are exact and the
// outputs bit-identical to the int32 forms.
// Lane L holds rows 2L, 2L+1 of the tile's top half in the low halves of
// lr0 / lr1 and rows 128+2L, 129+2L in the high halves; the bottom half
// runs 64 steps behind the top (the same anti-diagonal pipeline continued
// through lane 63 -> lane 0): at step s the low halves compute column
// x = s - L, the high halves x - 64. The cell above a lane's first row comes
// from lane L-1 (one DPP wave rotation); lane 0 takes the top row (low
// half) and lane 63's low row 127 (high half) through one byte permute with
// a per-lane selector. No masks: a column outside the tile has the "null"
// code, whose score byte is 0, and the top row is 0 beyond the tile — since
// G is monotone, max3(left, up, diag + 0) then leaves every row at its left
// value before the tile and at its right-column value after it.
typedef _Float16 sw_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ sw_h2 sw_as_h2(uint32_t v) { return __builtin_bit_cast(sw_h2, v); }
__device__ __forceinline__ uint32_t sw_as_u(sw_h2 v) { return __builtin_bit_cast(uint32_t, v); }
// f16 bits of an exact small integer (|v| <= 2048)
__device__ __forceinline__ uint32_t sw_f16_bits(int v) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)v);
}
// the score row of s2 code a as the HIGH bytes of f16 (score + 2 = 4, 0 or -2
// -> 0x44, 0x00, 0xC0; the low byte of each is 0): byte c for s1 code c + 1
__device__ __forceinline__ uint32_t sw_pk_row(int a) {
    return a == 1 ? 0xC000C044u : a == 2 ? 0x00C044C0u : a == 3 ? 0xC044C000u : 0x44C000C0u;
}
constexpr uint32_t kSwPkNull = 0x0Cu;  // v_perm selector byte of a constant 0x00
constexpr int kSwPkTh = 256;            // tile rows the packed body covers
constexpr int kSwPkMaxTw = 512;         // f16 exactness bound (see above)
// LDS words of the packed body's arrays for tiles ncols wide: the top row
// (x < ncols + 196, zeros past the tile) and four copies of the per-column
// permute selectors (x in [-64, ncols + 200)), copy o at word x + 64 + o
__host__ __device__ constexpr int sw_pk_topw(int ncols) { return (ncols + 196 + 3) & ~3; }
__host__ __device__ constexpr int sw_pk_selw(int ncols) { return (ncols + 268 + 3) & ~3; }

// Inputs and outputs in global memory are tagged granules {1 << 32 | H}:
// a reader polls the tags, so the producing tile's put need not wait for its
// stores to drain (SwDagPkKind::kTagged).
typedef unsigned long long sw_gran;
__device__ __forceinline__ sw_gran sw_granule(int h) { return (1ull << 32) | (uint32_t)h; }
struct SwPkTile {
    int R0, C0, ncols;
    const sw_gran *corner_src;  // H(R0, C0) from memory, or null:
    int corner_val;             //   this value (every v is G - G(R0, C0))
    const sw_gran *hin;         // top row (null: the boundary row, R0 == 0, or:)
    const int *top_lds;         // the top row's H already in LDS, or null
    const sw_gran *leftcol;     // H(R0 + 1 + k, C0), k < 256, in global memory, or null:
    const int *left_lds;        //   in LDS (the workgroup ran the left tile), or null: C0 == 0
    sw_gran *hout;              // bottom row out
    sw_gran *rightcol;          // right column out (global), may be null
    int *rightcol_lds;          // ... and in LDS, may be null
    sw_gran *corner_out;        // H(R0 + 256, C0 + ncols) out, may be null
    int *corner_out_lds;        // ... and in LDS, may be null
    int *corner_lds;            // H(R0, C0 + ncols) (the top row's last) into LDS, may be null
    // diagnostic (HX_DAG_TRACE builds): the task's trace record — [8] inputs
    // staged, [10] sweep done, [11] outputs issued; null otherwise
    unsigned long long *trec = nullptr;
};

// The tile as two waves of one workgroup: the sweep wave (wave 0) runs the
// dependent chain; the score wave (wave 1) feeds it the packed score words
// of every step through an LDS ring, so the sweep issues no score lookups.
// One wave issues at most one VALU operation per ~5 cycles whatever the rest
// of the CU does (profiles/r03/ub_valu.log), so a step's cost is its
// instruction count: moving the two lookups (v_perm) and the selector loads
// to a second wave leaves the sweep rot + up + 2 adds + 2 max3 + half a
// gather and half a ring load per step.
// Ring: kSwPkSlots chunks of 64 steps; a chunk is 32 step pairs x 64 lanes of
// uint4 {sc0(2p), sc1(2p), sc0(2p+1), sc1(2p+1)}. misc[5] = chunks written,
// misc[6] = chunks read (both reset between tiles).
constexpr int kSwPkSlots = 2;
// the sweep's operand prefetch distance (groups of 4 steps; 1-3 measured
// flat, profiles/r03/sw_pk_prefetch_ab.log)
constexpr int kSwPkPf = 3;
constexpr int kSwPkRingU4 = kSwPkSlots * 32 * 64;  // uint4 entries
// LDS: ring | top | sel x 4 | right columns [2][256] | misc[16] | score rows [4][64] | next top row [512]
constexpr int kSwPkMisc = 16;
__host__ __device__ constexpr int sw_pk_lds_words(int tw) {
    return kSwPkRingU4 * 4 + sw_pk_topw(tw) + 4 * sw_pk_selw(tw) + 2 * kSwPkTh + kSwPkMisc + 256 + kSwPkMaxTw;
}
inline size_t sw_pk_lds_bytes(int tw) { return (size_t)sw_pk_lds_words(tw) * 4; }

// wait until an LDS counter reaches `want` (bounded; device error on timeout)
// EQ: wait for the flag to equal `want` (a per-tile flag whose tiles are not
// monotone per workgroup: tile (1, 0) is id ntw and tile (0, 2) may run after
// it); otherwise for it to reach `want` (counters that only grow)
template <bool EQ = false>
__device__ __forceinline__ bool sw_pk_wait(const SwCtx &c, const int *flag, int want) {
    auto done = [&]() { return EQ ? lds_flag_ld(flag) == want : lds_flag_ld(flag) >= want; };
    if (done()) return true;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t n = 1; !done(); ++n) {
        __builtin_amdgcn_s_sleep(1);
        if ((n & 255) == 0) {
            if (ld_agent(c.err)) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * c.spin_ms) {
                if (lane_id() == 0) dev_error(c.err, kErrSpinTimeout);
                return false;
            }
        }
    }
    return true;
}

// The score wave's staging for a tile: its s1 codes as permute selectors
// (sel) and this lane's four score rows (tbl[q * 64 + lane]). Run for the
// tile itself, or ahead of time for the right neighbour (the tile the
// workgroup keeps when its own put releases it) while the sweep still runs.
// `mid` runs once the columns the first chunk reads (x < 64) and the score
// rows are staged (the first chunk's scores can start before the rest).
template <int KX, class Mid>
__device__ bool sw_pk_stage(const SwCtx &c, int R0, int C0, int ncols, int *sel, int *tbl, Mid &&mid) {
    const int lane = lane_id();
    const int selw = sw_pk_selw(ncols), xmax = ncols - 1;
    int code[KX];
#pragma unroll
    for (int k = 0; k < KX; ++k) {
        const int x = lane + 64 * k;
        code[k] = (int)c.s1[C0 + (x < ncols ? x : xmax)];
    }
    // this lane's rows: lo q0, lo q1, hi q0, hi q1 (as the sweep wave's)
    const int r0 = R0 + 1 + 2 * lane;
    const int s2a = c.s2[r0 - 1], s2b = c.s2[r0], s2c = c.s2[r0 + 127], s2d = c.s2[r0 + 128];
#pragma unroll
    for (int k = 0; k < KX; ++k)
        if (lane + 64 * k >= ncols) code[k] = (int)kSwPkNull;
        else code[k] -= 1;
    // selectors: word x = [hi: 4 + code(x - 64) | null][0x0C][lo: code(x)][0x0C]
    // (the score bytes of the low and the high half: S1 = the low rows' row,
    // S0 = the high rows'), staged for x in [-64, ncols + 200) in four copies
    // so that lane L reads four consecutive columns from copy L & 3 aligned
    auto selword = [](int lo, int hi) {
        const uint32_t hs = hi == (int)kSwPkNull ? kSwPkNull : (uint32_t)(4 + hi);
        return kSwPkNull | ((uint32_t)lo << 8) | (kSwPkNull << 16) | (hs << 24);
    };
    // x = lane + 64 k - 64 for k = 0 .. KX + 5: lo code = code[k - 1], hi = code[k - 2]
    auto stage = [&](int k) {
        const int x = lane + 64 * k - 64;
        if (x < ncols + 200) {
            const int lo = (k >= 1 && k - 1 < KX) ? code[k - 1] : (int)kSwPkNull;
            const int hi = (k >= 2 && k - 2 < KX) ? code[k - 2] : (int)kSwPkNull;
            const uint32_t w = selword(lo, hi);
#pragma unroll
            for (int o = 0; o < 4; ++o) sel[o * selw + x + 64 + o] = (int)w;
        }
    };
    stage(0);
    stage(1);
    tbl[lane] = (int)sw_pk_row(s2a);
    tbl[64 + lane] = (int)sw_pk_row(s2b);
    tbl[128 + lane] = (int)sw_pk_row(s2c);
    tbl[192 + lane] = (int)sw_pk_row(s2d);
    if (!mid()) return false;
#pragma unroll
    for (int k = 2; k < KX + 6; ++k) stage(k);
    return true;
}

// The score wave: every chunk's scores from the staged selectors and rows.
__device__ bool sw_pk_scores(const SwCtx &c, int ncols, uint4 *ring, const int *sel, const int *tbl, int *misc,
                             int k0 = 0, int k1 = 1 << 30) {
    const int lane = lane_id();
    const int selw = sw_pk_selw(ncols);
    const uint32_t mlo0 = (uint32_t)tbl[lane], mlo1 = (uint32_t)tbl[64 + lane];
    const uint32_t mhi0 = (uint32_t)tbl[128 + lane], mhi1 = (uint32_t)tbl[192 + lane];
    const int *selp = sel + (lane & 3) * selw + 64 + (lane & 3) - lane;  // + s: column s - lane, aligned
    const int nch = (ncols + 127 + 63) / 64;
    for (int k = k0; k < nch && k < k1; ++k) {
        if (k >= kSwPkSlots && !sw_pk_wait(c, &misc[6], k + 1 - kSwPkSlots)) return false;
        uint4 *dst = ring + (size_t)((k % kSwPkSlots) * 32) * 64 + lane;
        const int *sp = selp + 64 * k;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int4 sv = *(const int4 *)(sp + 4 * g);
            dst[(2 * g) * 64] = make_uint4(__builtin_amdgcn_perm(mhi0, mlo0, (uint32_t)sv.x),
                                           __builtin_amdgcn_perm(mhi1, mlo1, (uint32_t)sv.x),
                                           __builtin_amdgcn_perm(mhi0, mlo0, (uint32_t)sv.y),
                                           __builtin_amdgcn_perm(mhi1, mlo1, (uint32_t)sv.y));
            dst[(2 * g + 1) * 64] = make_uint4(__builtin_amdgcn_perm(mhi0, mlo0, (uint32_t)sv.z),
                                               __builtin_amdgcn_perm(mhi1, mlo1, (uint32_t)sv.z),
                                               __builtin_amdgcn_perm(mhi0, mlo0, (uint32_t)sv.w),
                                               __builtin_amdgcn_perm(mhi1, mlo1, (uint32_t)sv.w));
        }
        if (lane == 0) lds_flag_st(&misc[5], k + 1);
    }
    return true;
}

// The sweep wave: the tile's inputs, the sweep, its outputs. top: this
// workgroup's top-row array (sw_pk_topw words, 16-byte aligned). KX =
// columns per lane (ncols <= 64 KX).
template <int KX>
__device__ bool sw_pk_tile(const SwCtx &c, const SwPkTile &T, int *top, const uint4 *ring, int *misc) {
    const int lane = lane_id();
    const int ncols = T.ncols, R0 = T.R0, C0 = T.C0;
    const int topw = sw_pk_topw(ncols);
    // --- loads, all issued before any is used, none predicated (a
    // predicated load becomes a branch that waits for it on its own): the left
    // column, the top row and the corner (other tasks' granules, polled until
    // every tag is set — normally at once: their stores were issued before the
    // puts that released this tile). Unused operands read a valid word.
    const int xmax = ncols - 1;
    int rowq[4];  // matrix rows of lo q0, lo q1, hi q0, hi q1
    rowq[0] = R0 + 1 + 2 * lane;
    rowq[1] = rowq[0] + 1;
    rowq[2] = rowq[0] + 128;
    rowq[3] = rowq[1] + 128;
    const bool lglob = T.leftcol != nullptr;
    const sw_gran *lsrc = lglob ? T.leftcol : T.hout;
    const sw_gran *hsrc = T.hin ? T.hin : T.hout;
    sw_gran lg[4], th_[KX], cg = 0;
    if (HX_DAG_TRACE && T.trec && lane == 0) T.trec[14] = __builtin_amdgcn_s_memrealtime();  // body entered
#pragma unroll
    for (int q = 0; q < 4; ++q) lg[q] = 0;
#pragma unroll
    for (int k = 0; k < KX; ++k) th_[k] = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // (a kept tile whose top row the score wave already took reads nothing)
    for (uint32_t n = 0; T.hin || lglob || T.corner_src; ++n) {
#pragma unroll
        for (int q = 0; q < 4; ++q) lg[q] = ld_agent(&lsrc[lglob ? rowq[q] - R0 - 1 : 0]);
#pragma unroll
        for (int k = 0; k < KX; ++k) {
            const int x = lane + 64 * k;
            th_[k] = ld_agent(&hsrc[T.hin ? (x < ncols ? x : xmax) : 0]);
        }
        cg = ld_agent(T.corner_src ? T.corner_src : T.hout);
        bool ready = !T.corner_src || (cg >> 32) == 1ull;
#pragma unroll
        for (int q = 0; q < 4; ++q) ready = ready && (!lglob || (lg[q] >> 32) == 1ull);
#pragma unroll
        for (int k = 0; k < KX; ++k) ready = ready && (!T.hin || (th_[k] >> 32) == 1ull);
        if (__ballot(!ready) == 0) break;
        __builtin_amdgcn_s_sleep(1);
        if ((n & 63) == 63) {
            if (ld_agent(c.err)) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull * c.spin_ms) {
                if (lane == 0) dev_error(c.err, kErrSpinTimeout);
                return false;
            }
        }
    }
    if (HX_DAG_TRACE && T.trec && lane == 0) {
        T.trec[15] = __builtin_amdgcn_s_memrealtime();  // inputs loaded
        // [13]: where the inputs came from (scripts/sw_dag_trace.py)
        T.trec[13] = (T.top_lds ? 1ull : 0ull) | (T.hin ? 2ull : 0ull) | (lglob ? 4ull : 0ull) |
                     (T.corner_src ? 8ull : 0ull) | (T.left_lds ? 16ull : 0ull);
    }
    const int cget = (int)(uint32_t)cg;
    // the LDS inputs, every load issued before any is used: read per element
    // inside the conversion below, each load was a branch of its own and
    // waited behind the previous element's store (the arrays may alias) —
    // 0.9 us of a kept hop's 1.7 before its sweep (profiles/r05/sw_trace.json)
    const lds_i32 *lsl = (const lds_i32 *)(T.left_lds ? T.left_lds : (const int *)top);
    const lds_i32 *tsl = (const lds_i32 *)(T.top_lds ? T.top_lds : (const int *)top);
    int lq[4], tq[KX];
#pragma unroll
    for (int q = 0; q < 4; ++q) lq[q] = lsl[T.left_lds ? rowq[q] - R0 - 1 : 0];
#pragma unroll
    for (int k = 0; k < KX; ++k) {
        const int x = lane + 64 * k;
        tq[k] = tsl[T.top_lds && x < ncols ? x : 0];
    }
    int lh[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) lh[q] = T.left_lds ? lq[q] : (lglob ? (int)(uint32_t)lg[q] : -rowq[q]);
    // --- the left column as packed v
    const int base = (T.corner_src ? cget : T.corner_val) + R0 + C0;  // G(R0, C0)
    uint32_t l16[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) l16[q] = sw_f16_bits(lh[q] + rowq[q] + C0 - base);
    sw_h2 lr0 = sw_as_h2(l16[0] | (l16[2] << 16)), lr1 = sw_as_h2(l16[1] | (l16[3] << 16));
    // --- the top row as v (f16 in the low half), 0 past the tile
    // (branch-free per element: selects, one predicated store)
    const bool from_hin = T.hin != nullptr, top_known = T.hin != nullptr || T.top_lds != nullptr;
#pragma unroll
    for (int k = 0; k < KX + 4; ++k) {
        const int x = lane + 64 * k;
        int v = 0;
        if (k < KX) {
            const int src = from_hin ? (int)(uint32_t)th_[k] : tq[k];
            const int vk = top_known ? src + R0 + (C0 + 1 + x) - base : -base;
            v = x < ncols ? vk : 0;
        }
        const int bits = (int)sw_f16_bits(v);
        if (x < topw) top[x] = bits;
    }
    if (T.corner_lds) {
        // H(R0, C0 + ncols): the up tile's last bottom value (or the boundary)
        const int xl = ncols - 1;
        if ((xl & 63) == lane) {
            int h = -(C0 + ncols);
#pragma unroll
            for (int k = 0; k < KX; ++k)
                if (k == (xl >> 6) && T.hin) h = (int)(uint32_t)th_[k];
            if (T.top_lds) h = *((const lds_i32 *)T.top_lds + xl);
            *T.corner_lds = h;
        }
    }
    auto tstamp = [&](int k) {
        if (HX_DAG_TRACE && T.trec && lane == 0) T.trec[k] = __builtin_amdgcn_s_memrealtime();
    };
    tstamp(8);
    // --- the sweep: S = ncols + 127 steps in chunks of 64; the tile's bottom
    // row (lane 63's high row 255) leaves in pairs of steps, one DPP shift
    // per pair (see the chunk's end)
    const uint32_t selU = lane == 0 ? 0x05040100u : 0x07060504u;
    // the up value of step -1 (lane 0's top-row input: the corner, v = 0)
    sw_h2 upp = sw_as_h2(__builtin_amdgcn_perm((uint32_t)__builtin_amdgcn_mov_dpp((int)sw_as_u(lr1), 0x13C, 0xf, 0xf, false),
                                               0u, selU));
    const int nsteps = ncols + 127;
    const int Rb = R0 + kSwPkTh;  // the bottom row's matrix row
    for (int s0 = 0, k = 0; s0 < nsteps; s0 += 64, ++k) {
        if (!sw_pk_wait(c, &misc[5], k + 1)) return false;
        if (k == 0) tstamp(12);  // the first chunk's scores are there
        const uint4 *src = ring + (size_t)((k % kSwPkSlots) * 32) * 64 + lane;
        uint32_t acc = 0;
        // operands of group g + kPf are loaded while group g computes
        constexpr int kPf = kSwPkPf;
        int4 tq[kPf + 1];
        uint4 rq0[kPf + 1], rq1[kPf + 1];
        auto load_group = [&](int g) {
            tq[g % (kPf + 1)] = *(const int4 *)(top + s0 + 4 * g);
            rq0[g % (kPf + 1)] = src[(2 * g) * 64];
            rq1[g % (kPf + 1)] = src[(2 * g + 1) * 64];
        };
#pragma unroll
        for (int g = 0; g < kPf; ++g) load_group(g);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            if (g + kPf < 16) load_group(g + kPf);
            const int4 tc = tq[g % (kPf + 1)];
            const uint4 r0 = rq0[g % (kPf + 1)], r1 = rq1[g % (kPf + 1)];
            const int tv[4] = {tc.x, tc.y, tc.z, tc.w};
            const uint32_t s0v[4] = {r0.x, r0.z, r1.x, r1.z}, s1v[4] = {r0.y, r0.w, r1.y, r1.w};
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                // wave_ror:1 (every lane has a source: no old value to keep)
                const uint32_t rot = (uint32_t)__builtin_amdgcn_mov_dpp((int)sw_as_u(lr1), 0x13C, 0xf, 0xf, false);
                const sw_h2 up = sw_as_h2(__builtin_amdgcn_perm(rot, (uint32_t)tv[jj], selU));
                const sw_h2 h0 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(lr0, up), upp + sw_as_h2(s0v[jj]));
                const sw_h2 h1 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(lr1, h0), lr0 + sw_as_h2(s1v[jj]));
                if (jj & 1) {
                    // two steps' bottom-row values (lane 63's high halves) as one
                    // word, shifted down a lane (wave_shl:1; lane 63 keeps the pair)
                    const uint32_t pair = __builtin_amdgcn_perm(sw_as_u(h1), sw_as_u(lr1), 0x07060302u);
                    acc = (uint32_t)__builtin_amdgcn_update_dpp((int)pair, (int)acc, 0x130, 0xf, 0xf, false);
                }
                upp = up;
                lr0 = h0;
                lr1 = h1;
            }
        }
        if (lane == 0) lds_flag_st(&misc[6], k + 1);  // the chunk's ring slot is free
        // lanes 32 + p hold steps s0 + 2p (low half) and s0 + 2p + 1 (high)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int x = s0 + 2 * (lane - 32) + e - 127;  // the bottom row's column
            if (lane >= 32 && x >= 0 && x < ncols) {
                const sw_h2 pv = sw_as_h2(acc);
                const int h = (int)(float)(e ? pv.y : pv.x) + base - Rb - (C0 + 1 + x);
                st_agent(&T.hout[x], sw_granule(h));
                if (x == ncols - 1) {
                    if (T.corner_out) st_agent(T.corner_out, sw_granule(h));
                    if (T.corner_out_lds) *T.corner_out_lds = h;
                }
            }
        }
    }
    tstamp(10);
    // --- the right column: every row's value at its last column
    const int Cr = C0 + ncols;
    int rv[4];
    rv[0] = (int)(float)lr0.x + base - rowq[0] - Cr;
    rv[1] = (int)(float)lr1.x + base - rowq[1] - Cr;
    rv[2] = (int)(float)lr0.y + base - rowq[2] - Cr;
    rv[3] = (int)(float)lr1.y + base - rowq[3] - Cr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = rowq[q] - R0 - 1;
        if (T.rightcol) st_agent(&T.rightcol[k], sw_granule(rv[q]));
        if (T.rightcol_lds) T.rightcol_lds[k] = rv[q];
    }
    tstamp(11);
    tstamp(9);
    return true;
}

// The score wave, after staging the right neighbour (tile t + 1): poll its
// top row (the up-right tile's bottom row) into LDS while this tile's sweep
// runs (misc + kSwPkMisc + 256, then misc[8] = t + 1), so a kept neighbour
// starts without a global load. Gives up once this tile is done (misc[4]):
// the next tile then loads the row itself.
__device__ __forceinline__ void sw_pk_prefetch_top(const SwCtx &c, uint32_t t, int *misc) {
    int *ntop = misc + kSwPkMisc + 256;
    const sw_gran *src = c.gbot + (size_t)(t + 1 - (uint32_t)c.ntw) * c.tw;
    const int xmax = c.tw - 1;
    for (uint32_t n = 0;; ++n) {
        // this tile done: the workgroup's barrier waits for this wave, so no
        // new round trip is started once the sweep has finished
        if (n > 0 && lds_flag_ld(&misc[4]) == (int)t + 1) return;
        sw_gran g[kSwPkMaxTw / 64];
        bool ready = true;
#pragma unroll
        for (int k = 0; k < kSwPkMaxTw / 64; ++k) {
            const int x = lane_id() + 64 * k;
            g[k] = k * 64 < c.tw ? ld_agent(&src[x < c.tw ? x : xmax]) : (1ull << 32);
        }
#pragma unroll
        for (int k = 0; k < kSwPkMaxTw / 64; ++k) ready = ready && (g[k] >> 32) == 1ull;
        if (__ballot(!ready) == 0) {
#pragma unroll
            for (int k = 0; k < kSwPkMaxTw / 64; ++k) {
                const int x = lane_id() + 64 * k;
                if (x < c.tw) ntop[x] = (int)(uint32_t)g[k];
            }
            if (lane_id() == 0) lds_flag_st(&misc[8], (int)t + 1);
            return;
        }
        if (lds_flag_ld(&misc[4]) == (int)t + 1) return;
        __builtin_amdgcn_s_sleep(2);  // (8: 6.489 vs 6.473 ms, profiles/r06/ab_swpf.log)
    }
}

// The promise DAG with the packed body: workgroups of three waves, wave 0
// the sweep (and the tickets), wave 1 the scores, wave 2 run_dag_group's
// helper (waiter prefetch, datums: its global round trips stay off the
// score wave's start).
struct SwDagPkKind {
    using Ctx = SwCtx;
    static constexpr bool kSc1Payload = true;  // tile inputs/outputs move by ld_agent / st_agent
    static constexpr bool kTagged = true;      // ... as tagged granules: puts without a drain
    static constexpr bool kReserve = true;     // ready slots taken beside the counter decrements
    __device__ static int *misc_of(const SwCtx &c) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        return sw_lds + sw_pk_lds_words(c.tw) - kSwPkMisc - 256 - kSwPkMaxTw;
    }
    // misc: [0] the workgroup's last tile, [1..2] kept corners by parity,
    // [3] the corner datum, [4] the finished tile + 1 (wave 1 waits on it),
    // [5] / [6] score chunks written / read, [7] the tile whose selectors and
    // score rows are staged (misc + 16: the rows, [4][64]), [8] the tile whose
    // top row (H) is in LDS (misc + 16 + 256: the right neighbour's top row,
    // taken while this tile runs once every granule's tag is set)
    __device__ static bool run_group(const SwCtx &c, uint32_t t, const uint32_t *, int wave) {
        extern __shared__ __attribute__((aligned(16))) int sw_lds[];
        int *misc = misc_of(c);
        uint4 *ring = (uint4 *)sw_lds;
        int *top = sw_lds + kSwPkRingU4 * 4, *sel = top + sw_pk_topw(c.tw), *right_keep = sel + 4 * sw_pk_selw(c.tw);
        const int i = (int)(t / (uint32_t)c.ntw), j = (int)(t % (uint32_t)c.ntw);
        if (wave == 2) {
            // run_dag_group's helper (the workgroup's last wave): returns once
            // the tile's LDS outputs (the corner datum) exist
            return sw_pk_wait<true>(c, &misc[4], (int)t + 1);
        }
        if (wave == 1) {
            int *tbl = misc + kSwPkMisc;
            // staged ahead (misc[7] == t), or now: the first chunk's scores as
            // soon as its columns are staged, the rest after
            bool ok = true;
            if (misc[7] != (int)t) {
                auto first = [&]() { return sw_pk_scores(c, c.tw, ring, sel, tbl, misc, 0, 1); };
                ok = c.tw <= 256 ? sw_pk_stage<4>(c, i * kSwPkTh, j * c.tw, c.tw, sel, tbl, first)
                                 : sw_pk_stage<8>(c, i * kSwPkTh, j * c.tw, c.tw, sel, tbl, first);
                if (ok) ok = sw_pk_scores(c, c.tw, ring, sel, tbl, misc, 1);
            } else {
                ok = sw_pk_scores(c, c.tw, ring, sel, tbl, misc);
            }
            if (ok) {
                // while the sweep runs: stage the right neighbour
                const bool next = j + 1 < c.ntw;
                auto none = []() { return true; };
                if (next) {
                    if (c.tw <= 256) sw_pk_stage<4>(c, i * kSwPkTh, (j + 1) * c.tw, c.tw, sel, tbl, none);
                    else sw_pk_stage<8>(c, i * kSwPkTh, (j + 1) * c.tw, c.tw, sel, tbl, none);
                }
                if (lane_id() == 0) misc[7] = next ? (int)t + 1 : -1;
                // ... and its top row (the up-right tile's bottom row), polled
                // while this tile's sweep runs: kept, the right neighbour then
                // starts without a global load
                // (after the sweep wave has read this tile's own LDS top row: it
                // consumes chunk 0 only after that)
                if (next && i > 0 && sw_pk_wait(c, &misc[6], 1)) sw_pk_prefetch_top(c, t, misc);
            }
            // one exit, drained: a load this path might leave in flight
            // (the staging's, on a failed wait) would otherwise put a
            // vmcnt(0) where the waves' paths join behind the body, and the
            // sweep wave would wait there for its own output stores
            vm_drain();
            return ok;
        }
        const bool from_lds = j > 0 && misc[0] == (int)t - 1;
        SwPkTile T;
        T.R0 = i * kSwPkTh;
        T.C0 = j * c.tw;
        T.ncols = c.tw;
        T.corner_src = (T.R0 == 0 || j == 0 || from_lds) ? nullptr : &c.gcorner[t - (uint32_t)c.ntw - 1];
        T.corner_val = T.R0 == 0 ? -T.C0 : (j == 0 ? -T.R0 : (from_lds ? misc[1 + ((t - 1) & 1)] : 0));
        T.hin = i > 0 ? c.gbot + (size_t)(t - (uint32_t)c.ntw) * c.tw : nullptr;
        T.top_lds = (i > 0 && from_lds && misc[8] == (int)t) ? misc + kSwPkMisc + 256 : nullptr;
        if (T.top_lds) T.hin = nullptr;
        T.left_lds = j > 0 && from_lds ? right_keep + ((t - 1) & 1) * kSwPkTh : nullptr;
        T.leftcol = j > 0 && !from_lds ? c.gright + (size_t)(t - 1) * kSwPkTh : nullptr;
        T.hout = c.gbot + (size_t)t * c.tw;
        T.rightcol = c.gright + (size_t)t * kSwPkTh;
        T.rightcol_lds = right_keep + (t & 1) * kSwPkTh;
        T.corner_out = c.gcorner + t;
        T.corner_out_lds = &misc[3];
        T.corner_lds = &misc[1 + (t & 1)];
        T.trec = HX_DAG_TRACE && c.dtrace ? c.dtrace + (size_t)t * kDagTraceWords : nullptr;
        const bool ok = c.tw <= 256 ? sw_pk_tile<4>(c, T, top, ring, misc) : sw_pk_tile<8>(c, T, top, ring, misc);
        if (ok && lane_id() == 0) lds_flag_st(&misc[4], (int)t + 1);
        return ok;
    }
    // between tiles: this tile recorded as the workgroup's last, the score
    // ring's counters back to 0
    __device__ static void after_body(const SwCtx &c, uint32_t t) {
        if (threadIdx.x == 0) {
            int *misc = misc_of(c);
            misc[0] = (int)t;
            misc[5] = 0;
            misc[6] = 0;
        }
    }
    static constexpr int kPutN = 3;
    __device__ static void promises(const SwCtx &, uint32_t t, uint32_t (&p)[3]) {
        p[0] = 3u * t + 0u;
        p[1] = 3u * t + 1u;
        p[2] = 3u * t + 2u;
    }
    __device__ static void datums(const SwCtx &c, uint32_t, unsigned long long (&d)[3]) {
        d[0] = 0ull;
        d[1] = 0ull;
        d[2] = (unsigned long long)(uint32_t)misc_of(c)[3];  // c.corner[t] (:224-226)
    }
};

__global__ __launch_bounds__(192) void k_sw_dag_pk(SwCtx c, DagView v) {
    int *misc = SwDagPkKind::misc_of(c);
    if (threadIdx.x == 0) {
        misc[0] = -2;  // no tile yet (run_dag_group's first barrier orders these)
        misc[4] = 0;
        misc[5] = 0;
        misc[6] = 0;
        misc[7] = -1;  // no tile's scores staged
        misc[8] = -1;  // no tile's top row in LDS
    }
    run_dag_group<SwDagPkKind>(c, v, nullptr);
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
    // schedule: "rows" (default) = owner-computes tile rows with granule
    // hand-offs; "queue" = the generic DAG: dependency counters + ready list
    const char *sched = getenv("HCLIB_HIP_SW_SCHED");
    // the row schedule keeps two tile columns in LDS: wide tiles fall back
    const size_t rows_lds = 2 * (size_t)(((tw + 1 + 3) & ~3) * 4) + 68 * 4 + 2 * (size_t)((tw + 3) & ~3) + 16 +
                            2 * (size_t)(((th + 3) & ~3) * 4);
    const bool dag = sched && !strcmp(sched, "dag");
    const bool rows = !(sched && (!strcmp(sched, "queue") || dag)) && rows_lds <= 64 * 1024;
    // multi-wave tile rows (th / 64 waves per workgroup) unless "rows1" asks
    // for the one-wave-per-tile-row kernel
    // multi-wave band form (sw_pick_form): the DAG's tile tasks default to two
    // rows per lane (two waves per 256-row tile: one hand-off lag instead of
    // three), the row schedule to four (one band per 256-row tile row: the
    // per-row wavefront lag is paid once per 256 rows). SW-64K measured
    // (profiles/r02/sw_forms.log): rows 12: 4.4 ms, 212: 3.55, 412: 3.50;
    // dag 12: 11.2, 212: 9.4, 412: 9.6. Round 3, same box
    // (profiles/r03/sw_forms_k64.log): hand-offs every 64 steps for the DAG's
    // tiles, 212: 8.35 -> 214: 8.12-8.14 ms; rows 414 3.56 vs 412 3.49-3.51
    const int form = sw_pick_form(th, dag ? 214 : 412), bh = sw_form_bh(form);
    const bool band_shape = sw_band_ok(th, bh) && tw <= 65536;
    const bool band = rows && band_shape && !(sched && !strcmp(sched, "rows1"));
    // the promise DAG's 256-row tiles at most 512 wide: the packed-half body,
    // tagged outputs (HCLIB_HIP_SW_PK=0: the band forms)
    // (a two-sweep-wave body was exact but slower, 7.95 vs 6.56 ms, and was
    // removed in round 5: DESIGN.md Appendix A)
    const bool pk = dag && th == kSwPkTh && tw <= kSwPkMaxTw && env_int("HCLIB_HIP_SW_PK", 1) != 0;
    const size_t nt = ntw * nth;
    const size_t b_s1 = ntw * tw, b_s2 = nth * th;
    const size_t b_bot = (rows || pk) ? 0 : nt * tw * 4, b_right = (rows || pk) ? 0 : nt * th * 4, b_c = nt * 4,
                 b_dep = nt * 4, b_ready = nt * 4, b_gbot = (rows || pk) ? nt * tw * 8 : 0,
                 b_gright = pk ? nt * th * 8 : 0, b_gc = pk ? nt * 8 : 0;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t total = al(b_s1) + al(b_s2) + al(b_bot) + al(b_right) + al(b_c) + al(b_dep) +
                         al(b_ready) + al(b_gbot) + al(b_gright) + al(b_gc) + 1024;
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
    c.gbot = (unsigned long long *)(d + off); off += al(b_gbot);
    c.gright = (unsigned long long *)(d + off); off += al(b_gright);
    c.gcorner = (unsigned long long *)(d + off); off += al(b_gc);
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
    c.j0 = 0;
    c.j1 = (int)ntw;
    c.i0 = 0;
    c.i1 = (int)nth;
    c.left_in = nullptr;
    c.right_out = nullptr;
    c.progressive = env_int("HCLIB_HIP_SW_PROGRESSIVE", 1);
    c.dtrace = nullptr;
    c.form = form;
    c.bh = bh;
    int rc = HCLIB_HIP_OK;
    auto fail = [&](int r) { (void)hipFree(d); return r; };
    if ((rc = hip_check(hipMemcpyAsync((void *)c.s1, s1, b_s1, hipMemcpyHostToDevice, m.stream), "copy s1"))) return fail(rc);
    if ((rc = hip_check(hipMemcpyAsync((void *)c.s2, s2, b_s2, hipMemcpyHostToDevice, m.stream), "copy s2"))) return fail(rc);
    if ((rc = hip_check(hipMemsetAsync(misc, 0, 1024, m.stream), "memset"))) return fail(rc);
    {
        uint32_t one = 1;  // tile 0 already sits at ready[0]
        if ((rc = hip_check(hipMemcpyAsync(c.ready_tail, &one, 4, hipMemcpyHostToDevice, m.stream), "tail"))) return fail(rc);
    }
    if (rows || pk) {
        // every granule's tag starts at 0 (not yet put)
        if ((rc = hip_check(hipMemsetAsync(c.gbot, 0, b_gbot, m.stream), "memset granules"))) return fail(rc);
        if (pk && (rc = hip_check(hipMemsetAsync(c.gright, 0, al(b_gright) + b_gc, m.stream),
                                  "memset granules")))
            return fail(rc);
    }
    if (!rows) {
        hipLaunchKernelGGL(k_sw_init, dim3(1024), dim3(256), 0, m.stream, c.deps, c.ready, c.ntw, c.nth);
    }
    const size_t lds = band ? sw_band_lds_bytes(th / bh)
                            : 2 * (size_t)(((tw + 1 + 3) & ~3) * 4) + 68 * 4 + 2 * (size_t)((tw + 3) & ~3) + 16 +
                                  (rows ? 2 * (size_t)(((th + 3) & ~3) * 4) : 0);
    if (lds > 160 * 1024) return fail((set_error("hclib_hip_sw: tile too large for LDS"), HCLIB_HIP_EINVAL));
    int per_cu = (int)((160 * 1024) / lds);
    // rows: one wave per CU owns tile rows (all resident, so every wait ends)
    int wpc = env_int("HCLIB_HIP_SW_WAVES_PER_CU", rows ? 1 : 2);
    if (wpc > per_cu) wpc = per_cu;
    // the generic promise DAG launches at most 8 waves per CU
    // (hclib_hip_dag_begin); clamp here rather than fail its argument check
    if (dag && wpc > 8) wpc = 8;
    if (wpc < 1) wpc = 1;
    int grid = m.num_cus * wpc;
    if (rows && grid > (int)nth) grid = (int)nth;
    const void *kern = rows ? (c.progressive ? (const void *)k_sw_rows<true> : (const void *)k_sw_rows<false>)
                            : (dag ? (const void *)k_sw_dag : (const void *)k_sw);
    if (lds > 64 * 1024) (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hclib_hip_dag_stats_t dst{};
    if (dag) {
        // the tile program's futures as a CSR over 3 promises per tile
        std::vector<uint32_t> off(nt + 1, 0), ids;
        ids.reserve(3 * nt);
        for (size_t t = 0; t < nt; ++t) {
            const size_t i = t / ntw, j = t % ntw;
            if (j > 0) ids.push_back((uint32_t)(3 * (t - 1) + 0));
            if (i > 0) ids.push_back((uint32_t)(3 * (t - ntw) + 1));
            if (i > 0 && j > 0) ids.push_back((uint32_t)(3 * (t - ntw - 1) + 2));
            off[t + 1] = (uint32_t)ids.size();
        }
        // tile tasks on workgroups of th / 64 + 2 waves where the band
        // kernel applies (HCLIB_HIP_SW_DAG_WAVE=1: one wave per tile)
        const bool wg = band_shape && env_int("HCLIB_HIP_SW_DAG_WAVE", 0) == 0;
        hclib_hip_dag_launch_t L;
        if ((rc = hclib_hip_dag_begin((uint32_t)nt, (uint32_t)(3 * nt), 0, nullptr, off.data(), ids.data(), nullptr,
                                      nullptr, pk ? env_int("HCLIB_HIP_SW_PK_WGS_PER_CU", 1)
                                                  : (wg ? env_int("HCLIB_HIP_SW_DAG_WGS_PER_CU", 1) : wpc),
                                      c.spin_ms, &L)))
            return fail(rc);
        if (pk) {
            const size_t plds = sw_pk_lds_bytes(tw);
            c.dtrace = ((const DagView *)L.view)->trace;
            if (plds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k_sw_dag_pk,
                                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds);
            hipLaunchKernelGGL(k_sw_dag_pk, dim3(L.grid), dim3(192), plds, m.stream, c, *(const DagView *)L.view);
        } else if (wg) {
            const size_t blds = sw_band_lds_bytes(th / bh) + (4 + 2 * (size_t)th) * 4;  // + kept right columns
            if (blds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k_sw_dag_wg,
                                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)blds);
            c.dtrace = ((const DagView *)L.view)->trace;
            hipLaunchKernelGGL(k_sw_dag_wg, dim3(L.grid), dim3(64 * (th / bh) + 128), blds, m.stream, c,
                               *(const DagView *)L.view);
        } else {
            hipLaunchKernelGGL(k_sw_dag, dim3(L.grid), dim3(64), lds, m.stream, c, *(const DagView *)L.view);
        }
        // (the packed body's tagged puts are checked for double puts here)
        std::vector<uint8_t> sat(pk ? 3 * nt : 0);
        if ((rc = hclib_hip_dag_end("hclib_hip_sw (dag)", nullptr, pk ? sat.data() : nullptr, &dst))) return fail(rc);
    } else {
        if ((rc = hip_check(hipEventRecord(m.ev0, m.stream), "event"))) return fail(rc);
        if (band) {
            const int k = sw_band_rows_per_wg(th, bh), nblk = ((int)nth + k - 1) / k;
            const int g = nblk < m.num_cus ? nblk : m.num_cus;
            const size_t blds = sw_band_lds_bytes(k * (th / bh));
            if (blds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k_sw_band_rows,
                                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)blds);
            hipLaunchKernelGGL(k_sw_band_rows, dim3(g), dim3(64 * k * (th / bh) + 128), blds, m.stream, c);
        } else if (rows && c.progressive) hipLaunchKernelGGL(k_sw_rows<true>, dim3(grid), dim3(64), lds, m.stream, c);
        else if (rows) hipLaunchKernelGGL(k_sw_rows<false>, dim3(grid), dim3(64), lds, m.stream, c);
        else hipLaunchKernelGGL(k_sw, dim3(grid), dim3(64), lds, m.stream, c);
        if ((rc = hip_check(hipGetLastError(), "k_sw launch"))) return fail(rc);
        if ((rc = hip_check(hipEventRecord(m.ev1, m.stream), "event"))) return fail(rc);
    }
    uint32_t herr = 0;
    unsigned long long st[10] = {0};
    int corner = 0;
    if ((rc = hip_check(hipStreamSynchronize(m.stream), "k_sw"))) return fail(rc);
    (void)hipMemcpy(&herr, c.err, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(st, c.stats, sizeof(st), hipMemcpyDeviceToHost);
    if (HX_STAMPS && (band || (dag && band_shape))) {
        unsigned long long t[29] = {0};
        (void)hipMemcpy(t, c.stats, sizeof(t), hipMemcpyDeviceToHost);
        const double per = dag ? (double)nt : (double)nth;  // per tile (DAG) or per tile row
        for (int w = 0; w < 3 && w < th / bh; ++w)
            fprintf(stderr, "sw band wave %d phases (cycles per %s): compute %.0f wait-top %.0f chunk-top %.0f"
                            " publish %.0f prologue %.0f\n",
                    w, dag ? "tile" : "row", (double)t[4 + 6 * w] / per, (double)t[5 + 6 * w] / per,
                    (double)t[6 + 6 * w] / per, (double)t[7 + 6 * w] / per, (double)t[8 + 6 * w] / per);
        if (!dag)
            fprintf(stderr, "sw band: row start spacing %.3f us, last row %.3f us\n",
                    nth > 1 ? (double)(t[26] - t[27]) * 0.01 / (double)(nth - 1) : 0.0, (double)(t[28] - t[26]) * 0.01);
    } else if (HX_STAMPS && st[0])
        fprintf(stderr, "sw phases (cycles/tile): inputs %.0f band-setup %.0f ramp-in %.0f steady %.0f ramp-out %.0f outputs %.0f\n",
                (double)st[4] / st[0], (double)st[5] / st[0], (double)st[6] / st[0], (double)st[7] / st[0],
                (double)st[8] / st[0], (double)st[9] / st[0]);
    if (rows) {
        unsigned long long g = 0;  // bottom_row[tw-1] of the last tile (its granule)
        (void)hipMemcpy(&g, c.gbot + (nt * tw - 1), 8, hipMemcpyDeviceToHost);
        corner = (int)(uint32_t)g;
        // the edges the row schedule resolved: each tile's up, left and
        // diagonal futures (the same 3-per-interior-tile count as the queue)
        st[1] = 3ull * (ntw - 1) * (nth - 1) + (ntw - 1) + (nth - 1);
    } else if (pk) {
        unsigned long long g = 0;  // the last tile's corner granule
        (void)hipMemcpy(&g, c.gcorner + (nt - 1), 8, hipMemcpyDeviceToHost);
        corner = (int)(uint32_t)g;
    } else {
        (void)hipMemcpy(&corner, c.corner + (nt - 1), 4, hipMemcpyDeviceToHost);
    }
    if (dag) {  // the DAG's own counters: tasks run, and every future resolved
        st[0] = dst.tasks;
        st[1] = 3ull * (ntw - 1) * (nth - 1) + (ntw - 1) + (nth - 1);
    }
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

// ------------------------------------------------- column-band sessions
// Multi-GPU SW: each rank owns a band of tile columns
// and runs the row schedule over it in blocks of tile rows; between blocks
// the host moves the band's right column to the next rank (RCCL send/recv on
// the same stream, hclib_amd/dist.py). The band keeps its granules, s1 and s2
// on the device across blocks, so a block only needs its left column.
struct hclib_hip_sw_band {
    SwCtx c;
    char *mem;
    size_t lds;
    int grid_cap;
};

extern "C" int hclib_hip_sw_band_begin(const int8_t *s1, size_t n1, const int8_t *s2, size_t n2, int tw, int th,
                                       int j0, int j1, hclib_hip_sw_band_t **out) {
    if (!out || !s1 || !s2 || tw < 1 || th < 1 || tw > 16384) {
        set_error("hclib_hip_sw_band_begin: invalid arguments");
        return HCLIB_HIP_EINVAL;
    }
    *out = nullptr;
    const size_t ntw = n1 / (size_t)tw, nth = n2 / (size_t)th;
    if (ntw == 0 || nth == 0 || ntw * nth > 0x7fffffffull || j0 < 0 || j1 <= j0 || (size_t)j1 > ntw) {
        set_error("hclib_hip_sw_band_begin: empty grid or band [%d, %d) outside 0..%zu", j0, j1, ntw);
        return HCLIB_HIP_EINVAL;
    }
    for (size_t k = 0; k < ntw * (size_t)tw; ++k)
        if (s1[k] < 1 || s1[k] > 4) { set_error("hclib_hip_sw_band_begin: s1 must be coded 1..4"); return HCLIB_HIP_EINVAL; }
    for (size_t k = 0; k < nth * (size_t)th; ++k)
        if (s2[k] < 1 || s2[k] > 4) { set_error("hclib_hip_sw_band_begin: s2 must be coded 1..4"); return HCLIB_HIP_EINVAL; }
    const size_t lds = 2 * (size_t)(((tw + 1 + 3) & ~3) * 4) + 68 * 4 + 2 * (size_t)((tw + 3) & ~3) + 16 +
                       2 * (size_t)(((th + 3) & ~3) * 4);
    if (lds > 64 * 1024) {
        set_error("hclib_hip_sw_band_begin: tile too large for the row schedule");
        return HCLIB_HIP_EINVAL;
    }
    HX_TRY(ensure_device());
    Module &m = mod();
    const size_t nt = ntw * nth, b_s1 = ntw * tw, b_s2 = nth * th, b_gbot = nt * tw * 8;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t total = al(b_s1) + al(b_s2) + al(b_gbot) + 1024;
    hclib_hip_sw_band *h = new hclib_hip_sw_band();
    if (hipMalloc((void **)&h->mem, total) != hipSuccess) {
        delete h;
        set_error("hclib_hip_sw_band_begin: hipMalloc(%zu) failed", total);
        return HCLIB_HIP_ENOMEM;
    }
    SwCtx &c = h->c;
    memset(&c, 0, sizeof(c));
    size_t off = 0;
    c.s1 = (const int8_t *)(h->mem + off); off += al(b_s1);
    c.s2 = (const int8_t *)(h->mem + off); off += al(b_s2);
    c.gbot = (unsigned long long *)(h->mem + off); off += al(b_gbot);
    uint32_t *misc = (uint32_t *)(h->mem + off);
    c.err = misc + 128;
    c.stats = (unsigned long long *)(misc + 192);
    c.tw = tw;
    c.th = th;
    c.ntw = (int)ntw;
    c.nth = (int)nth;
    c.j0 = j0;
    c.j1 = j1;
    c.progressive = env_int("HCLIB_HIP_SW_PROGRESSIVE", 1);
    c.dtrace = nullptr;
    c.form = sw_pick_form(th, 412);
    c.bh = sw_form_bh(c.form);
    c.spin_ms = (uint32_t)env_int("HCLIB_HIP_SPIN_LIMIT_MS", 20000);
    h->lds = lds;
    h->grid_cap = m.num_cus;
    int rc;
    if ((rc = hip_check(hipMemcpy((void *)c.s1, s1, b_s1, hipMemcpyHostToDevice), "copy s1")) ||
        (rc = hip_check(hipMemcpy((void *)c.s2, s2, b_s2, hipMemcpyHostToDevice), "copy s2")) ||
        (rc = hip_check(hipMemset(misc, 0, 1024), "memset")) ||
        (rc = hip_check(hipMemset(c.gbot, 0, b_gbot), "memset granules"))) {
        (void)hipFree(h->mem);
        delete h;
        return rc;
    }
    *out = h;
    return HCLIB_HIP_OK;
}

extern "C" int hclib_hip_sw_band_rows(hclib_hip_sw_band_t *h, int i0, int i1, const int *left_in, int *right_out,
                                      void *stream) {
    if (!h || i0 < 0 || i1 <= i0 || i1 > h->c.nth || (h->c.j0 > 0 && !left_in)) {
        set_error("hclib_hip_sw_band_rows: invalid arguments (rows [%d, %d), left column %s)", i0, i1,
                  left_in ? "given" : "missing");
        return HCLIB_HIP_EINVAL;
    }
    SwCtx c = h->c;
    c.i0 = i0;
    c.i1 = i1;
    c.left_in = left_in;
    c.right_out = right_out;
    // one wave owns each tile row; every wave of the block is resident, so
    // each granule wait ends (rows above i0 finished in an earlier launch)
    int grid = i1 - i0;
    if (grid > h->grid_cap) grid = h->grid_cap;
    const char *sched = getenv("HCLIB_HIP_SW_SCHED");
    if (sw_band_ok(c.th, c.bh) && !(sched && !strcmp(sched, "rows1"))) {
        const int k = sw_band_rows_per_wg(c.th, c.bh), nblk = (i1 - i0 + k - 1) / k;
        const int g = nblk < h->grid_cap ? nblk : h->grid_cap;
        const size_t blds = sw_band_lds_bytes(k * (c.th / c.bh));
        if (blds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k_sw_band_rows,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)blds);
        hipLaunchKernelGGL(k_sw_band_rows, dim3(g), dim3(64 * k * (c.th / c.bh) + 128), blds, (hipStream_t)stream,
                           c);
    }
    else if (c.progressive) hipLaunchKernelGGL(k_sw_rows<true>, dim3(grid), dim3(64), h->lds, (hipStream_t)stream, c);
    else hipLaunchKernelGGL(k_sw_rows<false>, dim3(grid), dim3(64), h->lds, (hipStream_t)stream, c);
    return hip_check(hipGetLastError(), "k_sw_rows (band) launch");
}

extern "C" int hclib_hip_sw_band_end(hclib_hip_sw_band_t *h, void *stream, int *corner, uint64_t *tiles) {
    if (!h) {
        set_error("hclib_hip_sw_band_end: null band");
        return HCLIB_HIP_EINVAL;
    }
    int rc = hip_check(hipStreamSynchronize((hipStream_t)stream), "k_sw_rows (band)");
    uint32_t herr = 0;
    unsigned long long st[4] = {0}, g = 0;
    const SwCtx &c = h->c;
    if (!rc) {
        (void)hipMemcpy(&herr, c.err, 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(st, c.stats, sizeof(st), hipMemcpyDeviceToHost);
        // bottom-right cell of the band's last tile (the score for the last band)
        const size_t t = (size_t)(c.nth - 1) * c.ntw + (c.j1 - 1);
        (void)hipMemcpy(&g, c.gbot + t * c.tw + (c.tw - 1), 8, hipMemcpyDeviceToHost);
    }
    (void)hipFree(h->mem);
    delete h;
    if (rc) return rc;
    if (herr) {
        set_error("hclib_hip_sw_band_end: device error %u", herr);
        return HCLIB_HIP_EDEVICE;
    }
    if ((g >> 32) != 1ull) {
        set_error("hclib_hip_sw_band_end: the band's last tile was never computed (rows missing)");
        return HCLIB_HIP_EDEVICE;
    }
    if (corner) *corner = (int)(uint32_t)g;
    if (tiles) *tiles = st[0];
    return HCLIB_HIP_OK;
}
