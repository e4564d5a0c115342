// LDS write-pattern microbenchmark: cost of the push writes of one batch,
// measured as cycles from the first ds_write to a dependent ds_read's data.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void k_lds(unsigned long long *cyc, uint32_t *out, int iters, int mode, int active_stride,
                      int item_stride, int nwrites) {
    __shared__ uint4 ring[2048];
    const int lane = threadIdx.x;
    for (int i = lane; i < 2048; i += 64) ring[i] = make_uint4(i, 0, 0, 0);
    __syncthreads();
    const bool act = (lane % active_stride) == 0;
    const int pos = (lane / active_stride) * item_stride;  // item index of this lane's group
    uint32_t acc = 0;
    uint4 v = make_uint4(lane, 1, 2, 3);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (act) {
            for (int j = 0; j < nwrites; ++j) {
                const int slot = ((pos + j) * 2) & 2047;  // 32-B items = 2 uint4
                if (mode == 0) {
                    ring[slot] = v;
                    ring[slot + 1] = v;
                } else if (mode == 1) {
                    reinterpret_cast<uint2 *>(ring)[slot] = make_uint2(v.x, v.y);
                }
                v.x += 1;
            }
        }
        // dependent read of the slot just written by another lane (as the next batch does)
        const uint4 r = ring[((lane * 2) + it) & 2047];
        acc += r.x;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        v.y = acc;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    unsigned long long *cyc;
    uint32_t *out;
    hipMalloc(&cyc, 8);
    hipMalloc(&out, 256);
    struct Cfg { const char *name; int mode, astride, istride, nw; } cfgs[] = {
        {"read only (0 writes)", 0, 1, 1, 0},
        {"b128x2, 64 lanes, item stride 1", 0, 1, 1, 1},
        {"b128x2, 8 lanes (every 8th), 8 items each, stride 8 (T3 push)", 0, 8, 8, 8},
        {"b128x2, 13 lanes (every 5th), 5 items each, stride 5 (T3L push)", 0, 5, 5, 5},
        {"b128x2, 64 lanes, 1 item, stride 8", 0, 1, 8, 1},
        {"b128x2, 8 lanes, 1 item each, stride 8", 0, 8, 8, 1},
        {"b64, 8 lanes, 8 items each (descriptor writes)", 1, 8, 8, 8},
        {"b64, 13 lanes, 5 items each", 1, 5, 5, 5},
    };
    for (auto &c : cfgs) {
        const int iters = 2000;
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, cyc, out, iters, c.mode, c.astride, c.istride, c.nw);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, cyc, out, iters, c.mode, c.astride, c.istride, c.nw);
        unsigned long long h;
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-70s cycles/iter=%.1f\n", c.name, (double)h / iters);
    }
    return 0;
}
