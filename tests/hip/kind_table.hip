// The C drop-in's kind table (include/hclib.h): device code of the program's
// own, linked into a C program (tests/c/kind_table_main.c) that uses only
// include/hclib.h. This translation unit defines
//   * a device task kind for the program's host function `fib` — the
//     reference's nested-finish fib (test/fib/fib.c:57-71) as a device
//     program: every call a task, every FINISH a scope (hx_finish.h), the
//     sum the continuation run by the last child out;
//   * a device loop body for the program's host function `scale_body`:
//     y[i] = 3 * x[i] + i over the forasync iteration set;
// and registers both before main (HCLIB_HIP_DEVICE_ASYNC / _FORASYNC).
#include "hclib_hip_cpp.h"

extern "C" {
void fib(void *raw_args);                        // defined by the C program
void scale_body(void *raw_args, int i);          // ditto
}

namespace {

struct FibCtx {
    int n;
    hx::FinishArena fin;
};

struct FibKind {
    static constexpr int kTmplWords = 2;  // {n + 1 of the parent call, parent scope}
    static constexpr int kWords = 4;
    static constexpr bool kPure = false;
    static constexpr bool kBoundedChildren = true;
    using Ctx = FibCtx;
    struct Acc {
        __device__ void flush(hx::SchedGlobals *) {}
    };
    __device__ static int roots(const Ctx &c, Acc &, uint32_t *tmpl) {
        tmpl[0] = (uint32_t)c.n + 1;
        tmpl[1] = hx::kScopeRoot;
        return 1;
    }
    __device__ static int process(const Ctx &c, Acc &, const uint32_t *t, uint32_t k, uint32_t *child, uint32_t *err,
                                  bool) {
        const int n = (int)t[0] - 1 - (int)k;
        const uint32_t scope = hx::finish_open(c.fin, n >= 2, t[1], 2, 0, err);
        if (n < 2) {
            hx::finish_check_out(c.fin, t[1], (unsigned long long)n, hx::PassSum());
            return 0;
        }
        child[0] = (uint32_t)n;
        child[1] = scope;
        return scope == hx::kScopeRoot ? 0 : 2;
    }
};

struct FibArgs {  // test/fib/fib.c:50-53
    int n;
    long res;
};

int fib_launch(void *raw) {
    FibArgs *a = (FibArgs *)raw;
    if (a->n < 0 || a->n > 40) return HCLIB_HIP_EINVAL;
    // fib(n) opens fib(n + 1) - 1 scopes
    unsigned long long f0 = 0, f1 = 1;
    for (int i = 0; i < a->n + 1; ++i) {
        const unsigned long long t = f0 + f1;
        f0 = f1;
        f1 = t;
    }
    hclib::hip::finish_arena fin((uint32_t)f0 + 1);
    if (!fin.ok()) return HCLIB_HIP_ENOMEM;
    const int rc = hclib::hip::run_tasks<FibKind>(FibCtx{a->n, fin.view()});
    if (rc) return rc;
    a->res = (long)fin.root_value();
    return HCLIB_HIP_OK;
}

struct ScaleArgs {  // the C program's struct
    int *y;
    const int *x;
};

struct ScaleBody {
    int *y;
    const int *x;
    __device__ void operator()(int i, int, int) const { y[i] = 3 * x[i] + i; }
};

int scale_launch(void *raw, int dim, hclib_loop_domain_t *domain, int mode, void *stream) {
    const ScaleArgs *a = (const ScaleArgs *)raw;
    return hclib::hip::forasync_device(ScaleBody{a->y, a->x}, dim, domain, mode, stream);
}

}  // namespace

HCLIB_HIP_DEVICE_ASYNC(fib, fib_launch);
HCLIB_HIP_DEVICE_FORASYNC(scale_body, scale_launch);
