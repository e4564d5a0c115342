/*
 * hclib_hip.h — the MI355X `modules/hip` C ABI.
 *
 * HClib's plug-in ABI lets a module add a locale type and run work there
 * (inc/hclib-module.h:62-106, src/hclib_module.c:49-160). The reference's
 * only device module, modules/cuda, runs kernels from CPU tasks and polls
 * for completion (modules/cuda/inc/hclib_cuda.h:21-74). This module instead
 * moves the scheduler itself onto the GPU: every entry point below replaces
 * a piece of the reference's CPU hot path with a hand-written gfx950 kernel.
 *
 *   entry point                      replaces (reference file:line)
 *   -------------------------------  -------------------------------------------
 *   hclib_hip_forasync1d/2d/3d       hclib_forasync + forasync{1,2,3}D_{flat,
 *                                    recursive,runner}  src/hclib.c:110-464
 *   hclib_hip_forasync_triad_f32     the forasync1D_runner loop of a triad body
 *                                    src/hclib.c:110-120 (BASELINE config 1)
 *   hclib_hip_uts_search             core_work_loop/find_and_run_task/deque_*
 *                                    src/hclib-runtime.c:646-729,
 *                                    src/hclib-deque.c:50-139, driving the UTS
 *                                    tasks of test/uts/UTS.cpp:154-232
 *   hclib_hip_fib                    spawn/finish counters of test/fib/fib.c:57-71
 *                                    (async/finish) and 113-141 (DDT), i.e.
 *                                    src/hclib-runtime.c:431-446, 572-617,
 *                                    1219-1277
 *   hclib_hip_sw                     promise put / waiter release of
 *                                    src/hclib-promise.c:132-245 driving the tile
 *                                    DAG of test/smithwaterman/smith_waterman.cpp
 *                                    :119-239
 *   hclib_hip_dag_*                  the same dependency-counter release for any
 *                                    async_await DAG built through hclib.h
 *
 * Conventions (mirroring the reference's error behaviour):
 * plain pointers and sizes only; functions return 0 on success and a
 * negative HCLIB_HIP_E* code on failure, with a message retrievable via
 * hclib_hip_last_error(). Device-side failures (queue overflow, bounded
 * spins that time out) set a device error word that the host checks after
 * every launch. Nothing here ever falls back to the CPU: without a usable
 * gfx950 device every compute entry point fails with HCLIB_HIP_ENODEV.
 */
#ifndef HCLIB_HIP_H_
#define HCLIB_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HCLIB_HIP_OK 0
#define HCLIB_HIP_ENODEV (-1)   /* no HIP device / not gfx950 */
#define HCLIB_HIP_EINVAL (-2)   /* bad arguments */
#define HCLIB_HIP_ENOMEM (-3)   /* device allocation failed */
#define HCLIB_HIP_EDEVICE (-4)  /* device-side error word set (see message) */
#define HCLIB_HIP_EHIP (-5)     /* a HIP runtime call failed */

/* ---------------------------------------------------------------- module */
/* hclib_hip_init: bind the calling process to HIP device `device` (the
 * module's post-init hook, inc/hclib-module.h:62-64). Idempotent. */
int hclib_hip_init(int device);
void hclib_hip_finalize(void);
const char *hclib_hip_last_error(void);
/* Number of CUs / XCDs of the bound device (0 if none). */
int hclib_hip_num_cus(void);
/* the bound device (-1 before hclib_hip_init) and the module's HIP stream
 * (NULL before): what the hip plug-in module's memory callbacks run on */
int hclib_hip_device(void);
void *hclib_hip_stream(void);
/* Module version string, also proves the library loads without a GPU. */
const char *hclib_hip_version(void);
/* Scheduler counters of the last megakernel launch (HCLIB_STATS analogue,
 * src/hclib-runtime.c:83-104): [0..1] kind totals, [7..8] diagnostic phase
 * cycles (HCLIB_HIP_STAMPS=1), [9] busy, [10] idle, [11] spill cycles,
 * [12] waves, [13] batches, [14] chunks pushed, [15] chunks stolen. */
void hclib_hip_last_sched_counters(uint64_t out[16]);

/* Per-wave records of the last megakernel launch (the per-worker lines of
 * HCLIB_STATS, src/hclib-runtime.c:1370-1410): each wave writes its own
 * record as it leaves. Summed over the waves, batches / chunks_pushed /
 * chunks_stolen equal hclib_hip_last_sched_counters [13] / [14] / [15].
 * Copies at most `max` records to out; returns the number of waves. */
typedef struct {
    uint64_t executed;      /* tasks run (one lane of a batch each) */
    uint64_t spawned;       /* children created */
    uint64_t batches;
    uint64_t chunks_pushed; /* chunks given to the HBM deques */
    uint64_t chunks_stolen; /* chunks taken from a deque other than the wave's home deque */
    uint64_t items_stolen;  /* tasks in those chunks */
    uint64_t xcd;           /* the XCD the wave ran on */
    uint64_t reserved;
    uint64_t stolen_from[8]; /* chunks taken from each XCD's deques */
} hclib_hip_wave_stats_t;
int hclib_hip_last_wave_stats(hclib_hip_wave_stats_t *out, int max);
/* The narrow-frontier carry loop of the last launch (hx_sched.h): [0]
 * batches run in it, [1] shader-clock cycles spent in it, [2] entries. */
void hclib_hip_last_narrow_counters(uint64_t out[4]);
/* Diagnostic (HX_PHASES builds, zeros otherwise): [0] main-loop single
 * batches of the last megakernel launch, [1..4] their s_memtime cycles from
 * loop top to pop issued, pop landed, body done, batch end. */
void hclib_hip_last_phase_counters(uint64_t out[8]);
/* Worker timelines of the last megakernel launch (diagnostic: a library
 * built with `--variant timeline` and HCLIB_HIP_TIMELINE=<events per
 * worker>; hx_sched.h Timeline). Copies at most `max_words` events (worker w's
 * at [w * events_per_worker ...], 0 = unused) and returns the worker count
 * (0 when no timeline was recorded). */
int hclib_hip_last_timeline(uint64_t *out, uint64_t max_words, uint32_t *events_per_worker);

/* L2 atomic-throughput calibration: the saturated rate (million atomic
 * ops per second, whole GPU) of one access shape the runtime's atomics use,
 * the "peak" fib/SW/scheduler atomic rates are priced against.
 *   0 HCLIB_HIP_ATOMIC_SCATTER_RET64: every lane a returning 64-bit add on
 *     its own random 16-B record (fib join check-out, SW dependency counters)
 *   1 HCLIB_HIP_ATOMIC_HOT_WORD: lane 0 of every wave on ONE shared word
 *     (deque tickets, the `outstanding` termination counter)
 *   2 HCLIB_HIP_ATOMIC_COALESCED32: 64 consecutive non-returning 32-bit adds
 *     per wave instruction (the L2 atomic units' streaming peak)
 * `iters` atomic ops per lane (mode 1: per wave). */
#define HCLIB_HIP_ATOMIC_SCATTER_RET64 0
#define HCLIB_HIP_ATOMIC_HOT_WORD 1
#define HCLIB_HIP_ATOMIC_COALESCED32 2
int hclib_hip_atomic_calibrate(int mode, int iters, double *mops_per_s, double *kernel_ms);
/* The chip's UTS SHA-1 issue ceiling: `chains` (1 or 2) independent rng_spawn
 * chains per lane (the instruction stream k_uts_search runs per node),
 * waves_per_cu waves on every CU, `iters` spawns per chain; SHA-1
 * compressions per second over the timed launch (the peak of the UTS
 * kernel's VALU roofline; bench.py `roofline_uts`). */
int hclib_hip_sha1_calibrate(int chains, int waves_per_cu, int iters, double *sha1_per_s, double *kernel_ms);

/* ----------------------------------------------- user device task kinds */
/* The persistent-megakernel scheduler for task kinds compiled in the
 * caller's own HIP translation unit (include/hclib_hip_cpp.h,
 * hclib::hip::run_tasks<Kind>): begin() carves and resets the chunk deques
 * for `entry_words` u32 per queued item, resets the scheduler globals and
 * records the start event on the module stream; the caller launches
 * `grid` workgroups of 64 threads on `stream`; end() records the stop
 * event, waits, and returns the counters (see hclib_hip_last_sched_counters)
 * and the device error, if any, as HCLIB_HIP_EDEVICE. */
typedef struct {
    void *hdr;         /* deque headers */
    uint32_t *seq;     /* per-slot sequence words */
    uint32_t *cnt;     /* per-slot item counts */
    uint32_t *data;    /* chunk payloads */
    uint32_t nq, cap, chunk;
    void *globals;     /* scheduler globals (device) */
    void *stream;      /* hipStream_t of the module */
    int grid;          /* workgroups (waves) to launch */
    int num_cus;
} hclib_hip_sched_launch_t;

int hclib_hip_sched_begin(uint32_t entry_words, uint32_t chunk, int waves_per_cu,
                          hclib_hip_sched_launch_t *out);
int hclib_hip_sched_end(const char *who, uint64_t counters[16], uint64_t maxes[4],
                        double *kernel_ms);

/* ------------------------------------------------------------ forasync */
/* hclib_loop_domain_t of inc/hclib-task.h:53-58 (int bounds, 16 bytes). */
typedef struct {
    int low;
    int high;
    int stride;
    int tile;
} hclib_hip_loop_domain_t;

#define HCLIB_HIP_FORASYNC_FLAT 0      /* FORASYNC_MODE_FLAT, inc/hclib.h:161 */
#define HCLIB_HIP_FORASYNC_RECURSIVE 1 /* FORASYNC_MODE_RECURSIVE, inc/hclib.h:159 */

/* Device loop bodies. A host function pointer cannot run on the GPU, so a
 * forasync at the GPU locale names one of these registered body kinds. */
#define HCLIB_HIP_BODY_TRIAD_F32 1 /* a[i] = b[i] + s*c[i] (1-D) */
#define HCLIB_HIP_BODY_IOTA_CHECK 2 /* assert(ran[i]==-1); ran[i]=i, as test/c/forasync1DCh.c:45-49 (1-D) */
#define HCLIB_HIP_BODY_VISIT_COUNT 3 /* counts[linear(i,j,k)] += 1 (1/2/3-D) */

typedef struct {
    float *a;
    const float *b;
    const float *c;
    float s;
} hclib_hip_triad_args_t;

typedef struct {
    int *ran;      /* device pointer, indexed by i */
    int *errors;   /* device pointer to one int: number of failed checks */
} hclib_hip_iota_args_t;

typedef struct {
    int *counts;   /* device pointer */
    int base[3];   /* index origin per dim */
    int extent[3]; /* counts has extent[0]*extent[1]*extent[2] ints, row-major */
} hclib_hip_visit_args_t;

/* hclib_forasync (src/hclib.c:452-464) for dim in 1..3 at the GPU locale.
 * `domain` has `dim` entries; tile == -1 is replaced by
 * ceil((high-low)/nworkers) with nworkers = the module's worker count (the
 * number of resident waves, hclib_hip_num_workers()) and written back, as
 * the reference does. The iteration set is exactly the reference's for the
 * given mode (including the FLAT 1-D quirk of src/hclib.c:322-337).
 * `args` points to the body's argument struct (host memory, copied by
 * value). `stream` is a hipStream_t (NULL = default). Asynchronous: the
 * call returns after enqueueing; synchronize on the stream. */
int hclib_hip_forasync(int body, const void *args, int dim, hclib_hip_loop_domain_t *domain,
                       int mode, void *stream);

/* Fast path of hclib_hip_forasync for the triad over [0, n): coalesced
 * grid-stride float4 tiles, no FMA contraction (bit-exact with the CPU). */
int hclib_hip_forasync_triad_f32(float *a, const float *b, const float *c, float s, int64_t n,
                                 void *stream);

/* Resident worker waves the forasync/megakernel launches use. */
int hclib_hip_num_workers(void);

/* The iteration set of hclib_hip_forasync, for device loop bodies compiled
 * in the caller's own HIP translation unit (hclib::hip::forasync_device in
 * include/hclib_hip_cpp.h): plan() applies the reference's tiling (tile ==
 * -1 written back as in hclib_hip_forasync; FLAT and RECURSIVE sets exactly
 * as src/hclib.c:110-464 enumerate them) and uploads one table of runs per
 * dimension in `stream` order; iteration t of the sweep (0 <= t < total,
 * innermost dimension fastest) maps to (i, j, k) through the runs. release()
 * frees the tables in stream order after the sweep. */
typedef struct {
    int first, count, stride, pad;  /* indices first + m * stride, m < count */
} hclib_hip_run_t;
typedef struct {
    const hclib_hip_run_t *runs[3];
    const int64_t *prefix[3];  /* prefix[d][r] = iterations of dimension d before run r */
    int nruns[3];
    int ndim;
    int64_t total;
    void *mem;
} hclib_hip_sweep_plan_t;
int hclib_hip_forasync_plan(int dim, hclib_hip_loop_domain_t *domain, int mode, void *stream,
                            hclib_hip_sweep_plan_t *plan);
int hclib_hip_forasync_plan_release(hclib_hip_sweep_plan_t *plan, void *stream);

/* ----------------------------------------------------------------- UTS */
/* Tree parameters: the UTS CLI flags of test/uts/uts.c:380-420 (same field
 * order as oracle/uts_oracle.h so both sides read the same struct). */
typedef struct {
    int type;         /* -t: 0 BIN, 1 GEO, 2 HYBRID, 3 BALANCED */
    int shape_fn;     /* -a: 0 LINEAR, 1 EXPDEC, 2 CYCLIC, 3 FIXED */
    int gen_mx;       /* -d */
    int root_id;      /* -r */
    int non_leaf_bf;  /* -m */
    int compute_gran; /* -g */
    double b_0;       /* -b */
    double non_leaf_prob; /* -q */
    double shift_depth;   /* -f */
} hclib_hip_uts_params_t;

typedef struct {
    uint64_t nodes;     /* tree size   (UTS.cpp:241, uts.c:462) */
    uint64_t leaves;    /* num leaves */
    uint64_t max_depth; /* tree depth */
    uint64_t chunks_pushed;  /* work chunks spilled to the HBM deques */
    uint64_t chunks_stolen;  /* chunks taken from another worker's deque */
    uint64_t batches;        /* wave batches executed */
    double kernel_ms;        /* device time of the search launch (HIP events) */
    double busy_frac;        /* share of wave time spent inside batches */
    double us_per_batch;     /* average wave time per batch (incl. spills) */
} hclib_hip_uts_result_t;

/* Search the whole tree on the bound GPU (persistent megakernel: per-wave
 * LDS stacks, per-XCD chunk deques in HBM, device-atomic stealing,
 * outstanding-work termination). Multi-GPU sharding: with nshards > 1 every
 * shard expands the levels above split_depth identically (counted by shard
 * 0 only); shard `shard` keeps the depth-split_depth nodes whose first state
 * word is congruent to shard (mod nshards) and searches their subtrees.
 * Per-shard results sum to the whole tree (max for depth); with a global
 * region attached (hclib_hip_global_*) subtrees below the split also move
 * between shards. level_hist (host, may be NULL) receives nodes per depth
 * for depth < max_levels (max_levels <= 65536). */
int hclib_hip_uts_search(const hclib_hip_uts_params_t *params, int shard, int nshards,
                         int split_depth, hclib_hip_uts_result_t *result, uint64_t *level_hist,
                         int max_levels);

/* The launch shape hclib_hip_uts_search chose for its last search on this
 * thread's module (diagnostic: tests pin the bench's exact configuration).
 * mode: 0 rule tables in global memory, 1 in LDS, 2 BIN, 3 fixed-shape GEO;
 * feat: 0 the plain kernel, 1 sharding / per-level counts, 2 depth trace;
 * seeded: breadth-first seeding of the top levels (seed_target slots). */
typedef struct {
    int mode, feat, workers_per_group, grid, ring, seeded, seed_target, spill_lo, waves_per_cu;
} hclib_hip_uts_launch_t;
int hclib_hip_uts_last_launch(hclib_hip_uts_launch_t *out);

/* Cross-GPU work sharing for sharded searches (one process per GPU;
 * SURVEY 8e items 2-3; the reference's distributed UTS moves work between
 * ranks, test/performance-regression/full-apps/uts/uts_hclib_shmem_opt.cpp
 * :98-140). One region of hclib_hip_global_bytes(cap) bytes lives in one
 * rank's device memory; the other ranks map it with hclib_hip_ipc_import
 * (handle from hclib_hip_ipc_export: HIP_IPC_HANDLE_SIZE = 64 bytes). Before
 * each sharded launch one rank resets it (hclib_hip_global_init, nranks =
 * ranks that will launch) and every rank waits for that (a barrier); a rank
 * that attached it (hclib_hip_global_attach, NULL detaches) then shares
 * work in every sharded hclib_hip_uts_search: idle waves take chunks from
 * the region's ring, busy waves export chunks while some rank is idle, and
 * each rank's launch ends only when no rank holds work (the region's
 * `active` count, system-scope atomics). hclib_hip_global_read fills
 * out[0] active, out[1] idle ranks, out[2] chunks queued, then per rank r
 * out[3 + 2r] chunks exported and out[4 + 2r] chunks imported (r < 16).
 * hclib_hip_global_alloc allocates the region itself (kind 0 uncached device
 * memory, 1 fine-grained, 2 plain hipMalloc; free with hclib_hip_global_free)
 * so that its IPC handle names exactly that allocation. */
size_t hclib_hip_global_bytes(uint32_t cap);
int hclib_hip_global_alloc(uint32_t cap, int kind, void **region_out);
int hclib_hip_global_free(void *region);
int hclib_hip_global_init(void *region, uint32_t cap, int nranks);
int hclib_hip_global_attach(void *region, uint32_t cap, int rank);
int hclib_hip_global_read(const void *region, uint64_t out[35]);
int hclib_hip_ipc_export(void *dev_ptr, void *handle_out);
int hclib_hip_ipc_import(const void *handle, void **dev_ptr_out);
int hclib_hip_ipc_close(void *dev_ptr);

/* Host-side helper (no GPU needed): evaluate the integer numChildren rule
 * the device uses (threshold tables built from the reference's libm
 * formula, uts.c:171-274) for an explicit node; lets the CPU tests check
 * the tables against the oracle. st = the 5 big-endian state words. */
/* Host check (no GPU) of the device's bucketed numChildren lookup for
 * fixed-shape GEO trees: returns the number of rand values where the bucket
 * method disagrees with #{k : thr[k] <= rand} (0), checking every threshold
 * +-3, every bucket edge +-1 and `nrandom` pseudo-random values; *checked =
 * values compared (0 for trees without a threshold table). */
int hclib_hip_uts_bucket_check(const hclib_hip_uts_params_t *params, uint64_t nrandom, uint64_t *checked);
int hclib_hip_uts_num_children_host(const hclib_hip_uts_params_t *params, int height,
                                    const uint32_t st[5]);

/* ----------------------------------------------------------------- fib */
typedef struct {
    uint64_t tasks;      /* fib tasks executed (each fib(n) call is one task) */
    uint64_t joins;      /* finish scopes closed (join counters reaching 0) */
    uint64_t chunks_pushed;
    uint64_t chunks_stolen;
    double kernel_ms;
    double busy_frac;        /* share of wave time spent inside batches */
} hclib_hip_fib_result_t;

/* fib(n) with one task per call and a join counter per finish scope
 * (continuation by the last arriver). n <= 80. */
int hclib_hip_fib(int n, int64_t *value, hclib_hip_fib_result_t *result);

/* ---------------------------------------------- device promise DAG */
/* Device promises/futures with dependency-counter release
 * (include/hclib_hip/hx_dag.h; replaces hclib_promise_put's waiter walk,
 * src/hclib-promise.c:132-245, and spawn_await, src/hclib-runtime.c:596-644,
 * for device tasks). The caller describes `ntasks` tasks, each with
 * `payload_words` u32 of payload and the promises it awaits (CSR:
 * await_off[ntasks + 1], await_ids), and the promises already put before the
 * launch (preput[p] != 0, their datum in preput_datum; either may be NULL).
 * begin() uploads the graph, sizes every task's dependency counter, seeds
 * the ready list with the tasks that wait on nothing and records the start
 * event; the caller launches `grid` workgroups of 64 threads on `stream`
 * running hx::run_dag_worker<Kind> over `view` (hclib::hip::run_dag does
 * both); end() waits, copies each promise's datum / satisfied flag back
 * (either output may be NULL) and returns HCLIB_HIP_EDEVICE for a double put
 * or a task nothing releases (bounded spin, the reference's end_finish
 * deadlock). */
typedef struct {
    void *view;        /* hx::DagView (device pointers, by value) */
    void *stream;      /* hipStream_t of the module */
    int grid;          /* workgroups (waves) to launch */
    uint32_t ntasks, npromises;
} hclib_hip_dag_launch_t;

typedef struct {
    uint64_t tasks;      /* tasks executed */
    uint64_t puts;       /* device puts */
    uint64_t releases;   /* counter decrements that made a task ready */
    double kernel_ms;
} hclib_hip_dag_stats_t;

int hclib_hip_dag_begin(uint32_t ntasks, uint32_t npromises, uint32_t payload_words,
                        const uint32_t *payload, const uint32_t *await_off, const uint32_t *await_ids,
                        const uint8_t *preput, const uint64_t *preput_datum, int waves_per_cu,
                        uint32_t spin_limit_ms, hclib_hip_dag_launch_t *out);
int hclib_hip_dag_end(const char *who, uint64_t *datum_out, uint8_t *satisfied_out,
                      hclib_hip_dag_stats_t *stats);

/* ------------------------------------------ dynamic device dataflow */
/* Device tasks that create promises and async_await tasks while the launch
 * runs (include/hclib_hip/hx_dyn.h; hclib_promise_create / put and
 * spawn_await of src/hclib-promise.c:55-245, src/hclib-runtime.c:596-644 as
 * running tasks use them). begin() allocates the pools — task_cap tasks of
 * payload_words u32 each, promise_cap promises, node_cap wait nodes (one per
 * registered future) — seeds the ready list with the `nroots` root tasks
 * (payloads in root_payload) and records the start event; the caller
 * launches `grid` workgroups of 64 threads on `stream` running
 * hx::run_dyn_worker<Kind> over `view` (hclib::hip::run_dyn does both);
 * end() waits and returns HCLIB_HIP_EDEVICE for a double put, an exhausted
 * pool or tasks that wait on promises nothing puts (bounded spin, the
 * reference's end_finish deadlock). datum() then reads promises back. */
typedef struct {
    void *view;    /* hx::DynView (device pointers, by value) */
    void *stream;  /* hipStream_t of the module */
    int grid;      /* workgroups (waves) to launch */
} hclib_hip_dyn_launch_t;

typedef struct {
    uint64_t tasks;     /* tasks run (roots included) */
    uint64_t created;   /* tasks created by device async_await */
    uint64_t puts;      /* device puts */
    uint64_t releases;  /* waiters a put made runnable */
    uint64_t promises;  /* promises created on the device */
    double kernel_ms;
} hclib_hip_dyn_stats_t;

int hclib_hip_dyn_begin(uint32_t payload_words, const uint32_t *root_payload, uint32_t nroots, uint32_t task_cap,
                        uint32_t promise_cap, uint32_t node_cap, int waves_per_cu, uint32_t spin_limit_ms,
                        hclib_hip_dyn_launch_t *out);
int hclib_hip_dyn_end(const char *who, hclib_hip_dyn_stats_t *stats);
/* promises [first, first + n) of the last launch: data, and whether put */
int hclib_hip_dyn_datum(uint32_t first, uint32_t n, uint64_t *datum, uint8_t *put);

/* ---------------------------------------------------------------- SW */
typedef struct {
    uint64_t tiles;      /* tile tasks executed */
    uint64_t releases;   /* dependency-counter decrements */
    double kernel_ms;
    double cells_per_s;
    double tile_us;      /* average in-tile DP time per tile task */
    double release_us;   /* average dependency-release time per tile task */
} hclib_hip_sw_result_t;

/* Tiled global alignment of smith_waterman.cpp over host sequences coded
 * 1..4 (A,C,G,T). Tile grid = (n1/tw) x (n2/th); remainders dropped as the
 * reference does. tw must be a multiple of 64... no: any tw <= 4096, th a
 * multiple of 64 or th <= 64*16. Writes the score (bottom-right cell). */
int hclib_hip_sw(const int8_t *s1, size_t n1, const int8_t *s2, size_t n2, int tw, int th,
                 int *score, hclib_hip_sw_result_t *result);

/* Column-band session (multi-GPU SW, one band of tile columns per rank).
 * The reference runs the whole tile DAG in one address space
 * (smith_waterman.cpp:168-235); sharded, rank r owns tile columns [j0, j1)
 * and its only inputs from other ranks are the left band's right column
 * (the reference's right_column promises of tile column j0-1, :212-216) and
 * its bottom-right corners (:222-226), both carried by one int array:
 *   begin   uploads s1/s2 (coded 1..4) and allocates the band's granules;
 *   rows    launches tile rows [i0, i1) of the band on `stream` (a
 *           hipStream_t); left_in = device array of nth*th ints holding H of
 *           matrix column j0*tw for rows 1..nth*th (rows up to i1*th must be
 *           in place; NULL only when j0 == 0); right_out (device, nth*th
 *           ints, or NULL) receives H of column j1*tw for the same rows;
 *   end     synchronises the stream, checks the device error word, writes
 *           the band's bottom-right cell (the score for the last band) and
 *           the tiles executed, and frees the band. */
typedef struct hclib_hip_sw_band hclib_hip_sw_band_t;
int hclib_hip_sw_band_begin(const int8_t *s1, size_t n1, const int8_t *s2, size_t n2, int tw, int th,
                            int j0, int j1, hclib_hip_sw_band_t **band);
int hclib_hip_sw_band_rows(hclib_hip_sw_band_t *band, int i0, int i1, const int *left_in, int *right_out,
                           void *stream);
int hclib_hip_sw_band_end(hclib_hip_sw_band_t *band, void *stream, int *corner, uint64_t *tiles);

#ifdef __cplusplus
}
#endif
#endif /* HCLIB_HIP_H_ */
