/* global_sharing_model.c — a CPU model of the cross-GPU work-sharing and
 * termination protocol of include/hclib_hip/hx_sched.h (GlobalHdr /
 * GlobalView, global_enqueue / global_dequeue, wave_goes_idle, the import
 * path of run_worker), restated in C11 atomics and run under ThreadSanitizer
 * with random interleavings (tests/test_model.py).
 *
 * Mapping: a rank = one GPU's launch; a worker thread = one wave. Per rank:
 *   outstanding  chunks queued in the rank's local deque + workers holding work
 *   a local MPMC chunk ring (the HBM deques' {seq, cnt} slot format)
 * Shared by all ranks (rank 0's HBM on the device, system-scope atomics):
 *   active       ranks holding work + chunks queued in the global ring
 *   idle         ranks with no local work (the global hunger signal)
 *   held[r]      the handshake word of rank r's unit: 1 while the rank holds
 *                its unit of `active`, 0 once a release has fully landed
 *   a bounded MPMC global chunk ring, err (first error, every rank stops)
 *
 * Protocol (what the device does, in this order):
 *   release  (the worker whose outstanding decrement returns 1):
 *              idle += 1 (returning); held[r] = 0 (release); active -= 1
 *   import   (global_dequeue succeeded): prev = outstanding++;
 *              if prev == 0 (the rank had nothing):
 *                  wait held[r] == 0 (acquire), CAS held[r] 0 -> 1,
 *                  active += 1, idle -= 1
 *              then active -= 1 (the chunk's unit passes to the rank)
 *   export   (a rank is idle, none of this rank's workers is hungry):
 *              active += 1 before the chunk is published
 *   local spill / take: outstanding += 1 before publish; the taker inherits
 *   terminate: a worker with nothing leaves once outstanding == 0 and
 *              active == 0 (or err != 0)
 * Because the 1->0 and 0->1 transitions of a rank's `outstanding` strictly
 * alternate, and the importer waits for the previous release's idle += 1 to
 * land before its idle -= 1, `idle` never reads below 0 (round 2's protocol
 * did idle -= 1 without the handshake and could read 0xFFFFFFFF).
 *
 * Checked, for every seed: every node of the tree is processed exactly once
 * (count and a checksum of node ids), `active` never reads 0 while any
 * worker holds work or any chunk is queued (a monitor thread), `idle` always
 * reads within [0, ranks], and every worker terminates (watchdog).
 *
 * Usage: global_sharing_model [ranks workers seeds] [--old]
 *   --old: round 2's import path (no handshake), to show the underflow the
 *          handshake removes (reported, not asserted).
 * This file is a protocol model (test infrastructure); the product is the
 * device code it restates. */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define MAXR 16
#define MAXW 8
#define CHUNK 8
#define GCAP 32  /* global ring slots (small: exercises the full ring) */
#define LCAP 64  /* local ring slots per rank */
#define STACK 4096

typedef struct {
    uint32_t id;    /* node id (unique) */
    uint32_t depth;
} item_t;

typedef struct {
    _Atomic uint32_t seq; /* pos when free for ticket pos, pos + 1 once published */
    uint32_t cnt;
    item_t items[CHUNK];
} slot_t;

typedef struct {
    _Atomic uint32_t head, tail;
    slot_t *slots;
    uint32_t cap;
} ring_t;

static int R = 8, W = 3, OLD = 0;
static uint32_t MAXDEPTH = 9;

static _Atomic int32_t g_active, g_idle;
static _Atomic int32_t g_held[MAXR];
static _Atomic int g_err;
static ring_t g_ring;

static _Atomic int32_t r_outstanding[MAXR];
static ring_t r_ring[MAXR];

static _Atomic uint64_t done_nodes, done_sum;
static _Atomic int workers_left;
static _Atomic int32_t min_idle_seen, max_idle_seen;
static _Atomic long exports, imports, violations, early_decrements;
static _Atomic int32_t pending_rel[MAXR]; /* model-only: a release whose idle += 1 has not landed */

/* ---- the tree: node children from a hash of the id (skewed: a few deep
 * subtrees), total computed serially */
static uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
static uint32_t nchildren(item_t n) {
    if (n.depth >= MAXDEPTH) return 0;
    uint32_t h = hash32(n.id * 2654435761u + n.depth);
    return (h % 5 == 0) ? 6 : (h % 2 == 0 ? 2 : 0); /* mean 2: ~2^depth nodes per root */
}
static item_t child(item_t n, uint32_t k) {
    item_t c = {hash32(n.id ^ (k + 1) * 0x9e3779b9u) | 1u, n.depth + 1};
    return c;
}
static void serial_count(item_t n, uint64_t *cnt, uint64_t *sum) {
    *cnt += 1;
    *sum += n.id;
    uint32_t c = nchildren(n);
    for (uint32_t k = 0; k < c; ++k) serial_count(child(n, k), cnt, sum);
}

/* ---- random interleaving noise */
static __thread uint32_t t_rng;
static void jitter(void) {
    t_rng = hash32(t_rng + 0x1234567u);
    if ((t_rng & 15) == 0) sched_yield();
    else if ((t_rng & 15) == 1) {
        for (volatile int i = 0; i < (int)(t_rng >> 24); ++i) {
        }
    }
}

/* ---- bounded MPMC ring with the device's {seq, cnt} slot protocol */
static void ring_init(ring_t *q, uint32_t cap) {
    q->slots = calloc(cap, sizeof(slot_t));
    q->cap = cap;
    atomic_store(&q->head, 0);
    atomic_store(&q->tail, 0);
    for (uint32_t i = 0; i < cap; ++i) atomic_store(&q->slots[i].seq, i);
}
static int ring_push(ring_t *q, const item_t *it, uint32_t n, _Atomic int32_t *count_first) {
    uint32_t hd = atomic_load(&q->head), tl = atomic_load(&q->tail);
    if ((int32_t)(tl - hd) >= (int32_t)(q->cap / 2)) return 0; /* refuse a half-full ring */
    if (count_first) atomic_fetch_add(count_first, 1);          /* counted before visible */
    uint32_t pos = atomic_fetch_add(&q->tail, 1);
    slot_t *s = &q->slots[pos & (q->cap - 1)];
    long spins = 0;
    while (atomic_load_explicit(&s->seq, memory_order_acquire) != pos) {
        if (++spins > 200000000L) {
            atomic_store(&g_err, 1);
            return 1; /* (the device stops every rank through err) */
        }
        sched_yield();
    }
    memcpy(s->items, it, n * sizeof(item_t));
    s->cnt = n;
    jitter();
    atomic_store_explicit(&s->seq, pos + 1, memory_order_release);
    return 1;
}
static uint32_t ring_pop(ring_t *q, item_t *out) {
    uint32_t hd = atomic_load(&q->head), tl = atomic_load(&q->tail);
    if ((int32_t)(tl - hd) <= 0) return 0;
    if (!atomic_compare_exchange_strong(&q->head, &hd, hd + 1)) return 0;
    slot_t *s = &q->slots[hd & (q->cap - 1)];
    long spins = 0;
    while (atomic_load_explicit(&s->seq, memory_order_acquire) != hd + 1) {
        if (++spins > 200000000L) {
            atomic_store(&g_err, 2);
            return 0;
        }
        sched_yield();
    }
    uint32_t n = s->cnt;
    memcpy(out, s->items, n * sizeof(item_t));
    atomic_store_explicit(&s->seq, hd + q->cap, memory_order_release);
    return n;
}

/* ---- the protocol */
static void observe_idle(void) {
    int32_t v = atomic_load(&g_idle);
    int32_t m = atomic_load(&min_idle_seen);
    while (v < m && !atomic_compare_exchange_weak(&min_idle_seen, &m, v)) {
    }
    m = atomic_load(&max_idle_seen);
    while (v > m && !atomic_compare_exchange_weak(&max_idle_seen, &m, v)) {
    }
}

static void rank_release(int r) { /* wave_goes_idle: outstanding went 1 -> 0 */
    atomic_fetch_add(&g_idle, 1);
    atomic_store(&pending_rel[r], 0);
    jitter();
    if (!OLD) atomic_store_explicit(&g_held[r], 0, memory_order_release);
    jitter();
    atomic_fetch_sub(&g_active, 1);
}
static void worker_goes_idle(int r) {
    int32_t prev = atomic_fetch_sub(&r_outstanding[r], 1);
    if (prev == 1) {
        atomic_store(&pending_rel[r], 1);
        jitter(); /* the device's window: the rank's unit is released by later atomics */
        jitter();
        rank_release(r);
    }
}
static void rank_import(int r) { /* a global chunk arrived in rank r */
    int32_t prev = atomic_fetch_add(&r_outstanding[r], 1);
    if (prev == 0) {
        if (!OLD) {
            long spins = 0;
            int32_t z = 0;
            /* the release that took outstanding to 0 may still be landing */
            while (!atomic_compare_exchange_weak_explicit(&g_held[r], &z, 1, memory_order_acquire,
                                                          memory_order_relaxed)) {
                z = 0;
                if (++spins > 200000000L) {
                    atomic_store(&g_err, 3);
                    return;
                }
                sched_yield();
            }
        }
        atomic_fetch_add(&g_active, 1);
        jitter();
        /* idle -= 1 before this rank's own idle += 1 landed: the count reads
         * one rank short (below 0 when no other rank is idle) */
        if (atomic_load(&pending_rel[r])) atomic_fetch_add(&early_decrements, 1);
        atomic_fetch_sub(&g_idle, 1);
        observe_idle();
    }
    jitter();
    atomic_fetch_sub(&g_active, 1); /* the chunk's unit becomes the rank's */
}

typedef struct {
    int r, w;
    int seed_roots;
} warg_t;

static _Atomic int32_t holding_workers; /* monitor: workers with items in hand */
static _Atomic int32_t queued_chunks;   /* monitor: chunks in any ring */

static void *worker(void *p) {
    warg_t *a = p;
    const int r = a->r;
    t_rng = hash32((uint32_t)(r * 131 + a->w * 7 + 1) ^ (uint32_t)(uintptr_t)&a);
    item_t *st = malloc(sizeof(item_t) * STACK);
    uint32_t top = 0;
    int holding = 0;
    if (a->seed_roots) {
        /* every rank starts holding its unit (host: active = ranks,
         * outstanding = 1); the rank's roots go to its seeding worker */
        for (uint32_t i = 0; i < (uint32_t)(r == 0 ? 3 : (r % 3 == 1 ? 1 : 0)); ++i) {
            item_t root = {hash32(0xabcdef01u + (uint32_t)r * 977u + i) | 1u, 0};
            st[top++] = root;
        }
        holding = 1;
        atomic_fetch_add(&holding_workers, 1);
    }
    long spins = 0;
    for (;;) {
        if (top == 0) {
            if (holding) {
                holding = 0;
                atomic_fetch_sub(&holding_workers, 1);
                worker_goes_idle(r);
            }
            item_t buf[CHUNK];
            uint32_t n = ring_pop(&r_ring[r], buf);
            if (n) { /* inherits the chunk's unit of outstanding */
                atomic_fetch_add(&holding_workers, 1);
                atomic_fetch_sub(&queued_chunks, 1);
            } else if ((spins & 3) == 3) {
                n = ring_pop(&g_ring, buf);
                if (n) {
                    atomic_fetch_add(&holding_workers, 1);
                    atomic_fetch_sub(&queued_chunks, 1);
                    rank_import(r);
                    atomic_fetch_add(&imports, 1);
                }
            }
            if (n) {
                memcpy(st, buf, n * sizeof(item_t));
                top = n;
                holding = 1;
                spins = 0;
                continue;
            }
            if (atomic_load(&g_err)) break;
            if ((spins & 7) == 7 && atomic_load(&r_outstanding[r]) == 0 && atomic_load(&g_active) == 0) break;
            if (++spins > 400000000L) {
                atomic_store(&g_err, 4);
                break;
            }
            observe_idle();
            sched_yield();
            continue;
        }
        /* one "batch": pop an item, process it, push its children */
        item_t it = st[--top];
        atomic_fetch_add(&done_nodes, 1);
        atomic_fetch_add(&done_sum, it.id);
        uint32_t c = nchildren(it);
        if (top + c > STACK) {
            atomic_store(&g_err, 5);
            break;
        }
        for (uint32_t k = 0; k < c; ++k) st[top++] = child(it, k);
        jitter();
        /* hunger: some worker of this rank holds nothing and no chunk waits */
        int32_t outst = atomic_load(&r_outstanding[r]);
        int hungry = W - outst > 0;
        if (top > 2 * CHUNK && hungry) {
            atomic_fetch_add(&queued_chunks, 1);
            if (ring_push(&r_ring[r], st, CHUNK, &r_outstanding[r])) {
                memmove(st, st + CHUNK, (top - CHUNK) * sizeof(item_t));
                top -= CHUNK;
            } else {
                atomic_fetch_sub(&queued_chunks, 1);
            }
        } else if (top > 2 * CHUNK && (int32_t)atomic_load(&g_idle) > 0) {
            /* export the oldest items to an idle rank */
            atomic_fetch_add(&queued_chunks, 1);
            if (ring_push(&g_ring, st, CHUNK, &g_active)) {
                memmove(st, st + CHUNK, (top - CHUNK) * sizeof(item_t));
                top -= CHUNK;
                atomic_fetch_add(&exports, 1);
            } else {
                atomic_fetch_sub(&queued_chunks, 1);
            }
        }
    }
    if (holding) {
        atomic_fetch_sub(&holding_workers, 1);
        worker_goes_idle(r);
    }
    free(st);
    atomic_fetch_sub(&workers_left, 1);
    return NULL;
}

static void *monitor(void *p) {
    (void)p;
    while (atomic_load(&workers_left) > 0) {
        /* active == 0 must mean: no worker holds work, no chunk is queued
         * (read the work indicators AFTER active: anything created before
         * active read 0 must already be gone) */
        if (atomic_load(&g_active) == 0) {
            int32_t h = atomic_load(&holding_workers), q = atomic_load(&queued_chunks);
            if (h != 0 || q != 0) atomic_fetch_add(&violations, 1);
        }
        observe_idle();
        sched_yield();
    }
    return NULL;
}

static int run_seed(uint32_t seed) {
    MAXDEPTH = 9 + seed % 5;
    atomic_store(&g_active, R);
    atomic_store(&g_idle, 0);
    atomic_store(&g_err, 0);
    ring_init(&g_ring, GCAP);
    for (int r = 0; r < R; ++r) {
        atomic_store(&g_held[r], 1);
        atomic_store(&pending_rel[r], 0);
        atomic_store(&r_outstanding[r], 1);
        ring_init(&r_ring[r], LCAP);
    }
    atomic_store(&done_nodes, 0);
    atomic_store(&done_sum, 0);
    atomic_store(&holding_workers, 0);
    atomic_store(&queued_chunks, 0);
    atomic_store(&min_idle_seen, 0);
    atomic_store(&max_idle_seen, 0);
    atomic_store(&workers_left, R * W);
    uint64_t want_n = 0, want_s = 0;
    for (int r = 0; r < R; ++r)
        for (uint32_t i = 0; i < (uint32_t)(r == 0 ? 3 : (r % 3 == 1 ? 1 : 0)); ++i) {
            item_t root = {hash32(0xabcdef01u + (uint32_t)r * 977u + i) | 1u, 0};
            serial_count(root, &want_n, &want_s);
        }
    pthread_t th[MAXR * MAXW], mon;
    warg_t args[MAXR * MAXW];
    pthread_create(&mon, NULL, monitor, NULL);
    for (int r = 0; r < R; ++r)
        for (int w = 0; w < W; ++w) {
            args[r * W + w] = (warg_t){r, w, w == 0};
            pthread_create(&th[r * W + w], NULL, worker, &args[r * W + w]);
        }
    for (int i = 0; i < R * W; ++i) pthread_join(th[i], NULL);
    pthread_join(mon, NULL);
    int ok = 1;
    const uint64_t gn = atomic_load(&done_nodes), gs = atomic_load(&done_sum);
    if (atomic_load(&g_err)) {
        printf("seed %u: protocol error %d\n", seed, atomic_load(&g_err));
        ok = 0;
    }
    if (gn != want_n || gs != want_s) {
        printf("seed %u: nodes %llu (want %llu), checksum %llu (want %llu)\n", seed, (unsigned long long)gn,
               (unsigned long long)want_n, (unsigned long long)gs, (unsigned long long)want_s);
        ok = 0;
    }
    if (atomic_load(&g_active) != 0) {
        printf("seed %u: active %d at the end\n", seed, atomic_load(&g_active));
        ok = 0;
    }
    free(g_ring.slots);
    for (int r = 0; r < R; ++r) free(r_ring[r].slots);
    return ok;
}

static void on_alarm(int sig) {
    (void)sig;
    static const char msg[] = "watchdog: the model did not terminate\n";
    if (write(2, msg, sizeof msg - 1) < 0) {
    }
    _exit(3);
}

int main(int argc, char **argv) {
    int seeds = 20;
    int pos = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--old")) OLD = 1;
        else if (pos == 0) R = atoi(argv[i]), ++pos;
        else if (pos == 1) W = atoi(argv[i]), ++pos;
        else if (pos == 2) seeds = atoi(argv[i]), ++pos;
    }
    if (R < 1 || R > MAXR || W < 1 || W > MAXW) return 2;
    signal(SIGALRM, on_alarm);
    alarm(600);
    int ok = 1;
    int32_t min_idle = 0, max_idle = 0;
    for (int s = 0; s < seeds; ++s) {
        ok &= run_seed((uint32_t)s);
        if (atomic_load(&min_idle_seen) < min_idle) min_idle = atomic_load(&min_idle_seen);
        if (atomic_load(&max_idle_seen) > max_idle) max_idle = atomic_load(&max_idle_seen);
    }
    printf("ranks %d workers %d seeds %d protocol %s: exports %ld imports %ld, idle range [%d, %d], "
           "idle decrements before the rank's own release landed %ld, active==0-with-work violations %ld\n",
           R, W, seeds, OLD ? "round-2 (no handshake)" : "handshake", atomic_load(&exports),
           atomic_load(&imports), min_idle, max_idle, atomic_load(&early_decrements), atomic_load(&violations));
    if (atomic_load(&violations)) ok = 0;
    if (!OLD && atomic_load(&early_decrements)) ok = 0;
    if (!OLD && (min_idle < 0 || max_idle > R)) ok = 0;
    printf(ok ? "MODEL OK\n" : "MODEL FAILED\n");
    return ok ? 0 : 1;
}
