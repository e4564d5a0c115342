"""The N>1 path on CPU: two gloo ranks shard a UTS tree and combine the
counts with the same all-reduce code bench.py uses over RCCL. The shard
work here is the oracle's serial walk over disjoint root-child ranges (the
GPU shards by node hash at the split depth; tests/test_gpu.py checks that
those shards sum to the tree)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, args, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from hclib_amd import dist
    from oracle import loader as L

    r, w, _ = dist.init_from_env("gloo")
    p = L.parse_uts_args(args)
    root_nc = L.uts_num_children(p, p.type, 0, L.rng_init(p.root_id))
    per = (root_nc + w - 1) // w
    n, lv, d = L.uts_root_range(p, r * per, min(root_nc, (r + 1) * per), r == 0)
    tot = dist.combine_counts(n, lv, d, w, "gloo")
    t = dist.max_over_ranks(float(r), w, "gloo")
    dist.barrier(w, "gloo")
    dist.shutdown(w)
    q.put((r, tot, t))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_uts_counts_combine_over_gloo(golden, world):
    g = golden("uts_goldens.json")["published"]["T1"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, g["args"], q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, tot, t in res:
        assert tot == (g["nodes"], g["leaves"], g["depth"])
        assert t == world - 1


# ---------------------------------------------------------------- SW bands
# The sharded Smith-Waterman pipeline (hclib_amd/dist.py ShardedSw) over
# gloo: every rank runs its band of tile columns with a host DP standing in
# for the HIP band kernel (tests/test_gpu.py runs the same pipeline on the
# GPU), exchanging right columns block by block. Checked against the oracle:
# the score, and each band's right column against the oracle's last column
# of the matrix cut at that band's right edge (the column does not depend on
# anything to its right).

_M = [[-1] * 5, [-1, 2, -4, -2, -4], [-1, -4, 2, -4, -2], [-1, -2, -4, 2, -4], [-1, -4, -2, -4, 2]]


class _HostBand:
    """Host DP of one band: H[0][c] = -c, left column from the left band
    (or -r), smith_waterman.cpp:201-210 recurrence."""

    def __init__(self, s1, s2, tw, th, j0, j1):
        self.s1, self.s2, self.th = s1, s2, th
        self.c0, self.c1 = j0 * tw, j1 * tw
        self.prev = [-c for c in range(self.c0, self.c1 + 1)]  # H[row][c0..c1]
        self.row = 0
        self.tiles = 0
        self.tw_count = j1 - j0

    def rows(self, i0, i1, left, right):
        assert self.row == i0 * self.th
        for r in range(i0 * self.th + 1, i1 * self.th + 1):
            cur = [int(left[r - 1]) if left is not None else -r]
            m = _M[self.s2[r - 1]]
            for k, c in enumerate(range(self.c0 + 1, self.c1 + 1)):
                cur.append(max(cur[k] - 1, self.prev[k + 1] - 1, self.prev[k] + m[self.s1[c - 1]]))
            if right is not None:
                right[r - 1] = cur[-1]
            self.prev = cur
        self.row = i1 * self.th
        self.tiles += (i1 - i0) * self.tw_count

    def end(self):
        return self.prev[-1], self.tiles


def _sw_worker(rank, world, port, s1, s2, tw, th, block_rows, q, side_group=False):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch

    from hclib_amd import dist

    r, w, _ = dist.init_from_env("gloo")
    # side_group: the exchange on its own group, as bench.py runs it beside
    # an RCCL world group
    group = torch.distributed.new_group(backend="gloo") if side_group else None
    job = dist.ShardedSw(s1, s2, tw, th, r, w, "gloo", block_rows, band_factory=_HostBand,
                         device=torch.device("cpu"), group=group)
    score, tiles = job.run()
    right = None if job.right is None else job.right.tolist()
    dist.barrier(w, "gloo")
    dist.shutdown(w)
    q.put((r, score, tiles, job.j1, right))


@pytest.mark.parametrize("world,block_rows,side_group", [(2, 2, False), (3, 1, False), (3, 5, True)])
def test_sharded_sw_pipeline_over_gloo(world, block_rows, side_group):
    import random

    from oracle import loader as L

    rng = random.Random(world * 10 + block_rows)
    tw, th = 8, 6
    s1 = bytes(rng.randint(1, 4) for _ in range(7 * tw + 3))  # ragged tails are dropped
    s2 = bytes(rng.randint(1, 4) for _ in range(5 * th + 2))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sw_worker, args=(r, world, port, s1, s2, tw, th, block_rows, q, side_group))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = L.sw_score(s1, s2, tw, th)
    for r, score, tiles, j1, right in res:
        assert score == want
        assert tiles == 7 * 5
        if right is not None:
            _, _, col = L.sw_score(s1[:j1 * tw], s2, tw, th, want_edges=True)
            assert right == col[1:]


def test_sw_band_and_block_split():
    from hclib_amd import dist

    assert dist.sw_bands(256, 8) == [(32 * r, 32 * r + 32) for r in range(8)]
    assert dist.sw_bands(7, 3) == [(0, 2), (2, 4), (4, 7)]
    assert dist.sw_blocks(10, 4) == [(0, 4), (4, 8), (8, 10)]
    with pytest.raises(ValueError):
        dist.sw_bands(2, 3)
    with pytest.raises(ValueError):
        dist.sw_blocks(4, 0)


# ------------------------------------------------ cross-GPU sharing leg
# bench.py's N>1 work-sharing leg must never take the scaling run down: a
# rank that cannot set the shared region up (here: no GPU at all) reports it
# and every rank still reaches the same collectives, returning an error
# record instead of raising or hanging.
def _sharing_worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    import hclib_amd as H
    from hclib_amd import dist

    r, w, _ = dist.init_from_env("gloo")
    out = bench.skewed_sharing(H, r, w, "gloo")
    dist.barrier(w, "gloo")
    dist.shutdown(w)
    q.put((r, out))


def test_bench_work_sharing_leg_reports_setup_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the leg would run for real")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, out in res:
        assert "error" in out and "static" not in out and "shared" not in out
        assert out["workload"].startswith("test/uts T1L")


# ------------------------------------------------------ stalled-leg guard
# bench.py runs its N > 1 legs under dist.LegGuard: here rank 1 stalls in the
# first leg (it never enters the collective rank 0 waits in), so rank 0's leg
# times out; both ranks then skip the second leg (the stall is flagged in the
# rendezvous store), rank 0 still produces its line within the bound, and
# every rank leaves with os._exit as bench.py does.
def _stall_worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HCLIB_DIST_TIMEOUT_S": "60"})
    import threading
    import time

    import torch
    import torch.distributed as tdist

    from hclib_amd import dist

    r, w, _ = dist.init_from_env("gloo")
    legs = dist.LegGuard(w, 4.0)

    def leg_a():
        if r == 1:
            threading.Event().wait()  # stalls forever
        t = torch.ones(1)
        tdist.all_reduce(t)  # rank 0 waits here for rank 1
        return {"sum": float(t[0])}

    t0 = time.monotonic()
    a = legs.run("a", leg_a)
    b = legs.run("b", lambda: {"ok": True})
    q.put((r, a, b, legs.stalled, time.monotonic() - t0))
    q.close()
    q.join_thread()  # the feeder thread flushes before the hard exit
    os._exit(0)


def test_stalled_leg_is_reported_and_the_line_still_prints():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stall_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r, a, b, stalled, el in res:
        assert "timeout" in a["failed"], (r, a)
        assert b["failed"].startswith("skipped"), (r, b)
        assert stalled
        assert el < 30, el  # the guard's bound (4 s per leg), not the collective's 60 s


# ------------------------------------------- SW exchange fallback is collective
# bench.py's sharded SW leg (dist.sw_exchange): rank 1's exchange raises on
# its first receive of the primary attempt while rank 0 is blocked sending to
# it. Rank 1 flags the failure in the rendezvous store, rank 0's send wait
# sees the flag and stops, both agree on a gloo control group and re-measure
# together over a fresh gloo exchange group; the result is exact and the
# whole leg ends within seconds (not the group's 60 s timeout).
def _sw_fallback_worker(rank, world, port, s1, s2, tw, th, q, fail_gloo_too, fail_step=0):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HCLIB_DIST_TIMEOUT_S": "60"})
    import time

    import torch

    from hclib_amd import dist

    r, w, _ = dist.init_from_env("gloo")
    attempts = []

    def make_job(xb, group, abort):
        attempts.append(xb)
        first = len(attempts) == 1 + fail_step  # the primary attempt's step fail_step

        def inject():
            if r == 1 and (first or fail_gloo_too):
                raise RuntimeError("injected exchange failure")
        return dist.ShardedSw(s1, s2, tw, th, r, w, xb, 1, band_factory=_HostBand, device=torch.device("cpu"),
                              group=group, abort=abort, inject=inject)

    want = (__import__("oracle.loader", fromlist=["sw_score"]).sw_score(s1, s2, tw, th), (len(s1) // tw) * (len(s2) // th))
    t0 = time.monotonic()
    res = dist.sw_exchange(make_job, r, w, "gloo", want, steps=1 + fail_step)
    el = time.monotonic() - t0
    q.put((r, res, el, attempts))
    q.close()
    q.join_thread()
    os._exit(0)  # abandoned transfers of the failed attempt: no orderly shutdown


@pytest.mark.parametrize("fail_gloo_too,fail_step", [(False, 0), (True, 0), (False, 1)])
def test_sw_exchange_failure_falls_back_on_every_rank(fail_gloo_too, fail_step):
    """fail_step 1: rank 1 fails in the second step of the primary attempt,
    after a first step both ranks completed (round-5 advisor: the ranks must
    not end up in different collectives on the control group)."""
    import random

    rng = random.Random(7)
    tw, th = 8, 6
    s1 = bytes(rng.randint(1, 4) for _ in range(4 * tw))
    s2 = bytes(rng.randint(1, 4) for _ in range(5 * th))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sw_fallback_worker, args=(r, 2, port, s1, s2, tw, th, q, fail_gloo_too, fail_step))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r, out, el, attempts in res:
        assert el < 10.0, (r, el)
        # both ranks re-ran, together (one job per step of each attempt made)
        assert attempts[:1 + fail_step] == ["gloo"] * (1 + fail_step) and len(attempts) >= 2 + fail_step, (r, attempts)
        if fail_gloo_too:
            assert "failed" in out and "injected" in out["failed"], (r, out)
        else:
            assert "injected exchange failure" in out["fallback"], (r, out)
            assert out["exchange"] == "gloo" and out["ms"] > 0
