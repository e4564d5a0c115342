"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL.

The UTS search shards statically (hash of the node state at the split
depth, uts.hip), so the data path has no collective. The only exchange is
the termination/reduction step the reference's distributed UTS does with
SHMEM (test/performance-regression/full-apps/uts/uts_hclib_shmem_opt.cpp:
98-140: a global counter + final reductions): one all-reduce of
(nodes, leaves) with SUM and one of depth with MAX, plus a MAX of the
per-rank elapsed time for the bench. Backend "nccl" is RCCL on ROCm; the
same code runs on "gloo" for the CPU tests.
"""
from __future__ import annotations

import datetime
import os
import threading


def init_from_env(backend: str = "nccl", share_device: bool = False):
    """Initialise the process group from RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*.
    Returns (rank, world, local_rank); world == 1 needs no process group.
    share_device (rehearsals on a 1-GPU box, gloo only): every rank drives
    device 0 instead of device LOCAL_RANK."""
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if share_device and backend == "nccl" and world > 1:
        raise ValueError("share_device needs a non-RCCL backend (one GPU per RCCL rank)")
    dev = 0 if share_device else local
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a bounded rendezvous / collective timeout (HCLIB_DIST_TIMEOUT_S,
        # default 300 s): a rank that never arrives fails the job instead of
        # hanging it for torch's default; RCCL collectives that time out then
        # raise in the waiting rank (async error handling 2: abort the
        # communicator, keep the process) rather than killing it
        timeout = datetime.timedelta(seconds=int(os.environ.get("HCLIB_DIST_TIMEOUT_S", "300")))
        if backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev), timeout=timeout)
        else:
            if share_device:
                torch.cuda.set_device(dev)
            dist.init_process_group(backend, timeout=timeout)
    elif backend == "nccl":
        torch.cuda.set_device(dev)
    return rank, world, local


class LegGuard:
    """Wall-clock guard for the optional legs of a multi-rank run (bench.py's
    N > 1 extras: sharded triad, sharded SW, cross-GPU work sharing). Each leg
    runs in a worker thread; a leg with no result after `timeout_s` is
    reported as failed and marks the job stalled in the rendezvous store
    (served by rank 0's process, so it answers while any rank's main thread
    is blocked), after which every rank skips the remaining legs. A leg that
    raises is reported with its exception. The caller prints its line and,
    when `stalled`, leaves with os._exit (a blocked collective thread would
    hold a normal shutdown) and a non-zero status (bench.py: 3)."""

    KEY = "hclib_leg_stalled"

    def __init__(self, world: int, timeout_s: float, device: int | None = None, store=None):
        self.world, self.timeout_s, self.device = world, timeout_s, device
        self.stalled = False
        self.store = store
        if self.store is None and world > 1:
            import torch.distributed as dist

            try:
                self.store = dist.distributed_c10d._get_default_store()
            except Exception:  # noqa: BLE001 (no store: each rank only knows its own stalls)
                self.store = None

    def peer_stalled(self) -> bool:
        if self.store is None:
            return False
        try:
            return bool(self.store.check([self.KEY]))
        except Exception:  # noqa: BLE001
            return False

    def run(self, name: str, fn):
        """fn() -> dict; returns its result or {"failed": reason}."""
        if self.stalled or self.peer_stalled():
            self.stalled = True
            return {"failed": "skipped: an earlier leg stalled on some rank"}
        box = {}

        def target():
            try:
                if self.device is not None:
                    import torch

                    torch.cuda.set_device(self.device)
                box["r"] = fn()
            except BaseException as e:  # noqa: BLE001 (SystemExit from a mismatch included)
                box["e"] = f"{type(e).__name__}: {e}"

        th = threading.Thread(target=target, name=f"leg-{name}", daemon=True)
        th.start()
        th.join(self.timeout_s)
        if th.is_alive():
            self.stalled = True
            if self.store is not None:
                try:
                    self.store.set(self.KEY, name)
                except Exception:  # noqa: BLE001
                    pass
            return {"failed": f"timeout: no result after {self.timeout_s:g} s (wall-clock guard)"}
        if "e" in box:
            return {"failed": box["e"]}
        return box["r"]


def _device(backend: str):
    import torch

    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def combine_counts(nodes: int, leaves: int, depth: int, world: int, backend: str = "nccl"):
    """Sum nodes/leaves and max depth over ranks (the final UTS reduction)."""
    if world == 1:
        return nodes, leaves, depth
    import torch
    import torch.distributed as dist

    dev = _device(backend)
    t = torch.tensor([nodes, leaves], dtype=torch.int64, device=dev)
    d = torch.tensor([depth], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(d, op=dist.ReduceOp.MAX)
    return int(t[0]), int(t[1]), int(d[0])


def max_over_ranks(x: float, world: int, backend: str = "nccl") -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=_device(backend))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def gather_floats(x: float, world: int, backend: str = "nccl"):
    """Every rank's value of x, in rank order (all_gather)."""
    if world == 1:
        return [float(x)]
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=_device(backend))
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(o[0]) for o in out]


def describe(world: int, backend: str) -> dict:
    """What the collective layer is: world size and backend as the process
    group reports them (RCCL is torch's "nccl" backend on ROCm)."""
    if world == 1:
        return {"world_size": 1, "backend": None}
    import torch.distributed as dist

    be = dist.get_backend()
    return {"world_size": dist.get_world_size(), "backend": "rccl" if be == "nccl" else be}


def barrier(world: int, backend: str = "nccl") -> None:
    import torch

    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def shutdown(world: int) -> None:
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


# ------------------------------------------------------------------ SW bands
# Smith-Waterman sharded by tile columns. Rank r owns
# the contiguous band of tile columns sw_bands(ntw, world)[r] and runs it in
# blocks of tile rows (sw_blocks). Its only input from another rank is the
# left band's right column (the reference's right_column promises of tile
# column j0-1 and their bottom-right corners, smith_waterman.cpp:212-226),
# which arrives per block as one point-to-point message; it sends its own
# right column on to rank r+1 the same way. Block b of rank r therefore
# overlaps block b+1 of rank r-1 (a software pipeline over the ranks). Over
# RCCL every step is stream-ordered (recv -> kernel -> send on the device,
# the host never waits); over gloo (CPU tests, shared-device rehearsals) the
# messages are staged through host memory.


def sw_bands(ntw: int, world: int):
    """Contiguous tile-column bands [(j0, j1)] for each rank (ntw >= world)."""
    if ntw < world:
        raise ValueError(f"{ntw} tile columns cannot be split over {world} ranks")
    return [(r * ntw // world, (r + 1) * ntw // world) for r in range(world)]


def sw_blocks(nth: int, block_rows: int):
    """Tile-row blocks [(i0, i1)] exchanged as one message each."""
    if block_rows < 1:
        raise ValueError("block_rows must be >= 1")
    return [(i, min(nth, i + block_rows)) for i in range(0, nth, block_rows)]


def sw_block_rows(ntw: int, nth: int, world: int) -> int:
    """Rows per exchanged block. With band width W = ntw/world tiles, a block
    of K tile rows has a span of K + W - 1 tiles and the pipeline runs
    nth/K + world - 1 block steps, so the span is minimised near
    K = sqrt((W - 1) * nth / (world - 1))."""
    if world <= 1:
        return nth
    w = max(1, ntw // world)
    k = int(round(((w - 1) * nth / (world - 1)) ** 0.5))
    return max(1, min(nth, k))


class _HipBand:
    """A band on the GPU through hclib_hip_sw_band_* (the C-ABI)."""

    def __init__(self, s1, s2, tw, th, j0, j1):
        import torch

        from . import SwBand

        self.band = SwBand(s1, s2, tw, th, j0, j1)
        self.torch_stream = torch.cuda.current_stream()
        self.stream = self.torch_stream.cuda_stream

    def rows(self, i0, i1, left, right):
        self.band.rows(i0, i1, None if left is None else left.data_ptr(),
                       None if right is None else right.data_ptr(), self.stream)

    def end(self):
        return self.band.end(self.stream)


class ExchangeAborted(RuntimeError):
    """Another rank gave up on the column exchange (sw_exchange)."""


class ShardedSw:
    """One rank's share of a sharded SW run. __init__ uploads the band
    (outside any timed region); run() executes the pipeline once and
    returns (score, tiles over all ranks). `band_factory(s1, s2, tw, th, j0,
    j1)` defaults to the HIP band; the CPU tests pass a host DP band.
    `group` (default: the world group) carries the exchange; `backend` is
    that group's backend ("gloo" stages the columns through host memory).
    `abort` (optional, () -> reason or None) is polled while this rank waits
    on the exchange: a peer that failed sets it (sw_exchange), and the wait
    ends with ExchangeAborted instead of blocking until the group's timeout.
    `inject` (tests only) is called before each receive."""

    def __init__(self, s1: bytes, s2: bytes, tw: int, th: int, rank: int, world: int,
                 backend: str = "nccl", block_rows: int = 16, band_factory=None, device=None,
                 group=None, abort=None, inject=None):
        import torch

        self.rank, self.world, self.backend, self.group = rank, world, backend, group
        self.abort, self.inject = abort, inject
        self.th = th
        ntw, nth = len(s1) // tw, len(s2) // th
        self.j0, self.j1 = sw_bands(ntw, world)[rank]
        self.blocks = sw_blocks(nth, block_rows)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        n = nth * th
        self.left = torch.empty(n, dtype=torch.int32, device=device) if rank > 0 else None
        self.right = torch.empty(n, dtype=torch.int32, device=device) if rank < world - 1 else None
        self.band = (band_factory or _HipBand)(s1, s2, tw, th, self.j0, self.j1)

    def _wait(self, work):
        """Host wait on a gloo transfer, bounded by the peers: polls the
        transfer and `abort` instead of blocking in work.wait()."""
        if self.abort is None:
            work.wait()
            return
        # gloo's send/recv works complete only inside wait(): it runs on a
        # helper thread while this one polls `abort` (an aborted wait is left
        # behind on its daemon thread)
        box = {}

        def waiter():
            try:
                work.wait()
            except BaseException as e:  # noqa: BLE001 (re-raised on the caller's thread)
                box["e"] = e
        th = threading.Thread(target=waiter, daemon=True)
        th.start()
        th.join(0.002)
        while th.is_alive():
            why = self.abort()
            if why:
                raise ExchangeAborted(why)
            th.join(0.0005)
        if "e" in box:
            raise box["e"]

    def _recv(self, t):
        import torch
        import torch.distributed as dist

        if self.inject is not None:
            self.inject()
        if self.backend == "nccl":
            dist.recv(t, src=self.rank - 1, group=self.group)  # stream-ordered: the host does not wait
        elif t.device.type == "cpu":
            self._wait(dist.irecv(t, src=self.rank - 1, group=self.group))
        else:  # gloo carries host tensors only
            h = torch.empty_like(t, device="cpu")
            self._wait(dist.irecv(h, src=self.rank - 1, group=self.group))
            t.copy_(h)

    def _send(self, t):
        import torch.distributed as dist

        if self.backend == "nccl":
            dist.send(t, dst=self.rank + 1, group=self.group)
        else:
            self._wait(dist.isend(t if t.device.type == "cpu" else t.cpu(), dst=self.rank + 1, group=self.group))

    def _drain(self):
        """RCCL: the host waits for the band's stream (kernels, sends, receives)
        by polling an event and `abort`, so a peer's failure ends the wait."""
        import time

        import torch

        if self.abort is None or self.backend != "nccl":
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        while not ev.query():
            why = self.abort()
            if why:
                raise ExchangeAborted(why)
            time.sleep(0.0005)

    def run(self):
        import contextlib

        import torch

        th = self.th
        # the received column's copy, the band launch and the send's read all
        # run on the stream the band was built on, whatever stream is current
        # when run() is called
        ts = getattr(self.band, "torch_stream", None)
        ctx = torch.cuda.stream(ts) if ts is not None else contextlib.nullcontext()
        with ctx:
            for i0, i1 in self.blocks:
                if self.left is not None:
                    self._recv(self.left[i0 * th:i1 * th])
                self.band.rows(i0, i1, self.left, self.right)
                if self.right is not None:
                    self._send(self.right[i0 * th:i1 * th])
            self._drain()
            corner, tiles = self.band.end()
        if self.world == 1:
            return corner, tiles
        import torch.distributed as dist

        dev = _device(self.backend)
        sc = torch.tensor([corner if self.rank == self.world - 1 else 0], dtype=torch.int64, device=dev)
        tt = torch.tensor([tiles], dtype=torch.int64, device=dev)
        if self.backend == "nccl":
            dist.broadcast(sc, src=self.world - 1, group=self.group)
            dist.all_reduce(tt, op=dist.ReduceOp.SUM, group=self.group)
            self._drain()  # a peer that failed ends this wait too
        else:
            self._wait(dist.broadcast(sc, src=self.world - 1, group=self.group, async_op=True))
            self._wait(dist.all_reduce(tt, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        return int(sc[0]), int(tt[0])


def sw_exchange(make_job, rank: int, world: int, backend: str, expected, steps: int = 2, store=None,
                key: str = "hclib_sw_x"):
    """Measure a sharded SW run (best of `steps`, ms over the slowest rank)
    with its column exchange on `backend`, falling back to gloo TOGETHER if
    any rank's attempt fails.

    make_job(backend, group, abort) -> ShardedSw; `expected` = its run()'s
    (score, tiles). Each attempt's exchange runs on a group of its own (a
    failed RCCL one is aborted before the gloo attempt). Everything that decides or
    times lives on a gloo control group created here (never on an RCCL group
    an error may have aborted): the barriers around each run, the max over
    ranks, and the agreement after the attempt. A rank whose attempt raises
    sets `key` in the rendezvous store; the others' exchange waits poll that
    key (ShardedSw `abort`) and stop within milliseconds. Every rank then
    meets on the control group, and if any failed all re-measure over a
    fresh gloo exchange group. Returns {"ms", "exchange", "fallback"?} or
    {"failed": reason} when the gloo attempt fails as well."""
    import time

    import torch
    import torch.distributed as dist

    if store is None:
        store = dist.distributed_c10d._get_default_store()
    ctrl = dist.new_group(backend="gloo")  # collective: every rank, same order

    def abort_of(k):
        def check():
            try:
                if store.check([k]):
                    return store.get(k).decode(errors="replace")
            except Exception:  # noqa: BLE001 (a store we cannot read never aborts)
                return None
            return None
        return check

    def maxr(x):
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl)
        return float(t[0])

    def attempt(xb, k):
        group = dist.new_group(backend=xb)  # collective; a fresh group per attempt
        err = None
        best = None

        def fail(e):
            nonlocal err
            err = f"rank {rank}: {type(e).__name__}: {str(e)[:200]}"
            if not isinstance(e, ExchangeAborted):
                try:
                    store.set(k, err)
                except Exception:  # noqa: BLE001
                    pass

        def agreed_ok():
            # the one collective every rank reaches at every point below, so a
            # rank that failed anywhere and a rank that did not issue the same
            # collective on ctrl (a failed rank never sits in a barrier while
            # its peer is in an all-reduce); it doubles as the barrier
            return maxr(1.0 if (err or abort_of(k)()) else 0.0) == 0.0

        ok = True
        for _ in range(steps):
            job = None
            try:
                job = make_job(xb, group, abort_of(k))
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001 (agreed on at once, below)
                fail(e)
            if not agreed_ok():
                ok = False
                break
            t0 = time.perf_counter()
            try:
                score, tiles = job.run()
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3
                if (score, tiles) != tuple(expected):
                    raise RuntimeError(f"mismatch: score {score}, tiles {tiles}, want {tuple(expected)}")
                best = ms if best is None else min(best, ms)
            except Exception as e:  # noqa: BLE001
                fail(e)
            if not agreed_ok():
                ok = False
                break
        if not ok:
            if xb == "nccl":
                # kernels of the failed exchange may still wait on the band's
                # stream: abort the communicator so they end (best effort)
                try:
                    dist.distributed_c10d._abort_process_group(group)
                except Exception:  # noqa: BLE001
                    pass
            return None, abort_of(k)() or err or "failed on another rank"
        return maxr(best), None

    ms, why = attempt(backend, key)
    out = {"exchange": backend}
    if why is None:
        out["ms"] = ms
        return out
    out["fallback"] = f"{backend} exchange failed ({why}); measured over gloo on every rank"
    ms2, why2 = attempt("gloo", key + "_fallback")
    if why2 is not None:
        return {"failed": f"{out['fallback']}; gloo also failed: {why2}", "exchange": "gloo"}
    out.update({"ms": ms2, "exchange": "gloo"})
    return out


class GlobalPool:
    """Cross-GPU work sharing for sharded UTS searches:
    one region in rank 0's HBM (hclib_hip_global_*), mapped into every other
    rank's process over IPC; a rank's sharded searches then take chunks from
    / export chunks to it, and every rank's launch ends when no rank holds
    work. Collective: every rank constructs it, calls reset() before each
    sharded search (rank 0 re-initialises the region between two barriers)
    and close() at the end. `group` carries the handle and the barriers
    (default: the world group)."""

    def __init__(self, rank: int, world: int, backend: str = "nccl", cap: int = 1024, group=None):
        import torch.distributed as dist

        import hclib_amd as H

        self.rank, self.world, self.cap, self.group = rank, world, cap, group
        self.backend = backend
        self._buf = None
        self._imported = None
        # every rank takes part in the one broadcast whatever happens on rank
        # 0 (a failed allocation or export sends None and every rank raises),
        # so a caller's next collective is the same on all ranks
        # The region is uncached device memory when the driver grants it and
        # IPC exports it (every access from any GPU then reaches rank 0's
        # HBM), else fine-grained, else plain device memory; `mem_kind` says
        # which (HCLIB_GLOBAL_MEM picks one).
        handle = [None]
        self.mem_kind = None
        if rank == 0:
            errs = []
            kinds = [os.environ["HCLIB_GLOBAL_MEM"]] if os.environ.get("HCLIB_GLOBAL_MEM") else \
                ["uncached", "fine", "device"]
            for kind in kinds:
                p = None
                try:
                    p = H.global_alloc(cap, kind)
                    handle = [(H.ipc_export(p), kind)]
                    self._buf, self.ptr, self.mem_kind = p, p, kind
                    break
                except Exception as e:  # noqa: BLE001 (re-raised below, after the broadcast)
                    errs.append(f"{kind}: {e}")
                    if p:
                        H.global_free(p)
            if handle[0] is None:
                self._err = "; ".join(errs)
        if world > 1:
            dist.broadcast_object_list(handle, src=0, group=group)
        if handle[0] is None:
            raise H.HclibError(f"cross-GPU region setup failed on rank 0: {getattr(self, '_err', '')}")
        if rank != 0:
            self._imported = H.ipc_import(handle[0][0])
            self.ptr = self._imported
            self.mem_kind = handle[0][1]
        H.global_attach(self.ptr, cap, rank)

    def _barrier(self):
        import torch
        import torch.distributed as dist

        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier(group=self.group)

    def reset(self):
        import hclib_amd as H

        self._barrier()
        if self.rank == 0:
            H.global_init(self.ptr, self.cap, self.world)
        self._barrier()

    def read(self) -> dict:
        import hclib_amd as H

        return H.global_read(self.ptr)

    def close(self):
        import hclib_amd as H

        H.global_attach(None)
        self._barrier()
        if self._imported is not None:
            H.ipc_close(self._imported)
            self._imported = None
        self._barrier()
        if self._buf is not None:
            H.global_free(self._buf)
            self._buf = None
