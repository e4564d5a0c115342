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

import os


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
        if backend == "nccl":
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            if share_device:
                torch.cuda.set_device(dev)
            dist.init_process_group(backend)
    elif backend == "nccl":
        torch.cuda.set_device(dev)
    return rank, world, local


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
