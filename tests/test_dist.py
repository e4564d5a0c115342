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
