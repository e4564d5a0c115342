"""Cross-GPU work sharing rehearsal (dist.GlobalPool): N ranks (default 2) on
ONE GPU (gloo, every rank on device 0; the region is mapped into the other
ranks' processes over IPC exactly as on N GPUs). For skewed static
partitions (split depth 1 of T1L, split 64 of T3L, split 2 of T2L) each
sharded search runs once with the static partition only and once sharing
work; the counts must sum to the published tree either way, and rank 0
prints one JSON line per search with per-rank nodes / kernel ms and the
chunks each rank exported / imported.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      --master-port 29541 scripts/rehearse_global.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import hclib_amd as H  # noqa: E402
from hclib_amd import dist as D  # noqa: E402

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "uts_goldens.json")))["published"]
CASES = [c.split(":") for c in os.environ.get("REHEARSE_CASES", "T1L:1,T2L:2,T3L:64").split(",")]


def main():
    rank, world, _ = D.init_from_env("gloo", share_device=True)
    H.init(0)
    pool = D.GlobalPool(rank, world, "gloo")
    ok = True
    for name, split in CASES:
        pub = GOLD[name]
        for shared in (False, True):
            if shared:
                H.global_attach(pool.ptr, pool.cap, rank)
                pool.reset()
            else:
                H.global_attach(None)
                D.barrier(world, "gloo")
            r = H.uts(pub["args"], rank, world, int(split))
            D.barrier(world, "gloo")
            tot = D.combine_counts(r["nodes"], r["leaves"], r["max_depth"], world, "gloo")
            nodes = D.gather_floats(float(r["nodes"]), world, "gloo")
            kms = D.gather_floats(r["kernel_ms"], world, "gloo")
            g = pool.read() if shared else None
            exact = tot == (pub["nodes"], pub["leaves"], pub["depth"])
            ok = ok and exact
            if rank == 0:
                line = {"tree": name, "split": int(split), "ranks": world, "shared": shared, "bit_exact": exact,
                        "region_memory": pool.mem_kind,
                        "nodes_per_rank": [int(n) for n in nodes], "kernel_ms_per_rank": kms}
                if g:
                    line.update({"exported": g["exported"][:world], "imported": g["imported"][:world],
                                 "active_after": g["active"], "queued_after": g["queued"]})
                print(json.dumps(line), flush=True)
    pool.close()
    D.shutdown(world)
    if not ok:
        raise SystemExit("cross-GPU sharing: counts differ from the published tree")


if __name__ == "__main__":
    main()
