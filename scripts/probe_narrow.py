"""Narrow-frontier carry loop on the span-bound T3L (development aid): how
many batches run in the tight loop and their shader cycles per batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
trees = {"T3L": "-t 0 -b 2000 -q 0.200014 -m 5 -r 7", "T3": "-t 0 -b 2000 -q 0.124875 -m 8 -r 42"}
for name in sys.argv[1:] or ["T3L"]:
    for carry in ("1", "2"):
        os.environ["HCLIB_HIP_CARRY"] = carry
        best = None
        for _ in range(3):
            r = H.uts(trees[name])
            c = H.last_sched_counters()
            nw = H.last_narrow_counters()
            if best is None or r["kernel_ms"] < best[0]["kernel_ms"]:
                best = (r, c, nw)
        r, c, nw = best
        nb = max(1, c[13])
        print(f"{name} carry={carry}: {r['kernel_ms']:.2f} ms, batches {nb}, nodes/batch {r['nodes'] / nb:.1f}, "
              f"narrow batches {nw[0]} ({nw[0] / nb:.1%}), narrow cycles/batch {nw[1] / max(1, nw[0]):.0f}, "
              f"entries {nw[2]}, batches/entry {nw[0] / max(1, nw[2]):.1f}, busy cycles/batch "
              f"{c[9] / nb:.0f}", flush=True)
