"""Depth trace of T3L (diagnostic kernel variant, HCLIB_HIP_UTS_TRACE=1):
per depth the earliest time any wave reached it; the step from depth d to
d+1 along the leading edge is the critical path's per-level time. Prints
its distribution (how much of the run the slow steps take)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
T3L = "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"
plain = min(H.uts(T3L)["kernel_ms"] for _ in range(3))
os.environ["HCLIB_HIP_UTS_TRACE"] = "1"
r = H.uts(T3L, max_levels=17845)
t = (np.array(r["levels"], dtype=np.uint64) >> np.uint64(17)).astype(np.float64)  # low bits: worker, narrow
ok = t < 2 ** 46
t = (t[ok] - t[ok].min()) * 10.0  # ns (100 MHz)
d = np.diff(t)
print(f"plain {plain:.2f} ms, traced {r['kernel_ms']:.2f} ms, depths stamped {ok.sum()}, "
      f"leading edge spans {t[-1] / 1e6:.2f} ms", flush=True)
print(f"per-level step: mean {d.mean():.0f} ns, median {np.median(d):.0f} ns", flush=True)
edges = [0, 1000, 1200, 1400, 1600, 2000, 2500, 3000, 4000, 6000, 10000, 20000, 1e9]
for lo, hi in zip(edges[:-1], edges[1:]):
    m = (d >= lo) & (d < hi)
    print(f"  step [{lo:>6.0f}, {hi:>6.0f}) ns: {m.sum():6d} levels, {d[m].sum() / 1e6:7.2f} ms", flush=True)
