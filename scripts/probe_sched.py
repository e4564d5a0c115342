"""Scheduler counters of one UTS search (development aid): shader clock (from
s_memtime / s_memrealtime over the waves' lifetimes), batches, narrow-loop
share, chunk hand-offs and what each costs the giving wave."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
trees = {"T3L": "-t 0 -b 2000 -q 0.200014 -m 5 -r 7", "T1XL": "-t 1 -a 3 -d 15 -b 4 -r 19",
         "T1": "-t 1 -a 3 -d 10 -b 4 -r 19"}
for name in sys.argv[1:] or ["T3L"]:
    best = None
    for _ in range(3):
        r = H.uts(trees[name])
        c = H.last_sched_counters()
        nw = H.last_narrow_counters()
        if best is None or r["kernel_ms"] < best[0]["kernel_ms"]:
            best = (r, c, nw)
    r, c, nw = best
    ghz = c[5] / max(1, c[6]) * 0.1
    nb = max(1, c[13])
    nn = nw[0]
    busy = c[9]
    nbusy_other = busy - nw[1]
    print(f"{name}: {r['kernel_ms']:.2f} ms, clock {ghz:.2f} GHz, waves {c[12]}, batches {nb}, "
          f"nodes/batch {r['nodes'] / nb:.1f}", flush=True)
    print(f"  narrow: {nn} batches ({nn / nb:.1%}), {nw[1] / max(1, nn):.0f} cyc/batch, {nw[2]} entries; "
          f"other batches: {nb - nn}, {nbusy_other / max(1, nb - nn):.0f} cyc/batch", flush=True)
    print(f"  chunks pushed {c[14]}, stolen {c[15]}, spill cycles {c[11]} ({c[11] / max(1, c[14]):.0f}/push), "
          f"busy {busy / max(1, c[12]) / (ghz * 1e6):.2f} ms/wave, idle {c[10] / max(1, c[12]) / (ghz * 1e6):.2f} ms/wave",
          flush=True)
    if name == "T3L":
        lv = 17844
        print(f"  per level: {r['kernel_ms'] * 1e3 / lv:.3f} us = {r['kernel_ms'] * 1e6 * ghz / lv:.0f} cycles; "
              f"narrow batch {nw[1] / max(1, nn) / (ghz * 1e3):.3f} us", flush=True)
