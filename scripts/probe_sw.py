"""Time the SW-64K schedules (rows = multi-wave tile rows, rows1 = one wave
per tile row, dag = the reference's promise program on the device DAG)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s1 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string2-huge.txt"), "rb").read())[:65536]
for sched in os.environ.get("SW_SCHEDS", "rows,rows1,dag").split(","):
    os.environ["HCLIB_HIP_SW_SCHED"] = sched
    best = None
    for _ in range(int(os.environ.get("SW_REPS", "3"))):
        score, st = H.sw(s1, s2, 256, 256)
        assert score == 128772, (sched, score)
        best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
    print(f"sched={sched} score={score} kernel_ms={best['kernel_ms']:.3f} "
          f"Gcells/s={best['cells_per_s'] / 1e9:.1f} tiles={best['tiles']}", flush=True)
