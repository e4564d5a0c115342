"""A/B of the SW row schedule's bottom-row hand-off: whole row at the end of
a tile (HCLIB_HIP_SW_PROGRESSIVE=0) vs 64-column chunks as they are computed
(=1, default). SW 64K, 256x256 tiles, interleaved runs, min and median."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H.init(0)
s1 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string2-huge.txt"), "rb").read())[:65536]
res = {"0": [], "1": []}
for rep in range(6):
    for v in ("0", "1"):
        os.environ["HCLIB_HIP_SW_PROGRESSIVE"] = v
        score, st = H.sw(s1, s2, 256, 256)
        assert score == 128772, (v, score)
        res[v].append(st["kernel_ms"])
for v, xs in res.items():
    print(f"progressive={v} min {min(xs):.3f} ms median {statistics.median(xs):.3f} ms all {[round(x, 3) for x in xs]}",
          flush=True)
