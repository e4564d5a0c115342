"""One-tile-row SW band sweep (scripts/sw_band_sweep.py's probe) for
rocprofv3 --pmc: SW_FORM (default 212) over the 64K s1 string, one launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s1 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string2-huge.txt"), "rb").read())[:256]
os.environ["HCLIB_HIP_SW_FORM"] = os.environ.get("SW_FORM", "212")
H.init(0)
score, st = H.sw(s1, s2, 256, 256)
print("form", os.environ["HCLIB_HIP_SW_FORM"], "ms", st["kernel_ms"], "score", score, flush=True)
