"""The chip's UTS SHA-1 issue ceiling (hclib_hip_sha1_calibrate) over chains
per lane x waves per CU: the peak bench.py's `roofline_uts` divides by."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

H.init(0)
for ch, w in ((1, 4), (1, 8), (2, 8), (1, 12), (2, 12), (1, 16)):
    print(f"chains {ch} waves/CU {w:2d}: " + " ".join(f"{H.sha1_calibrate(ch, w, 2000)[0] / 1e9:6.2f}" for _ in range(2))
          + " G SHA-1/s", flush=True)
