"""SW 64K timing per schedule (development aid; with the stamps build it also
prints per-phase cycles per tile to stderr)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
s1 = H.sw_map(open("tests/golden/sw/string1-huge.txt", "rb").read())[:65536]
s2 = H.sw_map(open("tests/golden/sw/string2-huge.txt", "rb").read())[:65536]
for sched in (sys.argv[1:] or ["rows", "queue"]):
    os.environ["HCLIB_HIP_SW_SCHED"] = sched
    score, st = H.sw(s1, s2, 256, 256)
    print(sched, score, {k: round(v, 3) for k, v in st.items()}, flush=True)
