"""Time the SW 64K config on each schedule (rows / queue / dag). Dev aid."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
g = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "sw")
s1 = H.sw_map(open(os.path.join(g, "string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(g, "string2-huge.txt"), "rb").read())[:65536]
for sch in sys.argv[1:] or ["rows", "queue", "dag"]:
    os.environ["HCLIB_HIP_SW_SCHED"] = sch
    ms = []
    for _ in range(3):
        sc, st = H.sw(s1, s2, 256, 256)
        assert sc == 128772, (sch, sc)
        ms.append(st["kernel_ms"])
    print(f"{sch}: score {sc} best {min(ms):.3f} ms", flush=True)
