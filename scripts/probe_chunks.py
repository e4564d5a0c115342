"""Chunk traffic per batch on the UTS trees (development aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
for name, args in [("T1XL", "-t 1 -a 3 -d 15 -b 4 -r 29"), ("T1", "-t 1 -a 3 -d 10 -b 4 -r 19"),
                   ("T3L", "-t 0 -b 2000 -q 0.200014 -m 5 -r 7")]:
    for ring in (["512", "1024"] if name == "T1XL" else [""]):
        if ring:
            os.environ["HCLIB_HIP_UTS_RING"] = ring
        r = H.uts(args)
        nb = max(1, r["batches"])
        print(f"{name} ring={ring or 'default'}: ms={r['kernel_ms']:.2f} batches={nb} nodes/batch={r['nodes']/nb:.1f} "
              f"pushed/batch={r['chunks_pushed']/nb:.3f} stolen/batch={r['chunks_stolen']/nb:.3f} "
              f"busy={r['busy_frac']:.3f} us/batch={r['us_per_batch']:.3f}", flush=True)
    os.environ.pop("HCLIB_HIP_UTS_RING", None)
