"""Per-phase cycles of a GEO (T1XL) batch at 4 and 8 waves per CU (stamps build:
HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so; never quote its run time)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HCLIB_HIP_STAMPS"] = "1"
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
for wpc in ("4", "8"):
    os.environ["HCLIB_HIP_WAVES_PER_CU"] = wpc
    for name, args in [("T1XL", "-t 1 -a 3 -d 15 -b 4 -r 29"), ("T3L", "-t 0 -b 2000 -q 0.200014 -m 5 -r 7")]:
        r = H.uts(args)
        c = H.last_sched_counters()
        nb = max(1, c[13])
        print(f"wpc={wpc} {name}: ms={r['kernel_ms']:.2f} nodes/batch={r['nodes']/nb:.1f} cycles/batch: "
              f"form={c[7]/nb:.0f} process={c[8]/nb:.0f} push={c[4]/nb:.0f} busy={c[9]/nb:.0f} "
              f"spill={c[11]/nb:.0f} busy_frac={c[9]/max(1,c[9]+c[10]):.3f}", flush=True)
