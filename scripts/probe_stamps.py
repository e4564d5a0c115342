"""Per-phase cycle shares of a megakernel batch (diagnostic build flag
HCLIB_HIP_STAMPS=1; never quote its run time)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HCLIB_HIP_STAMPS"] = "1"
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
for name, args in [("T3L", "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"), ("T1XL", "-t 1 -a 3 -d 15 -b 4 -r 29"),
                   ("T1", "-t 1 -a 3 -d 10 -b 4 -r 19")]:
    r = H.uts(args)
    c = H.last_sched_counters()
    nb = max(1, c[13])
    print(f"{name}: ms={r['kernel_ms']:.2f} batches={nb} nodes/batch={r['nodes']/nb:.1f} cycles/batch: "
          f"form={c[7]/nb:.0f} process={c[8]/nb:.0f} push={c[4]/nb:.0f} busy={c[9]/nb:.0f} "
          f"spill={c[11]/nb:.0f} idle_total={c[10]:.3e} busy_frac={c[9]/max(1,c[9]+c[10]):.3f}", flush=True)
v, st = H.fib(30)
c = H.last_sched_counters()
nb = max(1, c[13])
print(f"fib30: ms={st['kernel_ms']:.2f} batches={nb} form={c[7]/nb:.0f} process={c[8]/nb:.0f} "
      f"busy={c[9]/nb:.0f} spill={c[11]/nb:.0f}", flush=True)
s1 = H.sw_map(open("tests/golden/sw/string1-huge.txt", "rb").read())[:65536]
s2 = H.sw_map(open("tests/golden/sw/string2-huge.txt", "rb").read())[:65536]
for wpc in ("8", "4", "2"):
    os.environ["HCLIB_HIP_SW_WAVES_PER_CU"] = wpc
    score, st = H.sw(s1, s2, 256, 256)
    print("sw64k wpc", wpc, score, {k: round(v, 3) for k, v in st.items()}, flush=True)
