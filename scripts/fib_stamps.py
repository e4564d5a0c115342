"""Per-phase cycles of fib(30)'s batches (stamps build; diagnostic only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HCLIB_HIP_STAMPS"] = "1"
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

H.init(0)
for local in ("0", "1"):
    os.environ["HCLIB_HIP_FIB_LOCAL"] = local
    H.fib(30)
    v, st = H.fib(30)
    c = H.last_sched_counters()
    nb = max(1, c[13])
    print(f"fib30 local={local}: ms={st['kernel_ms']:.3f} batches={nb} tasks/batch={st['tasks'] / nb:.1f} "
          f"cycles/batch form={c[7] / nb:.0f} process={c[8] / nb:.0f} push={c[4] / nb:.0f} busy={c[9] / nb:.0f} "
          f"spill={c[11] / nb:.0f} busy_frac={st['busy_frac']:.2f} | check-out cycles/batch={c[2] / nb:.0f} "
          f"climb iterations/batch={c[3] / nb:.2f}", flush=True)
