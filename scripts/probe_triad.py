"""Sweep the triad kernel variants / grid sizes (development aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import hclib_amd as H  # noqa: E402

H.init(0)
n = 1 << 28
b = torch.rand(n, device="cuda"); c = torch.rand(n, device="cuda"); a = torch.empty(n, device="cuda")
s = torch.cuda.current_stream()
exp = torch.add(b, torch.mul(c, 3.0))
import itertools
VARS = [int(x) for x in os.environ.get("TRIAD_VARS", "7,3,15,11,23,31,39,47").split(",")]
BPCS = [int(x) for x in os.environ.get("TRIAD_BPCS", "1,2,4").split(",")]
for var, bpc in itertools.product(VARS, BPCS):
    if True:
        os.environ["HCLIB_HIP_TRIAD_VARIANT"] = str(var)
        os.environ["HCLIB_HIP_TRIAD_BLOCKS_PER_CU"] = str(bpc)
        for _ in range(3):
            H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        ok = torch.equal(a, exp)
        print(f"variant={var} bpc={bpc} ms={ms:.4f} GB/s={12 * n / ms / 1e6:.1f} ok={ok}", flush=True)
