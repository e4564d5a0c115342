"""Triad kernel launches for rocprofv3 kernel-trace comparisons of variants
(env HCLIB_HIP_TRIAD_VARIANT / _BLOCKS_PER_CU); prints event timing too."""
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
for var in os.environ.get("TRIAD_VARS", "3,67,83,131,147").split(","):
    os.environ["HCLIB_HIP_TRIAD_VARIANT"] = var
    for _ in range(3):
        H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
    ts = []
    for _ in range(20):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    ok = torch.equal(a, exp)
    print(f"variant={var} median_ms={ts[10]:.4f} best_ms={ts[0]:.4f} GB/s(median)={12*n/ts[10]/1e6:.1f} ok={ok}", flush=True)
