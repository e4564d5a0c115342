"""Triad variants x workgroups per CU on the bench's staggered layout
(development aid; prints GB/s of 20 back-to-back launches, best of 3)."""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import hclib_amd as H  # noqa: E402

H.init(0)
n = 1 << 28
pad = 0x201000 // 4
buf = torch.empty(3 * n + 2 * pad, device="cuda")
b, c, a = buf[:n], buf[n + pad:2 * n + pad], buf[2 * n + 2 * pad:3 * n + 2 * pad]
b.copy_(torch.rand(n, device="cuda"))
c.copy_(torch.rand(n, device="cuda"))
exp = torch.add(b, torch.mul(c, 3.0))
s = torch.cuda.current_stream()
VARS = [int(x) for x in os.environ.get("TRIAD_VARS", "67,131,3,75,83,99,147,195").split(",")]
BPCS = [int(x) for x in os.environ.get("TRIAD_BPCS", "1,2,3,4").split(",")]
for var, bpc in itertools.product(VARS, BPCS):
    os.environ["HCLIB_HIP_TRIAD_VARIANT"] = str(var)
    os.environ["HCLIB_HIP_TRIAD_BLOCKS_PER_CU"] = str(bpc)
    best = 1e9
    for _ in range(3):
        for _ in range(3):
            H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20)
    ok = torch.equal(a, exp)
    print(f"variant={var} bpc={bpc} ms={best:.4f} GB/s={12 * n / best / 1e6:.1f} frac={12 * n / best / 8e9:.3f} ok={ok}",
          flush=True)
