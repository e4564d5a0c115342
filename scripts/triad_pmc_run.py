"""Run the forasync triad (2^28 fp32) a fixed number of times; used under
rocprofv3 --pmc to measure HBM bytes per launch (scripts/pmc_triad.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import hclib_amd as H  # noqa: E402

H.init(0)
n = 1 << 28
# the bench's layout (bench.py measure_triad): one allocation, the three
# arrays staggered by 2 MiB + 4 KiB, so the counters describe the timed launch
pad = 0x201000 // 4
buf = torch.empty(3 * n + 2 * pad, device="cuda")
b, c, a = buf[:n], buf[n + pad:2 * n + pad], buf[2 * n + 2 * pad:3 * n + 2 * pad]
b.copy_(torch.rand(n, device="cuda")); c.copy_(torch.rand(n, device="cuda"))
st = torch.cuda.current_stream()
for _ in range(10):
    H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, st.cuda_stream)
torch.cuda.synchronize()
print("ok")
