"""Run the forasync triad (2^28 fp32) a fixed number of times; used under
rocprofv3 --pmc to measure HBM bytes per launch (scripts/pmc_triad.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import hclib_amd as H  # noqa: E402

H.init(0)
n = 1 << 28
b = torch.rand(n, device="cuda"); c = torch.rand(n, device="cuda"); a = torch.empty(n, device="cuda")
st = torch.cuda.current_stream()
for _ in range(10):
    H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, st.cuda_stream)
torch.cuda.synchronize()
print("ok")
