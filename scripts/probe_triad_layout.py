"""Triad kernel time vs the relative placement of a, b, c in HBM (development aid).
One allocation of 3 arrays + padding; b at 0, c at n*4 + off, a at 2*(n*4 + off)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import hclib_amd as H  # noqa: E402

H.init(0)
n = 1 << 28
st = torch.cuda.current_stream()
if os.environ.get("PRE_UTS"):
    for _ in range(3):
        H.uts("-t 0 -b 2000 -q 0.200014 -m 5 -r 7")


VARS = os.environ.get("VARS", "67").split(",")


def run(b, c, a, tag):
    for v in VARS:
        os.environ["HCLIB_HIP_TRIAD_VARIANT"] = v
        run1(b, c, a, f"{tag} v{v}")


def run1(b, c, a, tag):
    for _ in range(3):
        H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, st.cuda_stream)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(20):
        H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, st.cuda_stream)
    e1.record(st); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ok = torch.equal(a, torch.add(b, torch.mul(c, 3.0)))
    print(f"{tag:40s} ms={ms:.4f} GB/s={12*n/ms/1e6:.1f} ok={ok}", flush=True)


g = torch.Generator(device="cuda").manual_seed(1)
b = torch.rand(n, device="cuda", generator=g); c = torch.rand(n, device="cuda", generator=g)
a = torch.empty(n, device="cuda")
print("separate allocs", hex(b.data_ptr()), hex(c.data_ptr()), hex(a.data_ptr()))
run(b, c, a, "separate torch allocations")
del a, b, c
torch.cuda.empty_cache()
OFFS = [int(x, 0) for x in os.environ.get('OFFS', '0,4096,65536,0x100000,0x101000,0x300000').split(',')]
for off in OFFS:
    buf = torch.empty(3 * n + 3 * off // 4 + 64, device="cuda")
    base = 0
    bb = buf[base:base + n]
    cc = buf[base + n + off // 4: base + 2 * n + off // 4]
    aa = buf[base + 2 * n + 2 * off // 4: base + 3 * n + 2 * off // 4]
    bb.copy_(torch.rand(n, device="cuda", generator=g)); cc.copy_(torch.rand(n, device="cuda", generator=g))
    run(bb, cc, aa, f"one buffer, stagger {off} B")
    del buf, aa, bb, cc
    torch.cuda.empty_cache()
