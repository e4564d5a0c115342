"""Quick GPU timing probe for the hot-path kernels (development aid)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

T1 = "-t 1 -a 3 -d 10 -b 4 -r 19"
T3L = "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"
T1L = "-t 1 -a 3 -d 13 -b 4 -r 29"


def run_uts(name, args, reps=3):
    best = None
    for _ in range(reps):
        r = H.uts(args)
        if best is None or r["kernel_ms"] < best["kernel_ms"]:
            best = r
    print(f"{name}: nodes={best['nodes']} ms={best['kernel_ms']:.3f} "
          f"Mnodes/s={best['nodes'] / best['kernel_ms'] / 1e3:.1f} batches={best['batches']} "
          f"pushed={best['chunks_pushed']} stolen={best['chunks_stolen']} busy={best['busy_frac']:.3f} "
          f"us/batch={best['us_per_batch']:.2f}", flush=True)
    c = H.last_sched_counters()
    if c[6]:
        mhz = 100.0 * c[5] / c[6]
        b = max(1, c[13])
        print(f"   clock={mhz:.0f}MHz form_us/batch={c[7] / b / mhz:.3f} proc_us/batch={c[8] / b / mhz:.3f} "
              f"push_us/batch={c[4] / b / mhz:.3f} spill_us/batch={c[11] / b / mhz:.3f}", flush=True)
    return best


def main():
    H.init(0)
    print("cus", H.num_cus(), flush=True)
    sweep = sys.argv[1:] if len(sys.argv) > 1 else ["base"]
    base_env = dict(os.environ)
    for tag in sweep:
        os.environ.clear()
        os.environ.update(base_env)
        if tag != "base":
            for kv in tag.split(","):
                k, v = kv.split("=")
                os.environ[k] = v
        print("== config", tag, flush=True)
        run_uts("T1", T1)
        run_uts("T3L", T3L, reps=1)
        run_uts("T1L", T1L, reps=1)
    v, st = H.fib(30)
    print("fib30", v, st, "Mtasks/s=%.1f" % (st["tasks"] / st["kernel_ms"] / 1e3), flush=True)
    s1 = H.sw_map(open("tests/golden/sw/string1-huge.txt", "rb").read())[:65536]
    s2 = H.sw_map(open("tests/golden/sw/string2-huge.txt", "rb").read())[:65536]
    score, st = H.sw(s1, s2, 256, 256)
    print("sw64k", score, st, flush=True)
    import torch
    if os.environ.get("PROBE_NO_TRIAD"):
        return
    n = 1 << 28
    b = torch.rand(n, device="cuda"); c = torch.rand(n, device="cuda"); a = torch.empty(n, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(3):
        H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n, s.cuda_stream)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print("triad ms=%.4f GB/s=%.1f" % (ms, 12 * n / ms / 1e6), flush=True)


if __name__ == "__main__":
    main()
