"""Workload for the L2-atomic PMC passes (scripts/pmc_atomics.sh): the three
calibration shapes (hclib_hip_atomic_calibrate) and one fib(30) megakernel
launch, each printed with its own rate so the counter CSV can be matched to
kernels by name (k_atomic_*, k_fib)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime with the module)
import hclib_amd as H  # noqa: E402


def main():
    H.init(0)
    for mode, name, iters in ((H.ATOMIC_SCATTER_RET64, "scatter_ret64", 256),
                              (H.ATOMIC_HOT_WORD, "hot_word", 256),
                              (H.ATOMIC_COALESCED32, "coalesced32", 256)):
        mops, ms = H.atomic_calibrate(mode, iters)
        print(f"calib {name}: {mops:.1f} Mops/s ({ms:.3f} ms)", flush=True)
    v, st = H.fib(30)
    assert v == 832040
    print(f"fib30: tasks {st['tasks']} joins {st['joins']} kernel {st['kernel_ms']:.3f} ms "
          f"check-out atomics/s {(st['tasks'] - 1) / (st['kernel_ms'] * 1e-3) / 1e6:.1f} M", flush=True)


if __name__ == "__main__":
    main()
