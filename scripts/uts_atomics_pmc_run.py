"""Workload for the UTS scheduler's L2-atomic PMC passes
(scripts/pmc_uts_atomics.sh): the scattered-returning-atomic calibration and
one launch each of UTS T3L (span-bound), T1XL (throughput-bound) and T1."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime with the module)
import hclib_amd as H  # noqa: E402

TREES = [("T3L", "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"), ("T1XL", "-t 1 -a 3 -d 15 -b 4 -r 29"),
         ("T1", "-t 1 -a 3 -d 10 -b 4 -r 19")]


def main():
    H.init(0)
    mops, ms = H.atomic_calibrate(H.ATOMIC_SCATTER_RET64, 256)
    print(f"calib scatter_ret64: {mops:.1f} Mops/s ({ms:.3f} ms)", flush=True)
    for name, args in TREES:
        r = H.uts(args)
        print(f"{name}: nodes {r['nodes']} kernel {r['kernel_ms']:.3f} ms batches {r['batches']} "
              f"pushed {r['chunks_pushed']} stolen {r['chunks_stolen']}", flush=True)


if __name__ == "__main__":
    main()
