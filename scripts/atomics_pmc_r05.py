"""Workload of the round-5 L2-atomic PMC passes (scripts/pmc_atomics_r05.sh):
the scattered-returning-atomic calibration (the peak the bench divides by),
then one launch each of fib(30), UTS T1 and UTS T1XL, each after an untimed
warm-up launch. Prints the per-launch figures the summary needs (fib's HBM
scope count comes from HCLIB_HIP_FIB_DEBUG on stderr)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime with the module)
import hclib_amd as H  # noqa: E402

TREES = [("T1", "-t 1 -a 3 -d 10 -b 4 -r 19", 4130071), ("T1XL", "-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272)]


def main():
    H.init(0)
    mops, ms = H.atomic_calibrate(H.ATOMIC_SCATTER_RET64, 256)
    out = {"calib_scatter_ret64_mops": mops}
    H.fib(30)
    v, st = H.fib(30)
    assert v == 832040
    out["fib30"] = {"tasks": st["tasks"], "joins": st["joins"], "kernel_ms": st["kernel_ms"]}
    for name, args, nodes in TREES:
        H.uts(args)
        r = H.uts(args)
        assert r["nodes"] == nodes
        out[name] = {"nodes": nodes, "kernel_ms": r["kernel_ms"], "chunks_pushed": r["chunks_pushed"],
                     "chunks_stolen": r["chunks_stolen"], "batches": r["batches"]}
    print("RESULT " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
