"""A/B of the scheduler's register carry (HCLIB_HIP_CARRY) on UTS and fib:
kernel ms per tree, bit-exact counts. Development aid."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

TREES = {"T1": ("-t 1 -a 3 -d 10 -b 4 -r 19", 4130071), "T3": ("-t 0 -b 2000 -q 0.124875 -m 8 -r 42", 4112897),
         "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631),
         "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272)}

H.init(0)
for carry in sys.argv[1:] or ["0", "1"]:
    os.environ["HCLIB_HIP_CARRY"] = carry
    for name, (args, nodes) in TREES.items():
        ms = []
        for _ in range(3):
            r = H.uts(args)
            assert r["nodes"] == nodes, (name, r["nodes"])
            ms.append(r["kernel_ms"])
        print(f"carry={carry} {name}: {min(ms):.3f} ms  {nodes / min(ms) / 1e6:.1f} M nodes/s", flush=True)
    v, st = H.fib(30)
    assert v == 832040
    print(f"carry={carry} fib30: {st['kernel_ms']:.3f} ms", flush=True)
