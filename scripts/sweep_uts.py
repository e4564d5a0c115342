"""Sweep scheduler knobs on one tree (development aid):
python scripts/sweep_uts.py T3L HCLIB_HIP_SPILL_LO=32,96,256 HCLIB_HIP_WAVES_PER_CU=2,4"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

TREES = {"T1": ("-t 1 -a 3 -d 10 -b 4 -r 19", 4130071),
         "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631),
         "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272), "fib30": ("fib", 0),
         "T1L": ("-t 1 -a 3 -d 13 -b 4 -r 29", 102181082)}
tree_arg, _, split_arg = sys.argv[1].partition(":")  # T1XL:7 = bench's 8-way shards at split 7 (slowest)
sys.argv[1] = tree_arg
if sys.argv[1] not in TREES:  # any published tree (tests/golden/uts_goldens.json)
    import json
    pub = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "uts_goldens.json")))
    TREES[sys.argv[1]] = (pub["published"][sys.argv[1]]["args"], pub["published"][sys.argv[1]]["nodes"])
args, nodes = TREES[sys.argv[1]]
knobs = [(k, v.split(",")) for k, v in (a.split("=") for a in sys.argv[2:])]
H.init(0)
for combo in itertools.product(*[v for _, v in knobs]):
    for (k, _), v in zip(knobs, combo):
        os.environ[k] = v
    ms = []
    for _ in range(3):
        if args == "fib":
            v, r = H.fib(30)
            assert v == 832040
        elif split_arg:
            worst, tot = 0.0, 0
            for sh in range(8):
                r = H.uts(args, sh, 8, int(split_arg))
                tot += r["nodes"]
                worst = max(worst, r["kernel_ms"])
            assert tot == nodes
            r = {"kernel_ms": worst}
        else:
            r = H.uts(args)
            assert r["nodes"] == nodes
        ms.append(r["kernel_ms"])
    print(" ".join(f"{k}={v}" for (k, _), v in zip(knobs, combo)), f"best {min(ms):.3f} ms", flush=True)
