"""One UTS search under rocprofv3 --pmc (args: tree name, grid; 0 = default)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

TREES = {"T3": "-t 0 -b 2000 -q 0.124875 -m 8 -r 42", "T3L": "-t 0 -b 2000 -q 0.200014 -m 5 -r 7",
         "T1": "-t 1 -a 3 -d 10 -b 4 -r 19", "T1L": "-t 1 -a 3 -d 13 -b 4 -r 29",
         "T1XL": "-t 1 -a 3 -d 15 -b 4 -r 29"}
tree = sys.argv[1] if len(sys.argv) > 1 else "T3"
if len(sys.argv) > 2 and int(sys.argv[2]) > 0:
    os.environ["HCLIB_HIP_GRID"] = sys.argv[2]
H.init(0)
r = H.uts(TREES[tree])
print(tree, "nodes", r["nodes"], "batches", r["batches"], "ms", r["kernel_ms"], flush=True)
