"""Per-batch SQ counter summary of scripts/pmc_uts.sh output (quad-cycle counters x4)."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcu"
d = collections.defaultdict(float)
for f in glob.glob(f"{root}/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "uts" in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
nb = nn = None
for f in glob.glob(f"{root}/p*.log"):
    t = open(f).read()
    m = re.search(r"batches (\d+)", t)
    if m:
        nb = int(m.group(1))
    m = re.search(r"nodes (\d+)", t)
    if m:
        nn = int(m.group(1))
print(root, "batches", nb, "nodes", nn)
quad = {"SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
        "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"}
for k in sorted(d):
    v = d[k] * (4 if k in quad else 1)
    per_node = f"  per 64 nodes {64 * v / nn:10.1f}" if nn else ""
    print(f"  {k:24s} {v:16.0f}  per batch {v / nb:10.1f}{per_node}" if nb else f"  {k} {v}")
