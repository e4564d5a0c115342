"""Per-batch view of scripts/pmc_uts.sh passes: python scripts/pmc_parse.py <batches>."""
import csv
import glob
import sys

nb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
agg = {}
for f in sorted(glob.glob("gpurun_out/pmcu/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "uts" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:16.0f} {agg[k] / nb:10.1f}/batch")
