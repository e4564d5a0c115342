"""Reduce the rocprofv3 --pmc passes of scripts/pmc_triad.sh to per-launch
HBM bytes for the triad kernel (profiles/triad_pmc.json, read by bench.py).

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3 section):
FETCH_SIZE (KB) reports half the bytes of a 16-B/lane streaming read on
gfx950 -> x2; WRITE_SIZE (KB) is exact for 16-B/lane streaming stores.
TCC_EA0_RDREQ/WRREQ x 64 B is the same tally (cross-check)."""
import collections
import csv
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/triad_pmc.json"
vals = collections.defaultdict(list)
for part in ("fetch/f", "write/w", "req/r"):
    for r in csv.DictReader(open(f"{root}/{part}_counter_collection.csv")):
        if "k_triad_f32" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
n = 1 << 28
algorithmic = 3 * 4 * n
fetch = avg["FETCH_SIZE"] * 1024 * 2
write = avg["WRITE_SIZE"] * 1024
res = {
    "kernel": "k_triad_f32 (hclib_hip_forasync_triad_f32, n=2^28 fp32)",
    "launches": len(vals["FETCH_SIZE"]),
    "algorithmic_bytes_per_launch": algorithmic,
    "hbm_bytes_per_launch": fetch + write,
    "fetch_bytes_corrected": fetch,
    "write_bytes": write,
    "raw_avg": avg,
    "rdreq_x64_x2_plus_wrreq_x64": (avg["TCC_EA0_RDREQ_sum"] * 2 + avg["TCC_EA0_WRREQ_sum"]) * 64,
    "traffic_over_algorithmic": (fetch + write) / algorithmic,
    "correction": "FETCH_SIZE x2 (gfx950 half-count of 16B/lane streaming reads), "
                  "WRITE_SIZE exact; KB -> bytes x1024",
    "source": "scripts/pmc_triad.sh: three separate rocprofv3 --pmc passes",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
