"""Batch fill of the UTS megakernel (diagnostic): nodes per batch, busy / idle / spill cycles per tree (H.last_sched_counters)."""
import sys, os, json
sys.path.insert(0, os.getcwd())
import torch  # noqa
import hclib_amd as H
H.init(0)
T = {"T1": "-t 1 -a 3 -d 10 -b 4 -r 19", "T1L": "-t 1 -a 3 -d 13 -b 4 -r 29", "T1XL": "-t 1 -a 3 -d 15 -b 4 -r 29", "T3L": "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"}
for name, a in T.items():
    for _ in range(2):
        r = H.uts(a)
    c = H.last_sched_counters()
    waves = c[12]; b = c[13]
    print(json.dumps({"tree": name, "ms": round(r["kernel_ms"], 3), "nodes": r["nodes"], "batches": int(b), "waves": int(waves),
                      "nodes_per_batch": round(r["nodes"] / max(1, b), 2), "busy": int(c[9]), "idle": int(c[10]), "spill": int(c[11]),
                      "pushed": int(c[14]), "stolen": int(c[15])}), flush=True)
