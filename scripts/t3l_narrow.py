"""How much of T3L's work runs in the narrow-frontier loop: batches and
cycles inside it (hclib_hip_last_narrow_counters) against all batches and
the waves' busy cycles (hclib_hip_last_sched_counters), per launch."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

H.init(0)
T3L = "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"
for wpg in os.environ.get("WPGS", "2,1").split(","):
    os.environ["HCLIB_HIP_WPG"] = wpg
    r = min((H.uts(T3L) for _ in range(3)), key=lambda x: x["kernel_ms"])
    H.uts(T3L)
    nb, ncyc, nin, _ = H.last_narrow_counters()
    sc = H.last_sched_counters()
    print(json.dumps({"wpg": wpg, "kernel_ms": round(r["kernel_ms"], 3), "batches": r.get("batches"),
                      "narrow_batches": nb, "narrow_entries": nin,
                      "narrow_cycles_per_batch": round(ncyc / max(nb, 1), 1),
                      "sched_counters": sc, "stats": {k: v for k, v in r.items() if k not in ("levels",)}}),
          flush=True)
