"""Main-loop batch phases of the UTS megakernel (diagnostic, `--variant
phases` library: HCLIB_AMD_LIB=hclib_amd/lib/phases/libhclib_amd.so):
cycles per main-loop single batch from the loop top to the pop issued, the
pop's loads landed, the body done and the batch end, and the narrow loop's
cycles per batch beside them."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

TREES = {"T3L": "-t 0 -b 2000 -q 0.200014 -m 5 -r 7", "T1XL": "-t 1 -a 3 -d 15 -b 4 -r 29",
         "T1": "-t 1 -a 3 -d 10 -b 4 -r 19", "T3": "-t 0 -b 2000 -q 0.124875 -m 8 -r 42"}
H.init(0)
for name in sys.argv[1:] or ["T3L", "T1XL"]:
    r = H.uts(TREES[name])
    r = H.uts(TREES[name])
    p = H.last_phase_counters()
    nb, ncyc, nin, _ = H.last_narrow_counters()
    n = max(1, p[0])
    c = H.last_sched_counters()
    print(json.dumps({"tree": name, "kernel_ms": round(r["kernel_ms"], 3), "main_batches": p[0],
                      "cycles_per_main_batch": {"top_to_pop": round(p[1] / n), "pop": round(p[2] / n),
                                                "body": round(p[3] / n), "push_spill": round(p[4] / n),
                                                "of_which_to_push": round(p[5] / n), "of_which_push": round(p[6] / n)},
                      "spill_section_cycles_per_main_batch": round(c[11] / n), "chunks_pushed": r["chunks_pushed"],
                      "narrow_batches": nb, "narrow_cycles_per_batch": round(ncyc / max(1, nb))}), flush=True)
