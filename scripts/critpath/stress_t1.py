"""Repeat small UTS trees (development aid): count launches whose node /
leaf / depth totals differ from the published ones."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hclib_amd as H  # noqa: E402

pub = json.load(open(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "uts_goldens.json")))["published"]
H.init(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for name in sys.argv[2:] or ["T1", "T3"]:
    p = pub[name]
    bad = []
    for i in range(reps):
        for ml in (0, 64):
            r = H.uts(p["args"], max_levels=ml)
            got = (r["nodes"], r["leaves"], r["max_depth"])
            if got != (p["nodes"], p["leaves"], p["depth"]):
                bad.append((i, ml, got))
    print(json.dumps({"tree": name, "reps": reps, "bad": bad[:10], "nbad": len(bad)}), flush=True)
