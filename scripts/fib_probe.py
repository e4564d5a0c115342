"""fib(30) on the device: launch times and scheduler statistics (busy
fraction, chunks pushed / stolen) over repeated launches, and the same with
env knobs (development aid): python scripts/fib_probe.py [KNOB=v1,v2 ...]"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

H.init(0)
knobs = [(k, v.split(",")) for k, v in (a.split("=") for a in sys.argv[1:])]
for combo in itertools.product(*[v for _, v in knobs]) if knobs else [()]:
    for (k, _), v in zip(knobs, combo):
        os.environ[k] = v
    runs = []
    for _ in range(5):
        v, st = H.fib(30)
        assert v == 832040
        runs.append(st)
    best = min(runs, key=lambda r: r["kernel_ms"])
    print(json.dumps({"knobs": dict(zip([k for k, _ in knobs], combo)),
                      "ms": [round(r["kernel_ms"], 3) for r in runs],
                      "busy_frac": round(best["busy_frac"], 3), "tasks": best["tasks"],
                      "chunks_pushed": best["chunks_pushed"], "chunks_stolen": best["chunks_stolen"]}), flush=True)
