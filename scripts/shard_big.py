"""Same-box A/B of the sharded T3L search's big shard (split 64, 8 shards,
the shard holding 110.5 M of 111.3 M nodes) against the whole tree, between
library builds, interleaved; kernel ms best of `reps` (development aid).
    python scripts/shard_big.py reps rounds name=lib.so ..."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import hclib_amd as H
H.init(0)
args = "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"
reps = int(sys.argv[2])
H.uts(args, 1, 8, 64)
big = min(H.uts(args, 1, 8, 64)["kernel_ms"] for _ in range(reps))
feat = H.uts_last_launch()["feat"]
whole = min(H.uts(args)["kernel_ms"] for _ in range(reps))
print(json.dumps({"big": round(big, 3), "whole": round(whole, 3), "feat": feat}))
'''
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps, rounds = int(sys.argv[1]), int(sys.argv[2])
for rnd in range(rounds):
    for a in sys.argv[3:]:
        name, lib = a.split("=", 1)
        env = dict(os.environ, HCLIB_AMD_LIB=lib)
        p = subprocess.run([sys.executable, "-c", CHILD, root, str(reps)], env=env, capture_output=True, text=True,
                           timeout=300)
        if p.returncode:
            print(name, "FAILED", p.stderr[-2000:], flush=True)
            continue
        d = json.loads(p.stdout.strip().splitlines()[-1])
        print(f"round {rnd} {name:8s} big shard {d['big']} ms (feat {d['feat']}), whole {d['whole']} ms, "
              f"excess {d['big'] - d['whole']:+.3f}", flush=True)
