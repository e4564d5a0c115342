"""Same-box A/B of an 8-shard UTS partition between library builds: T1XL
split 7 (bench.py's N = 8 wide-tree leg) or, with TREE=T3L, T3L split 64
(the headline's partition); per build, every shard's kernel time and the
whole tree's, best of `reps` (development aid).
    python scripts/shard_ab.py reps name=lib.so ...   (SPLIT=d: another split depth)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
import hclib_amd as H
H.init(0)
TREES = {"T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272, 7), "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631, 64)}
args, total, split = TREES[os.environ.get("TREE", "T1XL")]
reps = int(sys.argv[2])
split = int(os.environ.get("SPLIT", str(split)))
shards = [None] * 8
order = list(range(8))[::-1] if os.environ.get("ORDER") == "rev" else list(range(8))
if os.environ.get("WARM", "1") == "1":
    H.uts(args, order[-1], 8, split)  # the first launch of a process runs cold (shard_order.log)
for s in order:
    best = None
    for _ in range(reps):
        r = H.uts(args, s, 8, split)
        best = r["kernel_ms"] if best is None else min(best, r["kernel_ms"])
    shards[s] = (r["nodes"], round(best, 3))
assert sum(n for n, _ in shards) == total
whole = min(H.uts(args)["kernel_ms"] for _ in range(reps))
print(json.dumps({"shards": shards, "whole": round(whole, 3), "feat": H.uts_last_launch()["feat"]}))
'''
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps = int(sys.argv[1])
for a in sys.argv[2:]:
    name, lib = a.split("=", 1)
    env = dict(os.environ, HCLIB_AMD_LIB=lib)
    p = subprocess.run([sys.executable, "-c", CHILD, root, str(reps)], env=env, capture_output=True, text=True,
                       timeout=600)
    if p.returncode:
        print(name, "FAILED", p.stderr[-2000:], flush=True)
        continue
    d = json.loads(p.stdout.strip().splitlines()[-1])
    slow = max(t for _, t in d["shards"])
    print(f"{name} {os.environ.get('TREE', 'T1XL')} split {os.environ.get('SPLIT', 'default')} order {os.environ.get('ORDER', 'fwd')}: whole {d['whole']} ms, "
          f"shards {[t for _, t in d['shards']]} ms, nodes (M) {[round(n / 1e6, 1) for n, _ in d['shards']]}, slowest {slow}, "
          f"projected efficiency {d['whole'] / (8 * slow):.3f}", flush=True)
