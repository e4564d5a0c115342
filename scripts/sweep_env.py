"""Interleaved knob sweep (development aid): each setting runs in a fresh
child process, rounds interleaved. Usage: sweep_env.py TREE ROUNDS 'K=V K2=V2' ...
(an empty string = defaults)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["HX_ROOT"])
import torch
import hclib_amd as H
H.init(0)
T = {"T1": ("-t 1 -a 3 -d 10 -b 4 -r 19", 4130071), "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631),
     "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272), "T1L": ("-t 1 -a 3 -d 13 -b 4 -r 29", 102181082),
     "T3": ("-t 0 -b 2000 -q 0.124875 -m 8 -r 42", 4112897)}
args, nodes = T[os.environ["HX_TREE"]]
ms = []
for _ in range(int(os.environ.get("HX_REPS", "3"))):
    r = H.uts(args)
    assert r["nodes"] == nodes, r["nodes"]
    ms.append(r["kernel_ms"])
print(json.dumps(sorted(ms)))
'''
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree, rounds, settings = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
res = {s: [] for s in settings}
for r in range(rounds):
    for s in settings:
        env = dict(os.environ, HX_ROOT=root, HX_TREE=tree)
        for kv in s.split():
            k, v = kv.split("=", 1)
            env[k] = v
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-1500:], flush=True)
            sys.exit(1)
        res[s] += json.loads(p.stdout.strip().splitlines()[-1])
        print(f"round {r} [{s or 'default'}]: {min(res[s]):.3f} ms best so far", flush=True)
for s in settings:
    v = sorted(res[s])
    print(f"{tree} [{s or 'default'}] best {v[0]:.4f} median {v[len(v) // 2]:.4f} mean {sum(v) / len(v):.4f} ms "
          f"({len(v)} launches)", flush=True)
