"""Interleaved A/B of two builds of the library (development aid): each round
runs every workload once per library in a fresh child process, so both see
the same box and clock. Usage: ab_lib.py LIB_A LIB_B [rounds]."""
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
     "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272)}
out = {}
for name, (args, nodes) in T.items():
    ms = []
    for _ in range(3 if name != "T1XL" else 2):
        r = H.uts(args)
        assert r["nodes"] == nodes, (name, r["nodes"])
        ms.append(r["kernel_ms"])
    out[name] = min(ms)
v, st = H.fib(30)
assert v == 832040
out["fib30"] = st["kernel_ms"]
print(json.dumps(out))
'''

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sys.argv[1:3]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
res = {lib: [] for lib in libs}
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, HCLIB_AMD_LIB=os.path.abspath(lib), HX_ROOT=root)
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:], flush=True)
            sys.exit(1)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        res[lib].append(d)
        print(f"round {r} {lib}: " + " ".join(f"{k} {v:.3f}" for k, v in d.items()), flush=True)
for lib in libs:
    best = {k: min(d[k] for d in res[lib]) for k in res[lib][0]}
    print(f"best {lib}: " + " ".join(f"{k} {v:.3f} ms" for k, v in best.items()), flush=True)
