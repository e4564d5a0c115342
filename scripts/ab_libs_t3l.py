"""Interleaved A/B of library builds on one tree (development aid):
python scripts/ab_libs_t3l.py T3L hclib_amd/lib/libhclib_amd.so hclib_amd/lib/walk0/libhclib_amd.so ...
Each library runs in its own process (best of 5 launches), rounds interleaved."""
import os
import subprocess
import sys

tree, libs = sys.argv[1], sys.argv[2:]
code = r'''
import os, sys
sys.path.insert(0, os.getcwd())
import torch
import hclib_amd as H
sys.path.insert(0, "scripts")
from uts_probe import TREES
H.init(0)
a, n = TREES[sys.argv[1]]
best = 1e9
for _ in range(6):
    r = H.uts(a)
    assert r["nodes"] == n
    best = min(best, r["kernel_ms"])
print(f"{best:.3f}")
'''
res = {l: [] for l in libs}
for rnd in range(3):
    for lib in libs:
        env = dict(os.environ, HCLIB_AMD_LIB=lib)
        out = subprocess.run([sys.executable, "-c", code, tree], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(lib, "FAILED", out.stderr[-2000:], flush=True)
            sys.exit(1)
        res[lib].append(float(out.stdout.strip().splitlines()[-1]))
        print(rnd, lib, res[lib][-1], flush=True)
for lib, v in res.items():
    print(f"{tree} {lib}: best {min(v):.3f} ms, all {v}")
