"""Interleaved A/B of library builds on fib(n) (development aid):
python scripts/ab_libs_fib.py 30 hclib_amd/lib/libhclib_amd.so hclib_amd/lib/fib_base/libhclib_amd.so
Each library runs in its own process (best of 8 launches), rounds interleaved."""
import os
import subprocess
import sys

n, libs = int(sys.argv[1]), sys.argv[2:]
code = r'''
import os, sys
sys.path.insert(0, os.getcwd())
import hclib_amd as H
H.init(0)
n = int(sys.argv[1])
best = 1e9
for _ in range(8):
    v, st = H.fib(n)
    assert st["tasks"] > 0
    best = min(best, st["kernel_ms"])
print(f"{best:.3f}")
'''
res = {l: [] for l in libs}
for rnd in range(3):
    for lib in libs:
        env = dict(os.environ, HCLIB_AMD_LIB=lib)
        out = subprocess.run([sys.executable, "-c", code, str(n)], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(lib, "failed:", out.stderr[-2000:], flush=True)
            sys.exit(1)
        res[lib].append(float(out.stdout.strip().split()[-1]))
        print(rnd, lib, res[lib][-1], flush=True)
for lib in libs:
    print(f"fib({n}) {lib}: best {min(res[lib]):.3f} ms, all {res[lib]}", flush=True)
