"""Interleaved A/B of library builds on the SW-64K promise DAG (development aid):
python scripts/ab_libs_sw.py hclib_amd/lib/libhclib_amd.so hclib_amd/lib/base/libhclib_amd.so
Each library runs in its own process (best of 6 launches), rounds interleaved."""
import os
import subprocess
import sys

libs = sys.argv[1:]
code = r'''
import os, sys
sys.path.insert(0, os.getcwd())
import hclib_amd as H
G = os.path.join(os.getcwd(), "tests", "golden", "sw")
a = H.sw_map(open(os.path.join(G, "string1-huge.txt"), "rb").read())[:65536]
b = H.sw_map(open(os.path.join(G, "string2-huge.txt"), "rb").read())[:65536]
os.environ["HCLIB_HIP_SW_SCHED"] = "dag"
H.init(0)
best = 1e9
for _ in range(6):
    score, st = H.sw(a, b, 256, 256)
    assert score == 128772
    best = min(best, st["kernel_ms"])
print(f"{best:.3f}")
'''
res = {l: [] for l in libs}
for rnd in range(3):
    for lib in libs:
        env = dict(os.environ, HCLIB_AMD_LIB=lib)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(lib, "failed:", out.stderr[-2000:], flush=True)
            sys.exit(1)
        res[lib].append(float(out.stdout.strip().split()[-1]))
        print(rnd, lib, res[lib][-1], flush=True)
for lib in libs:
    print(f"SW-64K dag {lib}: best {min(res[lib]):.3f} ms, all {res[lib]}", flush=True)
