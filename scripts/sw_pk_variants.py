"""SW-64K promise DAG kernel time for several library builds, alternating in
one process each (HCLIB_AMD_LIB): usage sw_pk_variants.py LIB [LIB ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys
sys.path.insert(0, %r)
import hclib_amd as H
from tests.conftest import GOLD
H.init(0)
a = open(os.path.join(GOLD, "sw", "string1-huge.txt"), "rb").read()
b = open(os.path.join(GOLD, "sw", "string2-huge.txt"), "rb").read()
s1, s2 = H.sw_map(a)[:65536], H.sw_map(b)[:65536]
os.environ["HCLIB_HIP_SW_SCHED"] = "dag"
ms = []
for _ in range(4):
    score, st = H.sw(s1, s2, 256, 256)
    ms.append(round(st["kernel_ms"], 3))
print(os.environ["HCLIB_AMD_LIB"], "score", score, "kernel_ms", ms, flush=True)
''' % ROOT

for rep in range(2):
    for lib in sys.argv[1:]:
        env = dict(os.environ, HCLIB_AMD_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
        print(r.stdout.strip() or r.stderr[-500:], flush=True)
