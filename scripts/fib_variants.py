"""fib(30) kernel time for several library builds, alternating in one
process each (HCLIB_AMD_LIB): usage fib_variants.py LIB [LIB ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import os, sys
sys.path.insert(0, %r)
import hclib_amd as H
H.init(0)
ms = []
for _ in range(6):
    v, st = H.fib(30)
    assert v == 832040
    ms.append(round(st["kernel_ms"], 3))
print(os.environ["HCLIB_AMD_LIB"], "fib(30) kernel_ms", ms, flush=True)
''' % ROOT

for rep in range(2):
    for lib in sys.argv[1:]:
        env = dict(os.environ, HCLIB_AMD_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
        print(r.stdout.strip() or r.stderr[-500:], flush=True)
