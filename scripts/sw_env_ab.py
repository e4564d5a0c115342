"""Same-box A/B of environment settings on SW-64K's promise DAG
(HCLIB_HIP_SW_SCHED=dag), interleaved, each setting in a fresh process:
    python scripts/sw_env_ab.py ROUNDS 'K=V ...' 'K=V ...'   (development aid)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
import hclib_amd as H
H.init(0)
os.environ["HCLIB_HIP_SW_SCHED"] = "dag"
s1 = H.sw_map(open(os.path.join(sys.argv[1], "tests/golden/sw/string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(sys.argv[1], "tests/golden/sw/string2-huge.txt"), "rb").read())[:65536]
ms = []
for _ in range(5):
    sc, st = H.sw(s1, s2, 256, 256)
    assert sc == 128772 and st["tiles"] == 65536, (sc, st)
    ms.append(st["kernel_ms"])
print(json.dumps(sorted(ms)))
'''
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rounds, settings = int(sys.argv[1]), sys.argv[2:]
res = {s: [] for s in settings}
for r in range(rounds):
    for s in settings:
        env = dict(os.environ)
        for kv in s.split():
            k, v = kv.split("=", 1)
            env[k] = v
        p = subprocess.run([sys.executable, "-c", CHILD, root], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode:
            print(s, "FAILED", p.stderr[-2000:], flush=True)
            sys.exit(1)
        res[s] += json.loads(p.stdout.strip().splitlines()[-1])
        print(f"round {r} [{s}]: best so far {min(res[s]):.3f} ms", flush=True)
for s in settings:
    v = sorted(res[s])
    print(f"SW-64K dag [{s}] best {v[0]:.3f} median {v[len(v) // 2]:.3f} ms ({len(v)} launches)", flush=True)
