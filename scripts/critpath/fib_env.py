"""fib(30) under environment settings, interleaved in one process
(development aid): python fib_env.py ROUNDS 'K=V ...' ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import hclib_amd as H  # noqa: E402

H.init(0)
rounds, cfgs = int(sys.argv[1]), sys.argv[2:] or [""]
res = {c: [] for c in cfgs}
for _ in range(rounds):
    for c in cfgs:
        env = dict(kv.split("=", 1) for kv in c.split())
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        best = None
        for _ in range(3):
            v, st = H.fib(30)
            assert v == 832040
            best = st["kernel_ms"] if best is None else min(best, st["kernel_ms"])
        res[c].append(best)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
for c, v in res.items():
    print(f"fib30 [{c or 'default'}] mean {sum(v) / len(v):.4f} min {min(v):.4f} max {max(v):.4f} n {len(v)}", flush=True)
