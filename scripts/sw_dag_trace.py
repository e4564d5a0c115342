"""SW-64K promise DAG: one tile's timeline along the critical path (VERDICT r2
item 7). Runs the reference's 3-promise tile program (HCLIB_HIP_SW_SCHED=dag)
on the diagnostic build (HX_TRACE: hclib_amd/lib/trace/, these stamps
only; HCLIB_AMD_LIB may name the heavier stamps build) with the per-task
trace on (hx_dag.h kDagTraceWords: released / started / body done / puts
done, kept, workgroup, releaser), then walks back from the last tile through
the task whose put released each tile. Per hop it splits the time into
  release: releaser's body done -> the counter decrement that released it
  pickup:  released -> the tile's workgroup has its id (kept or ready list)
  body:    started -> every wave of the tile drained
and prints the totals by hop kind (row hop = left neighbour released it,
column hop = up neighbour, diagonal). Build first:
  python -m hclib_amd.build --variant trace"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HCLIB_AMD_LIB", os.path.join(ROOT, "hclib_amd", "lib", "trace", "libhclib_amd.so"))
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "sw_dag_trace.bin")
os.makedirs(os.path.dirname(out), exist_ok=True)
os.environ["HCLIB_HIP_SW_SCHED"] = "dag"
import numpy as np  # noqa: E402
import hclib_amd as H  # noqa: E402

s1 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string2-huge.txt"), "rb").read())[:65536]
plain = []
for _ in range(2):
    score, st = H.sw(s1, s2, 256, 256)
    assert score == 128772
    plain.append(st["kernel_ms"])
os.environ["HCLIB_HIP_DAG_TRACE"] = out
score, st = H.sw(s1, s2, 256, 256)
del os.environ["HCLIB_HIP_DAG_TRACE"]
assert score == 128772
ntw = nth = 256
tr = np.fromfile(out, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
assert tr.shape[0] == ntw * nth
t0 = tr[0, 1]
ns = lambda x: float(x) * 10.0  # 100 MHz ticks -> ns
hops = []
t = ntw * nth - 1


def since_start(t, k):
    """stamp k of task t relative to its start, in ns; None when the build or
    the task's path did not write it (a zero stamp)"""
    return ns(tr[t, k] - tr[t, 1]) if tr[t, k] != 0 else None


while t != 0:
    r = int(tr[t, 6])
    i, j = divmod(t, ntw)
    ri, rj = divmod(r, ntw)
    kind = "row" if (ri, rj) == (i, j - 1) else "col" if (ri, rj) == (i - 1, j) else "diag"
    hops.append({"t": t, "kind": kind, "kept": int(tr[t, 4]),
                 "release": ns(tr[t, 0] - tr[r, 2]), "pickup": ns(tr[t, 1] - tr[t, 0]),
                 "body": ns(tr[t, 2] - tr[t, 1]),
                 # the task's own put done (an early put, hx_dag.h kEarlyPut, lands
                 # before the body's barrier: negative)
                 "put": ns(tr[t, 3] - tr[t, 2]) if tr[t, 3] != 0 else None,
                 # inside the body, from its start: inputs staged, first scores
                 # there (loop start), sweep done, outputs issued
                 "in_ingress": since_start(t, 8), "in_w0_loop": since_start(t, 12),
                 "in_wave0": since_start(t, 10), "in_egress": since_start(t, 11),
                 "in_entered": since_start(t, 14), "in_loaded": since_start(t, 15),
                 # where the inputs came from (sw.hip trace word 13)
                 "top_lds": int(tr[t, 13]) & 1, "top_mem": (int(tr[t, 13]) >> 1) & 1,
                 "left_mem": (int(tr[t, 13]) >> 2) & 1, "corner_mem": (int(tr[t, 13]) >> 3) & 1})
    t = r
hops.reverse()
total = ns(tr[ntw * nth - 1, 2] - t0)
res = {"plain_ms": plain, "traced_ms": st["kernel_ms"], "critical_hops": len(hops),
       "first_start_to_last_body_ms": total / 1e6, "tile0_body_us": ns(tr[0, 2] - tr[0, 1]) / 1e3}
for kind in ("row", "col", "diag", "all"):
    hs = [h for h in hops if kind == "all" or h["kind"] == kind]
    if not hs:
        continue
    res[kind] = {"hops": len(hs), "kept": sum(h["kept"] for h in hs),
                 "top_from_lds": sum(h["top_lds"] for h in hs), "top_from_memory": sum(h["top_mem"] for h in hs),
                 "left_from_memory": sum(h["left_mem"] for h in hs),
                 "corner_from_memory": sum(h["corner_mem"] for h in hs)}
    for k in ("release", "pickup", "body", "put", "in_entered", "in_loaded", "in_ingress", "in_w0_loop", "in_wave0",
              "in_egress"):
        v = [h[k] for h in hs if h[k] is not None]
        res[kind][k + "_us"] = round(float(np.mean(v)) / 1e3, 3) if v else None
        res[kind][k + "_ms_total"] = round(float(np.sum(v)) / 1e6, 3) if v else None
    # per hop, the time that is not the sweep: release + pickup + body - sweep
    sweep = [h["in_wave0"] - h["in_w0_loop"] for h in hs if h["in_wave0"] is not None and h["in_w0_loop"] is not None]
    if sweep:
        res[kind]["sweep_us"] = round(float(np.mean(sweep)) / 1e3, 3)
        res[kind]["non_sweep_per_hop_us"] = round(
            res[kind]["release_us"] + res[kind]["pickup_us"] + res[kind]["body_us"] - res[kind]["sweep_us"], 3)
# every tile (not only the critical path): body and pickup distributions
body = (tr[:, 2] - tr[:, 1]) * 10.0
pick = (tr[1:, 1] - tr[1:, 0]) * 10.0
res["all_tiles"] = {"body_us_median": float(np.median(body)) / 1e3, "body_us_p10": float(np.percentile(body, 10)) / 1e3,
                    "body_us_p90": float(np.percentile(body, 90)) / 1e3,
                    "pickup_us_median": float(np.median(pick)) / 1e3, "kept_frac": float(tr[:, 4].mean())}
print(json.dumps(res, indent=1), flush=True)
