"""T3L per-depth-band table: for each band of depths,
the tree's width there (nodes per level, from the kernel's own per-level
histogram), and the leading edge's time per level from the diagnostic trace
(HCLIB_HIP_UTS_TRACE=1: per depth the earliest 100 MHz stamp any wave
reached it), in ns and in 2.4 GHz cycles, against the 2,636-cycle one-wave
SHA-1 step (profiles/r02/ub_sha_split.log). Prints one JSON object per band
and a summary line; `--bands N` sets the band width in levels."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--band", type=int, default=1000)
ap.add_argument("--tree", default="-t 0 -b 2000 -q 0.200014 -m 5 -r 7")
a = ap.parse_args()

H.init(0)
levels = 17845
plain = [H.uts(a.tree, max_levels=levels) for _ in range(3)]
width = np.array(plain[0]["levels"], dtype=np.int64)
os.environ["HCLIB_HIP_UTS_TRACE"] = "1"
r = H.uts(a.tree, max_levels=levels)
del os.environ["HCLIB_HIP_UTS_TRACE"]
raw = np.array(r["levels"], dtype=np.uint64)
# depth 0 is not stamped (the root comes from roots(), which counts into
# slot 0 instead): the leading edge starts at depth 1. A stamp is
# (100 MHz time << 17) | worker << 1 | 1 when the batch that reached the
# depth ran in the scheduler's narrow-frontier loop
raw[0] = raw[1]
ok = raw != np.uint64(2 ** 64 - 1)  # unstamped depths keep the 0xff.. fill
depth = int(ok.sum())
narrow = (raw[:depth] & np.uint64(1)).astype(bool)
wid = ((raw[:depth] >> np.uint64(1)) & np.uint64(0xffff)).astype(np.int64)
t = (raw[:depth] >> np.uint64(17)).astype(np.float64)
t = (t - t.min()) * 10.0  # ns
step = np.diff(t)  # step[d] = time from reaching depth d to depth d + 1
ghz = 2.4
print(json.dumps({"tree": a.tree, "plain_ms": [round(p["kernel_ms"], 3) for p in plain],
                  "traced_ms": round(r["kernel_ms"], 3), "depths": depth,
                  "edge_ms": round(t[-1] / 1e6, 3)}), flush=True)
rows = []
for d0 in range(0, depth - 1, a.band):
    d1 = min(d0 + a.band, depth - 1)
    s = step[d0:d1]
    w = width[d0:d1]
    rows.append({"depths": [d0, d1], "nodes_per_level_mean": round(float(w.mean()), 1),
                 "nodes_per_level_max": int(w.max()), "ns_per_level": round(float(s.mean()), 1),
                 "cycles_per_level": round(float(s.mean()) * ghz, 0),
                 "excess_cycles_over_sha": round(float(s.mean()) * ghz - 2636, 0),
                 "band_ms": round(float(s.sum()) / 1e6, 3),
                 "levels_over_2x_sha": int((s * ghz > 2 * 2636).sum())})
    print(json.dumps(rows[-1]), flush=True)
# widths vs step time across all levels: where the excess lives
tot_excess = sum(max(0.0, (q["cycles_per_level"] - 2636)) * (q["depths"][1] - q["depths"][0]) for q in rows)
worst = max(rows, key=lambda q: q["excess_cycles_over_sha"] * (q["depths"][1] - q["depths"][0]))
for lo, hi in [(0, 64), (64, 256), (256, 1024), (1024, 4096), (4096, 10 ** 9)]:
    m = (width[:depth - 1] >= lo) & (width[:depth - 1] < hi)
    if m.any():
        print(json.dumps({"width": [lo, hi], "levels": int(m.sum()), "ns_per_level": round(float(step[m].mean()), 1),
                          "ms": round(float(step[m].sum()) / 1e6, 3)}), flush=True)
# step into depth d + 1 by how depth d + 1 was first reached
nx = narrow[1:depth]
print(json.dumps({"reached_in_narrow_loop": {"levels": int(nx.sum()), "ns_per_level": round(float(step[nx].mean()), 1),
                                             "ms": round(float(step[nx].sum()) / 1e6, 3)},
                  "reached_in_main_loop": {"levels": int((~nx).sum()), "ns_per_level": round(float(step[~nx].mean()), 1),
                                           "ms": round(float(step[~nx].sum()) / 1e6, 3)}}), flush=True)
# the leading edge moving to another worker between consecutive depths
same = wid[1:depth] == wid[:depth - 1]
print(json.dumps({"edge_stays_on_worker": {"levels": int(same.sum()), "ns_per_level": round(float(step[same].mean()), 1),
                                           "ms": round(float(step[same].sum()) / 1e6, 3)},
                  "edge_moves_to_another_worker": {"levels": int((~same).sum()),
                                                   "ns_per_level": round(float(step[~same].mean()), 1),
                                                   "ms": round(float(step[~same].sum()) / 1e6, 3)},
                  "distinct_workers_on_edge": int(len(set(wid[1:depth].tolist())))}), flush=True)
# step-time distribution of the edge's same-worker steps, narrow loop or not
for name, m in (("same_worker_narrow", same & nx), ("same_worker_main", same & ~nx)):
    if m.any():
        q = np.percentile(step[m] * ghz, [10, 50, 90, 99])
        med = float(q[1])
        print(json.dumps({name: {"levels": int(m.sum()), "cycles_p10_p50_p90_p99": [round(float(x)) for x in q],
                                 "ms_above_1p5x_median": round(float(step[m][step[m] * ghz > 1.5 * med].sum()) / 1e6, 3),
                                 "ms_at_median": round(med * int(m.sum()) / ghz / 1e6, 3)}}), flush=True)
print(json.dumps({"summary": True, "excess_ms_total": round(tot_excess / ghz / 1e6, 3),
                  "worst_band": worst["depths"]}), flush=True)
