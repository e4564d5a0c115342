"""Where T3L's critical path spends its time (diagnostic): follows one
deepest root-to-leaf chain (profiles/r05/t3l_chain.bin, written by
scripts/critpath/uts_chain.c) through the product-shaped search
(HCLIB_HIP_UTS_TRACE=2: the kernel flags the chain's nodes and stamps when
and where each ran, uts.hip FEAT 3) and splits the chain's 17,844 levels by
how the step from depth d to d + 1 went: same worker in the narrow loop, same
worker in the main loop (single or dual batch), or the node moved to another
worker (a sibling wave of the workgroup through its LDS inbox, or another
CU through the HBM deques).

    python scripts/critpath/t3l_chain.py ['K=V K=V' ...] > out.jsonl   (CHAIN=path, RUNS, PLAIN)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

T3L = "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"
path = os.environ.get("CHAIN", "profiles/r05/t3l_chain.bin")
chain = np.fromfile(path, dtype=np.uint32)
D = int(chain[0])
H.init(0)
ALL = np.uint64(2 ** 64 - 1)


def analyse(r, raw):
    t = raw[1:D + 1, 0]
    info = raw[1:D + 1, 1]
    give_raw = raw[1:D + 1, 2]
    take_raw = raw[1:D + 1, 3]
    if (t == ALL).any():
        return {"error": "unstamped depths", "missing": int((t == ALL).sum()),
                "first_missing": int(np.argmax(t == ALL)) + 1}
    t = t.astype(np.float64) * 10.0  # ns (100 MHz ticks)
    wid = (info & np.uint64(0xffff)).astype(np.int64)
    narrow = ((info >> np.uint64(16)) & np.uint64(1)).astype(bool)
    dual = ((info >> np.uint64(17)) & np.uint64(1)).astype(bool)
    fill = ((info >> np.uint64(20)) & np.uint64(0x7f)).astype(np.int64)
    step = np.diff(t)  # step[i]: chain node i+1 ran at t[i], its child at t[i+1]
    same = wid[1:] == wid[:-1]
    wpg = int(H.uts_last_launch()["workers_per_group"])
    sib = (~same) & ((wid[1:] // wpg) == (wid[:-1] // wpg))
    far = (~same) & (~sib)
    nx, dx = narrow[1:], dual[1:]
    cats = {"same_narrow": same & nx, "same_main_single": same & ~nx & ~dx, "same_main_dual": same & ~nx & dx,
            "moved_sibling": sib, "moved_far": far}
    out = {"kernel_ms": round(r["kernel_ms"], 3), "chain_ms": round((t[-1] - t[0]) / 1e6, 3)}
    for name, m in cats.items():
        if not m.any():
            out[name] = {"levels": 0}
            continue
        s = step[m] * 2.4  # cycles at 2.4 GHz
        q = np.percentile(s, [10, 50, 90, 99])
        out[name] = {"levels": int(m.sum()), "ms": round(float(step[m].sum()) / 1e6, 3),
                     "cycles_p10_p50_p90_p99": [round(float(x)) for x in q],
                     "mean_fill": round(float(fill[1:][m].mean()), 1)}
    med = float(np.median(step[cats["same_narrow"]])) if cats["same_narrow"].any() else float(np.median(step))
    # a move's parts: creation (the parent ran) -> given away -> taken -> run
    top = np.uint64(1 << 63)
    for name in ("moved_sibling", "moved_far"):
        m = cats[name]
        g = give_raw[1:][m]
        k = take_raw[1:][m]
        ok = (g != ALL) & (k != ALL)
        if not ok.any():
            continue
        tg = (g[ok] & ~top).astype(np.float64) * 10.0
        tk = (k[ok] & ~top).astype(np.float64) * 10.0
        tc = t[:-1][m][ok]
        tr = t[1:][m][ok]
        parts = {"in_giver_ring": tg - tc, "handoff": tk - tg, "taker_to_run": tr - tk}
        out[name]["parts_cycles_p50"] = {p: round(float(np.median(v)) * 2.4) for p, v in parts.items()}
        out[name]["parts_ms"] = {p: round(float(v.sum()) / 1e6, 3) for p, v in parts.items()}
        out[name]["stamped"] = int(ok.sum())
        out[name]["via_inbox"] = int(((g[ok] & top) != 0).sum())
    out["ms_if_every_step_at_narrow_median"] = round(med * (D - 1) / 1e6, 3)
    out["excess_ms_by_category"] = {name: round(float((step[m] - med).sum()) / 1e6, 3) for name, m in cats.items()}
    return out


configs = sys.argv[1:] or [""]
for cfg in configs:
    env = dict(kv.split("=", 1) for kv in cfg.split())
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    plain = [H.uts(T3L)["kernel_ms"] for _ in range(int(os.environ.get("PLAIN", "3")))]
    os.environ["HCLIB_HIP_UTS_TRACE"] = "2"
    os.environ["HCLIB_HIP_UTS_CHAIN"] = os.path.abspath(path)
    for ri in range(int(os.environ.get("RUNS", "1"))):
        r = H.uts(T3L, max_levels=4 * (D + 1))
        raw = np.array(r["levels"], dtype=np.uint64).reshape(-1, 4)
        out = {"config": cfg, "plain_ms": [round(x, 3) for x in plain], "run": ri,
               "nodes_ok": r["nodes"] == 111345631, "launch": H.uts_last_launch()}
        out.update(analyse(r, raw))
        print(json.dumps(out), flush=True)
    del os.environ["HCLIB_HIP_UTS_TRACE"]
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
