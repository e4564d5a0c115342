"""Active-worker timelines of the UTS megakernel (diagnostic; VERDICT r03
item 1). Runs on the `--variant timeline` library (hx_sched.h Timeline):

    HCLIB_AMD_LIB=hclib_amd/lib/timeline/libhclib_amd.so \
        python scripts/uts_timeline.py out.jsonl [T1 T1L T1XL:7]

`T1XL:7` searches every shard of bench's 8-way partition at split depth 7
(bench.py's N=8 wide-tree leg, one shard at a time). For each launch the line
holds: the kernel time, when the workers started (launch ramp), when 10 / 50
/ 90 % of them first held work, when the last work item was finished (the
last busy -> idle), when the workers saw termination and left, and the
active-worker count per time bin. Timeline launches run slower than the
product build by their stores; quote the product build's times.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("HCLIB_HIP_TIMELINE", "2048")
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

TREES = {"T1": ("-t 1 -a 3 -d 10 -b 4 -r 19", 4130071),
         "T1L": ("-t 1 -a 3 -d 13 -b 4 -r 29", 102181082),
         "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272),
         "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631)}


def summarise(tl, kernel_ms, bins=100):
    starts = [e[0] for w in tl for e in w if e[1] == 1]
    t0 = min(starts)
    us = lambda t: (t - t0) / 100.0  # 100 MHz ticks -> us
    first_busy, last_idle, terms, ends = [], [], [], []
    intervals = []
    spills = 0
    for w in tl:
        busy_since = None
        for t, ev, val in w:
            if ev == 2:
                if busy_since is None:
                    busy_since = t
                if not first_busy or len(first_busy) < len(tl):
                    pass
            elif ev == 3 and busy_since is not None:
                intervals.append((us(busy_since), us(t)))
                last_idle.append(us(t))
                busy_since = None
            elif ev == 4:
                spills += 1
            elif ev == 5:
                terms.append(us(t))
            elif ev == 6:
                ends.append(us(t))
        fb = [us(t) for t, ev, _ in w if ev == 2]
        first_busy.append(min(fb) if fb else None)
    held = sorted(x for x in first_busy if x is not None)
    nw = len(tl)
    end = max(ends) if ends else max(last_idle)
    width = end / bins
    curve = [0.0] * bins
    for a, b in intervals:  # worker-time inside each bin / bin width = mean active workers
        i0, i1 = int(a / width), min(bins - 1, int(b / width))
        for i in range(i0, i1 + 1):
            lo, hi = max(a, i * width), min(b, (i + 1) * width)
            if hi > lo:
                curve[i] += (hi - lo) / width
    # chunks given away (spill) and taken (busy from a deque / inbox) per bin,
    # and the chunks queued at each bin's end: queued work with idle workers
    # means discovery is slow; none queued means production is
    gave, took = [0] * bins, [0] * bins
    for w in tl:
        for t, ev, val in w:
            i = min(bins - 1, int(us(t) / width))
            if ev == 4:
                gave[i] += 1
            elif ev == 2 and (val >> 16) in (1, 2, 3, 4):
                took[i] += 1
    # seeding levels: when the first / last worker saw each level complete
    seed = {}
    for w in tl:
        for t, ev, val in w:
            if ev == 8:
                a, b = seed.get(val, (1e18, 0))
                seed[val] = (min(a, us(t)), max(b, us(t)))
    probe = [0, 0, 0, 0]  # probes, empty deques, lost CASes, publish-wait us (each x16)
    for w in tl:
        for t, ev, val in w:
            if ev == 7:
                probe[val >> 16] += 16 * (val & 0xFFFF)
    queued, q = [], 0
    for i in range(bins):
        q += gave[i] - took[i]
        queued.append(q)
    # per worker: termination seen / exit / last busy->idle / the event before termination
    per = []
    for w in tl:
        ev = [(us(t), e, v) for t, e, v in w]
        tt = [t for t, e, _ in ev if e == 5]
        te = [t for t, e, _ in ev if e == 6]
        ti = [t for t, e, _ in ev if e == 3]
        k = next((i for i, (_, e, _) in enumerate(ev) if e == 5), None)
        before = ev[k - 1][1:] if k else None
        per.append([round(tt[0], 2) if tt else None, round(te[0], 2) if te else None,
                    round(ti[-1], 2) if ti else None, before, len(ev)])
    term_sorted = sorted(x[0] for x in per if x[0] is not None)
    tq = lambda f: term_sorted[min(len(term_sorted) - 1, int(f * len(term_sorted)))] if term_sorted else None
    exit_cost = sorted(x[1] - x[0] for x in per if x[0] is not None and x[1] is not None)
    pct = lambda f: held[min(len(held) - 1, int(f * nw))] if len(held) > f * nw else None
    busy_us = sum(b - a for a, b in intervals)
    return {
        "kernel_ms": kernel_ms, "workers": nw, "workers_that_held_work": len(held),
        "start_spread_us": us(max(starts)),
        "first_work_us": {"10%": pct(0.1), "50%": pct(0.5), "90%": pct(0.9)},
        "last_item_done_us": max(last_idle) if last_idle else None,
        "term_seen_us": [min(terms), max(terms)] if terms else None,
        "last_exit_us": end, "busy_worker_us": busy_us, "mean_active": busy_us / end if end else 0,
        "spills": spills, "bin_us": width, "active_per_bin": [round(c, 1) for c in curve],
        "seed_levels_us": {int(k): [round(v[0], 2), round(v[1], 2)] for k, v in sorted(seed.items())},
        "probes": dict(zip(("probes", "empty", "lost_cas", "publish_wait_us"), probe)),
        "gave_per_bin": gave, "took_per_bin": took, "queued_per_bin": queued,
        "term_quantiles_us": {q: tq(q) for q in (0.0, 0.5, 0.9, 0.99, 1.0)},
        "exit_cost_us": {q: exit_cost[min(len(exit_cost) - 1, int(q * len(exit_cost)))] for q in (0.5, 0.9, 1.0)}
        if exit_cost else None,
        "per_worker": per,
    }


def main():
    out = sys.argv[1]
    names = sys.argv[2:] or ["T1", "T1L", "T1XL:7"]
    H.init(0)
    with open(out, "a") as f:
        for name in names:
            if name == "fib30":
                H.fib(30)
                v, st = H.fib(30)
                assert v == 832040
                s = summarise(H.last_timeline(), st["kernel_ms"])
                s.update({"tree": "fib30", "env": {k: v for k, v in os.environ.items() if k.startswith("HCLIB_HIP_")}})
                f.write(json.dumps(s) + "\n")
                print("fib30", f"{st['kernel_ms']:.3f} ms", "held", s["first_work_us"], "done",
                      round(s["last_item_done_us"], 1), "exit", round(s["last_exit_us"], 1), "mean_active",
                      round(s["mean_active"], 1), flush=True)
                continue
            tree, _, split = name.partition(":")
            args, nodes = TREES[tree]
            shards = [(s, 8, int(split)) for s in range(8)] if split else [(0, 1, 0)]
            tot = 0
            for shard, nsh, sp in shards:
                H.uts(args, shard, nsh, sp)  # warm (tables, code)
                r = H.uts(args, shard, nsh, sp)
                tot += r["nodes"]
                s = summarise(H.last_timeline(), r["kernel_ms"])
                s.update({"tree": tree, "shard": shard, "nshards": nsh, "split": sp, "nodes": r["nodes"],
                          "env": {k: v for k, v in os.environ.items() if k.startswith("HCLIB_HIP_")}})
                f.write(json.dumps(s) + "\n")
                f.flush()
                print(tree, shard, f"{r['kernel_ms']:.3f} ms", "start", round(s["start_spread_us"], 1),
                      "held", s["first_work_us"], "done", round(s["last_item_done_us"], 1), "term",
                      s["term_seen_us"], "exit", round(s["last_exit_us"], 1), "mean_active",
                      round(s["mean_active"], 1), "term_q", s["term_quantiles_us"], "exit_cost",
                      s["exit_cost_us"], "probes", s["probes"], flush=True)
            assert tot == nodes, (name, tot, nodes)


if __name__ == "__main__":
    main()
