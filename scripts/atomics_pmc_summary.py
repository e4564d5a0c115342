"""Reduce the passes of scripts/pmc_atomics_r05.sh to profiles/atomics_pmc.json
(read by bench.py's `atomics`): per kernel the launches profiled, their
average duration (kernel-trace pass), the counted L2 atomic requests per
launch (TCC_ATOMIC_sum; TCC_EA0_ATOMIC_sum beside it) and their rate against
the calibrated scattered-returning peak. Each workload kernel ran twice
(warm-up + measured); counters are averaged over its launches.
    python scripts/atomics_pmc_summary.py gpurun_out/pmcat profiles/atomics_pmc.json"""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcat"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/atomics_pmc.json"


def one(pattern):
    f = glob.glob(f"{root}/{pattern}", recursive=True)
    if not f:
        raise SystemExit(f"missing {root}/{pattern}")
    return f[0]


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name


# the workload's k_uts_search launches in dispatch order (atomics_pmc_r05.py:
# warm-up + measured launch per tree)
UTS_ORDER = ["T1", "T1", "T1XL", "T1XL"]


def labelled(rows):
    """(label, row) in dispatch order; k_uts_search launches get their tree."""
    n = 0
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        k = short(r["Kernel_Name"])
        if k == "k_uts_search":
            k = f"k_uts_search[{UTS_ORDER[n] if n < len(UTS_ORDER) else n}]"
            n += 1
        yield k, r


def counters(part):
    vals = collections.defaultdict(list)
    for k, r in labelled(list(csv.DictReader(open(one(f"{part}/**/*counter_collection.csv"))))):
        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return vals


dur = collections.defaultdict(list)
for k, r in labelled(list(csv.DictReader(open(one("trace/**/*kernel_trace.csv"))))):
    dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
atom = counters("atomic")
ea = counters("ea")
plain = open(one("plain.log")).read()
res_line = [l for l in plain.splitlines() if l.startswith("RESULT ")]
run = json.loads(res_line[-1][7:]) if res_line else {}
m = re.search(r"fib\(30\): (\d+) of (\d+) scopes in HBM", plain)
hbm_scopes = int(m.group(1)) if m else None

kern = {}
for (k, c), v in atom.items():
    if c != "TCC_ATOMIC_sum" or not k.startswith("k_"):
        continue
    d = dur.get(k, [])
    rec = {"launches_counted": len(v), "tcc_atomic_per_launch": sum(v) / len(v),
           "tcc_ea0_atomic_per_launch": (sum(ea[(k, "TCC_EA0_ATOMIC_sum")]) / len(ea[(k, "TCC_EA0_ATOMIC_sum")])
                                         if ea.get((k, "TCC_EA0_ATOMIC_sum")) else None)}
    if d:
        rec["avg_ns"] = sum(d) / len(d)
        rec["launches_traced"] = len(d)
        rec["tcc_atomic_per_s"] = rec["tcc_atomic_per_launch"] / (rec["avg_ns"] * 1e-9)
    kern[k] = rec
peak = kern.get("k_atomic_scatter_ret64", {}).get("tcc_atomic_per_s")
for k, rec in kern.items():
    if peak and "tcc_atomic_per_s" in rec:
        rec["frac_of_scatter_peak"] = rec["tcc_atomic_per_s"] / peak
res = {"kernels": kern, "workload": run, "peak_scatter_ret64_per_s": peak}
fib = kern.get("k_fib")
if fib and run.get("fib30"):
    checkouts = run["fib30"]["tasks"] - 1  # every task checks out once (the root's is a store)
    res["fib30"] = {
        "algorithmic_checkouts_per_launch": checkouts,
        "counted_l2_atomics_per_launch": fib["tcc_atomic_per_launch"],
        "hbm_scopes": hbm_scopes, "scopes": run["fib30"]["joins"],
        # an HBM scope takes its 2 check-outs as L2 atomics; LDS scopes none
        "lds_checkout_share": (1.0 - 2.0 * hbm_scopes / checkouts) if hbm_scopes is not None else None,
        "l2_atomics_per_checkout": fib["tcc_atomic_per_launch"] / checkouts,
    }
for tree in ("T1", "T1XL"):
    rec = kern.get(f"k_uts_search[{tree}]")
    if rec and run.get(tree):
        rec["nodes"] = run[tree]["nodes"]
        rec["l2_atomics_per_node"] = rec["tcc_atomic_per_launch"] / run[tree]["nodes"]
res["note"] = ("rocprofv3 --pmc TCC_ATOMIC_sum / TCC_EA0_ATOMIC_sum, one counter per pass, and a --kernel-trace "
               "pass of the same workload (scripts/pmc_atomics_r05.sh, scripts/atomics_pmc_r05.py). Counts are "
               "L2 atomic requests: a wave instruction whose lanes hit one 64-B line counts once per line. "
               "The uts kernels' counts include every scheduler atomic (chunk tickets, outstanding, steals).")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
