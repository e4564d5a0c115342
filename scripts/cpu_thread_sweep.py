#!/usr/bin/env python3
"""CPU-port thread sweep on UTS T3L: the host-CPU HClib
restatement (oracle/hclib_cpu.c) at 1, 8, 16, 32, 64 and the allowed worker
count, with the box's CPU allotment evidence (bench.cpu_allotment). One JSON
object on stdout; progress on stderr.

    python scripts/cpu_thread_sweep.py [--counts 1,8,16,32,64] [--min-seconds 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="1,8,16,32,64")
    ap.add_argument("--min-seconds", type=float, default=3.0)
    ap.add_argument("--max-threads", type=int, default=256)
    a = ap.parse_args()
    allot = bench.cpu_allotment()
    counts = [int(c) for c in a.counts.split(",") if c]
    if allot["allowed_cpus"] not in counts:
        counts.append(allot["allowed_cpus"])
    counts = sorted({min(c, a.max_threads) for c in counts})
    rows = []
    for t in counts:
        t0 = time.perf_counter()
        v, n, s = bench.cpu_t3l(t, a.min_seconds if t > 1 else 0.0, max_searches=50 if t > 1 else 1)
        rows.append({"threads": t, "nodes_per_s": v, "searches": n, "search_s": s})
        print(f"threads {t:4d}: {v / 1e6:9.1f} M nodes/s ({n} searches, {s:.2f} s; wall "
              f"{time.perf_counter() - t0:.1f} s)", file=sys.stderr, flush=True)
    print(json.dumps({"workload": f"UTS T3L ({bench.T3L}) on oracle/hclib_cpu.c",
                      "cpu_model": bench.cpu_model(), "allotment": allot, "sweep": rows}, indent=1))


if __name__ == "__main__":
    main()
