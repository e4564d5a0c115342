"""Compact table of t3l_chain.py output lines (development aid)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "error" in d:
        print(d)
        continue
    print(f"[{d['config']}] plain {d['plain_ms']} traced {d['kernel_ms']} chain {d['chain_ms']}")
    for c in ("same_narrow", "same_main_single", "same_main_dual", "moved_sibling", "moved_far"):
        x = d[c]
        if not x.get("levels"):
            continue
        extra = ""
        if "parts_cycles_p50" in x:
            extra = f" parts p50 {x['parts_cycles_p50']} ms {x['parts_ms']} inbox {x['via_inbox']}/{x['stamped']}"
        print(f"  {c:17s} {x['levels']:6d} lv {x['ms']:6.2f} ms p10/50/90/99 {x['cycles_p10_p50_p90_p99']} "
              f"fill {x['mean_fill']}{extra}")
    print("  excess", d["excess_ms_by_category"])
