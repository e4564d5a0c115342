"""UTS / fib launch probe (development aid): best-of-N kernel time and the
scheduler's own counters per tree, bit-exact checked.
    python scripts/uts_probe.py [T1 T1L T1XL T1XL:7 T3L fib30] [--reps 3]
`T1XL:7` searches every shard of bench's 8-way partition at split 7."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

TREES = {"T1": ("-t 1 -a 3 -d 10 -b 4 -r 19", 4130071), "T1L": ("-t 1 -a 3 -d 13 -b 4 -r 29", 102181082),
         "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272),
         "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631),
         "T3": ("-t 0 -b 2000 -q 0.124875 -m 8 -r 42", 4112897)}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
    if "--reps" in sys.argv:
        args.remove(str(reps))
    H.init(0)
    for name in args or ["T1", "T1L", "T1XL:7", "T3L", "fib30"]:
        if name == "fib30":
            best = None
            for _ in range(reps + 1):
                v, st = H.fib(30)
                assert v == 832040
                best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
            print(f"fib30 {best['kernel_ms']:.3f} ms busy {best['busy_frac']:.2f} pushed {best['chunks_pushed']} "
                  f"stolen {best['chunks_stolen']}", flush=True)
            continue
        tree, _, split = name.partition(":")
        targs, nodes = TREES[tree]
        shards = [(s, 8, int(split)) for s in range(8)] if split else [(0, 1, 0)]
        tot, worst = 0, 0.0
        for shard, nsh, sp in shards:
            best = None
            for _ in range(reps + 1):
                r = H.uts(targs, shard, nsh, sp)
                best = r if best is None or r["kernel_ms"] < best["kernel_ms"] else best
            tot += best["nodes"]
            worst = max(worst, best["kernel_ms"])
            print(f"{tree}{'' if nsh == 1 else f' shard {shard}/{nsh}'} {best['kernel_ms']:.3f} ms "
                  f"{best['nodes'] / best['kernel_ms'] / 1e6:.2f} G nodes/s  nodes/batch "
                  f"{best['nodes'] / max(1, best['batches']):.1f} us/batch {best['us_per_batch']:.2f} "
                  f"busy {best['busy_frac']:.2f} pushed {best['chunks_pushed']} stolen {best['chunks_stolen']}",
                  flush=True)
        assert tot == nodes, (name, tot, nodes)
        if split:
            print(f"{tree} split {split}: slowest shard {worst:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
