"""A/B of the SW-64K promise DAG's tile bodies on one box (diagnostic):
    python scripts/sw_pk_ab.py [reps] [pk values...]
Alternates HCLIB_HIP_SW_PK over the values given (default 1 2), `reps` runs
each, and prints every kernel time plus the best / median per value."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "sw")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    vals = sys.argv[2:] or ["1", "2"]
    a = H.sw_map(open(os.path.join(GOLD, "string1-huge.txt"), "rb").read())[:65536]
    b = H.sw_map(open(os.path.join(GOLD, "string2-huge.txt"), "rb").read())[:65536]
    os.environ["HCLIB_HIP_SW_SCHED"] = "dag"
    H.init(0)
    times = {v: [] for v in vals}
    for r in range(reps + 1):
        for v in vals:
            os.environ["HCLIB_HIP_SW_PK"] = v
            score, st = H.sw(a, b, 256, 256)
            assert score == 128772, (v, score)
            if r:
                times[v].append(st["kernel_ms"])
            print(f"pk={v} rep {r} {st['kernel_ms']:.3f} ms", flush=True)
    for v in vals:
        print(f"pk={v}: best {min(times[v]):.3f} median {statistics.median(times[v]):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
