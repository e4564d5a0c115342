"""Single-wave / small-grid UTS probes: the pure batch cost without contention."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

T3 = "-t 0 -b 2000 -q 0.124875 -m 8 -r 42"
T1 = "-t 1 -a 3 -d 10 -b 4 -r 19"
T3L = "-t 0 -b 2000 -q 0.200014 -m 5 -r 7"


def show(tag, r):
    c = H.last_sched_counters()
    mhz = 100.0 * c[5] / c[6] if c[6] else 2400.0
    b = max(1, c[13])
    print(f"{tag}: nodes={r['nodes']} ms={r['kernel_ms']:.3f} batches={r['batches']} "
          f"nodes/batch={r['nodes'] / b:.1f} us/batch={r['us_per_batch']:.3f} busy={r['busy_frac']:.3f} "
          f"pushed={r['chunks_pushed']} clock={mhz:.0f} "
          f"form={c[7] / b / mhz:.3f} proc={c[8] / b / mhz:.3f} push={c[4] / b / mhz:.3f}", flush=True)


def main():
    H.init(0)
    for spec in sys.argv[1:]:
        tag, env = spec.split(":", 1) if ":" in spec else (spec, "")
        saved = dict(os.environ)
        for kv in filter(None, env.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        args = {"T3": T3, "T1": T1, "T3L": T3L}[tag]
        show(f"{tag} [{env}]", H.uts(args))
        os.environ.clear()
        os.environ.update(saved)


if __name__ == "__main__":
    main()
