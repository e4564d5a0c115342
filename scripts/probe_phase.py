"""Per-phase cycles of a megakernel batch (development aid).

Run with HCLIB_AMD_LIB=hclib_amd/lib/stamps/libhclib_amd.so HCLIB_HIP_STAMPS=1
for the stamped breakdown (never quote the stamped run time)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import hclib_amd as H  # noqa: E402

TREES = {"T1": "-t 1 -a 3 -d 10 -b 4 -r 19", "T3": "-t 0 -b 2000 -q 0.124875 -m 8 -r 42",
         "T3L": "-t 0 -b 2000 -q 0.200014 -m 5 -r 7", "T1L": "-t 1 -a 3 -d 13 -b 4 -r 29"}


def main():
    H.init(0)
    for spec in sys.argv[1:]:
        name, _, env = spec.partition(":")
        saved = dict(os.environ)
        for kv in filter(None, env.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        r = H.uts(TREES[name])
        c = H.last_sched_counters()
        os.environ.clear()
        os.environ.update(saved)
        nb = max(1, c[13])
        mhz = 100.0 * c[5] / c[6] if c[6] else 2400.0
        print(f"{spec}: nodes={r['nodes']} ms={r['kernel_ms']:.3f} batches={nb} nodes/batch={r['nodes']/nb:.1f} "
              f"busy_cyc/batch={c[9]/nb:.0f} form={c[7]/nb:.0f} proc={c[8]/nb:.0f} push={c[4]/nb:.0f} "
              f"spill={c[11]/nb:.0f} pushed={c[14]} stolen={c[15]} clock={mhz:.0f}", flush=True)


if __name__ == "__main__":
    main()
