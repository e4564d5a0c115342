"""SW-64K promise DAG: the packed-half tile body (HCLIB_HIP_SW_PK=1) against
the int32 band form (0), alternating, same process. usage: sw_pk_ab.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import hclib_amd as H  # noqa: E402
from tests.conftest import GOLD  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    H.init(0)
    a = open(os.path.join(GOLD, "sw", "string1-huge.txt"), "rb").read()
    b = open(os.path.join(GOLD, "sw", "string2-huge.txt"), "rb").read()
    s1, s2 = H.sw_map(a)[:65536], H.sw_map(b)[:65536]
    os.environ["HCLIB_HIP_SW_SCHED"] = "dag"
    for extra in [dict(), {"HCLIB_HIP_SW_PK_WGS_PER_CU": "2"}]:
        for _ in range(reps):
            for pk in ("1", "0"):
                os.environ["HCLIB_HIP_SW_PK"] = pk
                os.environ.update(extra)
                score, st = H.sw(s1, s2, 256, 256)
                for k in extra:
                    del os.environ[k]
                print(f"pk={pk} {extra} score={score} tiles={st['tiles']} kernel_ms={st['kernel_ms']:.3f}", flush=True)


if __name__ == "__main__":
    main()
