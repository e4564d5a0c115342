"""Per-step cost of the SW band kernel's column sweep, isolated: the row
schedule on ONE tile row (s2 = 256 codes) over the 64K s1 string is a single
workgroup sweeping 65,536 columns, so kernel time / 65,536 is the time per
column step of each form (HCLIB_HIP_SW_FORM = 100 R + 10 S + K / 16); two
and four tile rows add the row-to-row lag. Scores are checked against the
oracle-free invariant that every form agrees."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hclib_amd as H  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s1 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string1-huge.txt"), "rb").read())[:65536]
s2 = H.sw_map(open(os.path.join(ROOT, "tests/golden/sw/string2-huge.txt"), "rb").read())
H.init(0)
for rows in [int(x) for x in os.environ.get("SW_ROWS", "1,2,4").split(",")]:
    ref = None
    for form in os.environ.get("SW_FORMS", "412,212,12,22,411,211").split(","):
        os.environ["HCLIB_HIP_SW_FORM"] = form
        best = None
        for _ in range(3):
            score, st = H.sw(s1, s2[:256 * rows], 256, 256)
            best = st["kernel_ms"] if best is None else min(best, st["kernel_ms"])
        ref = score if ref is None else ref
        # (the HX_SW_EXP timing builds compute wrong scores by design)
        assert score == ref or "swexp" in os.environ.get("HCLIB_AMD_LIB", ""), (form, score, ref)
        print(f"tile rows {rows} form {form:>3}: {best:.3f} ms = {best * 1e6 / 65536:.1f} ns "
              f"= {best * 1e6 / 65536 * 2.4:.0f} cycles per column step (score {score})", flush=True)
