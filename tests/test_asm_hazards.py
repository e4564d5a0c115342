"""Inline-asm wide stores must carry their own wait states.

A VMEM store of more than 8 bytes (dwordx3 / dwordx4) reads its data VGPRs
after it issues. The compiler's hazard recognizer inserts the wait states
that protect those registers from a following VALU write only for stores it
generated itself; it cannot see inside an inline-asm string. Round 5 shipped
exactly that bug: the next store's address was built in the data registers
of a 16-byte hand-off store, and UTS T1 lost or duplicated nodes in 42 of 60
launches (hx_common.h st_sc1_x4). The rule: inside one asm
statement, every global/buffer/flat store of dwordx3 or dwordx4 is followed
at once by `s_nop N` with N >= 1 (the hazard needs 1 wait state on
gfx950; st_sc1_x4 keeps 3). This test scans the product's device sources
(include/hclib_hip, hclib_amd/csrc) and fails on any statement that breaks it.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCAN = [os.path.join(ROOT, "include", "hclib_hip"), os.path.join(ROOT, "hclib_amd", "csrc"),
        os.path.join(ROOT, "include")]
WIDE_STORE = re.compile(r"\b(global|buffer|flat)_store_dwordx[34]\b")
NOP = re.compile(r"^s_nop\s+(0x[0-9a-fA-F]+|\d+)$")
ASM = re.compile(r"\b(?:asm|__asm__)\s*(?:volatile|__volatile__)?\s*\(")
STR = re.compile(r'\s*"((?:[^"\\]|\\.)*)"')


def asm_statements(text):
    """(line, template) for every asm statement: its adjacent string literals
    joined, escapes for newline and tab decoded."""
    out = []
    for m in ASM.finditer(text):
        pos, parts = m.end(), []
        while True:
            s = STR.match(text, pos)
            if not s:
                break
            parts.append(s.group(1))
            pos = s.end()
        tmpl = "".join(parts).replace("\\n", "\n").replace("\\t", "\t").replace("\\\"", "\"")
        out.append((text.count("\n", 0, m.start()) + 1, tmpl))
    return out


def violations(text, name="<text>"):
    bad = []
    for line, tmpl in asm_statements(text):
        insts = [i.strip() for i in re.split(r"[\n;]", tmpl) if i.strip()]
        for k, ins in enumerate(insts):
            if WIDE_STORE.search(ins):
                nxt = insts[k + 1] if k + 1 < len(insts) else ""
                m = NOP.match(nxt)
                if not m or int(m.group(1), 0) < 1:
                    bad.append(f"{name}:{line}: '{ins}' is not followed by s_nop >= 1 in the same asm statement")
    return bad


def _sources():
    seen = set()
    for d in SCAN:
        for dp, _, fs in os.walk(d):
            for f in fs:
                p = os.path.join(dp, f)
                if p not in seen and f.endswith((".h", ".hip", ".cpp", ".hpp")):
                    seen.add(p)
                    yield p


def test_every_inline_asm_wide_store_has_its_wait_states():
    bad, stores = [], 0
    for p in _sources():
        text = open(p, encoding="utf-8", errors="replace").read()
        stores += sum(len(WIDE_STORE.findall(t)) for _, t in asm_statements(text))
        bad += violations(text, os.path.relpath(p, ROOT))
    assert stores >= 1, "the scan found no inline-asm wide store at all (st_sc1_x4 moved?)"
    assert not bad, "\n".join(bad)


def test_the_check_fails_without_the_nop():
    # hx_common.h's st_sc1_x4 as it is, and with its s_nop removed or zeroed
    src = open(os.path.join(ROOT, "include", "hclib_hip", "hx_common.h")).read()
    assert violations(src) == []
    stripped = src.replace("\\n\\ts_nop 2", "")
    assert stripped != src
    assert len(violations(stripped)) == 1
    assert len(violations(src.replace("s_nop 2", "s_nop 0"))) == 1
    # a store followed by a VALU write in the same statement
    assert violations('asm volatile("global_store_dwordx3 %0, %1, off\\n\\tv_mov_b32 %1, 0" ::);')
    # several statements, concatenated literals, an 8-byte store (no hazard)
    ok = ('asm volatile("buffer_store_dwordx4 %0, %1, 0 offen\\n" "s_nop 1" ::);\n'
          'asm("global_store_dwordx2 %0, %1, off" ::);')
    assert violations(ok) == []
