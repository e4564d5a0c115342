#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists).

Sources of truth, in order:
  1. numbers the reference publishes (test/uts/sample_trees.sh:17-43,
     test/smithwaterman/run.sh:23-44, test/fib/fib.c:38-46);
  2. the reference's own UTS generator compiled in place (oracle/_ref,
     `make -C oracle ref`) for SHA-1 vectors, numChildren vectors and the
     per-level T1 histogram;
  3. the oracle restatement, only where (1) and (2) pin it (SW edge
     checksums for the smaller tile configs; asserted against (1) first).
The data files under tests/golden/sw/ are the reference's own input files
(test/smithwaterman/input/*.txt), copied verbatim as fixtures.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import loader as L  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

# test/uts/sample_trees.sh:17-77 (published; XL and larger not regenerated here)
PUBLISHED_UTS = {
    "T1": ("-t 1 -a 3 -d 10 -b 4 -r 19", 4130071, 10, 3305118),
    "T5": ("-t 1 -a 0 -d 20 -b 4 -r 34", 4147582, 20, 2181318),
    "T2": ("-t 1 -a 2 -d 16 -b 6 -r 502", 4117769, 81, 2342762),
    "T3": ("-t 0 -b 2000 -q 0.124875 -m 8 -r 42", 4112897, 1572, 3599034),
    "T4": ("-t 2 -a 0 -d 16 -b 6 -r 1 -q 0.234375 -m 4 -r 1", 4132453, 134, 3108986),
    "T1L": ("-t 1 -a 3 -d 13 -b 4 -r 29", 102181082, 13, 81746377),
    "T2L": ("-t 1 -a 2 -d 23 -b 7 -r 220", 96793510, 67, 53791152),
    "T3L": ("-t 0 -b 2000 -q 0.200014 -m 5 -r 7", 111345631, 17844, 89076904),
    "T1XL": ("-t 1 -a 3 -d 15 -b 4 -r 29", 1635119272, 15, 1308100063),
}

# test/smithwaterman/run.sh:14-44 (tile width, tile height, expected score)
PUBLISHED_SW = {
    "tiny": (4, 4, 12),
    "medium": (232, 240, 3640),
    "large": (2320, 2400, 36472),
    "huge": (11600, 12000, 364792),
}
# first 65,536 ACGT characters of each huge input
SW64K_SHA = (
    "32b635bb615e21be2f49d2e4fbf94bceb3b78fe267ef9cfce4916e7f6a88de8d",
    "b498a26cdfeb0d61a98c59c60a7096bdc48626e7eddb51682d92d34482de396a",
)
SW64K_SCORE = 128772


def ref_args(s: str):
    toks = ["uts"] + s.split()
    return len(toks), (C.c_char_p * len(toks))(*[t.encode() for t in toks])


def be_words(b: bytes):
    return [int.from_bytes(b[4 * k:4 * k + 4], "big") for k in range(5)]


def gen_uts(ref, full: bool):
    out = {"published": {}, "sha1": {}, "num_children": {}, "levels": {}}
    for name, (args, n, d, lv) in PUBLISHED_UTS.items():
        out["published"][name] = {"args": args, "nodes": n, "depth": d, "leaves": lv,
                                  "source": "test/uts/sample_trees.sh"}
    # reference run of the small trees (+ T3L when --full): must equal the published numbers
    names = ["T1", "T2", "T3", "T4", "T5"] + (["T3L", "T1L"] if full else [])
    for name in names:
        args = PUBLISHED_UTS[name][0]
        argc, argv = ref_args(args)
        nn, nl, md = C.c_ulonglong(), C.c_ulonglong(), C.c_ulonglong()
        hist = (C.c_ulonglong * 128)()
        ref.ref_uts_run(argc, argv, C.byref(nn), C.byref(nl), C.byref(md), hist, 128)
        _, n, d, lv = PUBLISHED_UTS[name]
        assert (nn.value, md.value, nl.value) == (n, d, lv), (name, nn.value, md.value, nl.value)
        if md.value < 128:
            out["levels"][name] = list(hist)[: md.value + 1]
        print(f"ref {name}: ok {n} nodes")
    # SHA-1 / rng vectors from the reference brg_sha1.c
    vec = []
    for seed in [0, 1, 7, 19, 29, 34, 42, 220, 502, 2**31 - 1]:
        b = (C.c_ubyte * 20)()
        ref.ref_rng_init(seed, b)
        root = bytes(b)
        kids = {}
        for i in [0, 1, 2, 4, 99, 1999]:
            c = (C.c_ubyte * 20)()
            ref.ref_rng_spawn(b, i, c)
            kids[str(i)] = bytes(c).hex()
        vec.append({"seed": seed, "root": root.hex(), "rand": ref.ref_rng_rand(b),
                    "children": kids})
    out["sha1"] = vec
    # numChildren vectors for every small tree shape, states drawn from
    # spawn chains, heights spanning the tree's range
    rng = random.Random(1234)
    for name in ["T1", "T2", "T3", "T4", "T5", "T3L"]:
        args = PUBLISHED_UTS[name][0]
        argc, argv = ref_args(args)
        ref.ref_uts_set_params(argc, argv)
        p = L.parse_uts_args(args)
        rows = []
        b = (C.c_ubyte * 20)()
        ref.ref_rng_init(p.root_id, b)
        cur = bytes(b)
        maxh = PUBLISHED_UTS[name][2] + 2
        for k in range(400):
            c = (C.c_ubyte * 20)()
            ref.ref_rng_spawn((C.c_ubyte * 20)(*cur), rng.randrange(0, 100), c)
            cur = bytes(c)
            h = rng.randrange(0, maxh + 1) if k % 4 else 0
            nc = ref.ref_uts_num_children(p.type, h, (C.c_ubyte * 20)(*cur))
            rows.append([cur.hex(), h, nc])
        out["num_children"][name] = rows
    return out


def gen_sw(full: bool):
    res = {"published": {}, "configs": []}
    seqs = {}
    for size in ["tiny", "medium", "large", "huge"]:
        s1 = L.sw_map(open(os.path.join(GOLD, "sw", f"string1-{size}.txt"), "rb").read())
        s2 = L.sw_map(open(os.path.join(GOLD, "sw", f"string2-{size}.txt"), "rb").read())
        seqs[size] = (s1, s2)
        tw, th, exp = PUBLISHED_SW[size]
        res["published"][size] = {"tile_w": tw, "tile_h": th, "score": exp,
                                  "len1": len(s1), "len2": len(s2),
                                  "source": "test/smithwaterman/run.sh"}
        if size != "huge" or full:
            got = L.sw_score(s1, s2, tw, th)
            assert got == exp, (size, got, exp)
            print(f"oracle sw {size}: {got} == published")
    s1, s2 = seqs["huge"]
    p1, p2 = s1[:65536], s2[:65536]
    # the survey hashed the ACGT characters as text
    t1 = bytes(b"_ACGT"[x] for x in p1)
    t2 = bytes(b"_ACGT"[x] for x in p2)
    assert hashlib.sha256(t1).hexdigest() == SW64K_SHA[0]
    assert hashlib.sha256(t2).hexdigest() == SW64K_SHA[1]
    res["sw64k"] = {"len": 65536, "tile": 256, "score": SW64K_SCORE,
                    "sha256_1": SW64K_SHA[0], "sha256_2": SW64K_SHA[1],
                    "source": "SURVEY.md 8c (reference runtime run at 1/4/8 workers)"}
    if full:
        got = L.sw_score(p1, p2, 256, 256)
        assert got == SW64K_SCORE, got
        print("oracle sw64k: 128772 == survey golden")
    # oracle-derived edge checksums for smaller configs (oracle pinned above)
    for size, tw, th, n1, n2 in [("medium", 232, 240, None, None), ("medium", 16, 16, None, None),
                                 ("large", 64, 64, None, None), ("large", 256, 256, None, None),
                                 ("huge", 256, 256, 8192, 8192), ("huge", 64, 32, 4000, 3000)]:
        a, b = seqs[size]
        if n1:
            a, b = a[:n1], b[:n2]
        score, lr, lc = L.sw_score(a, b, tw, th, want_edges=True)
        res["configs"].append({"input": size, "len1": len(a), "len2": len(b), "tile_w": tw,
                               "tile_h": th, "score": score,
                               "last_row_sum": int(sum(lr)), "last_col_sum": int(sum(lc))})
    return res


def main():
    full = "--full" in sys.argv
    ref = L.ref_uts()
    if ref is None:
        sys.exit("build the reference harness first: make -C oracle ref")
    uts = gen_uts(ref, full)
    json.dump(uts, open(os.path.join(GOLD, "uts_goldens.json"), "w"), indent=1)
    sw = gen_sw(full)
    json.dump(sw, open(os.path.join(GOLD, "sw_goldens.json"), "w"), indent=1)
    fib = {"source": "test/fib/fib.c:38-46 fib_iter",
           "values": {str(n): L.fib_iter(n) for n in range(0, 41)}}
    json.dump(fib, open(os.path.join(GOLD, "fib_goldens.json"), "w"), indent=1)
    print("wrote", GOLD)


if __name__ == "__main__":
    main()
