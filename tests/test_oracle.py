"""Pin the CPU oracle (oracle/) against the reference's golden vectors.

Every assertion here compares the restatement with numbers the reference
publishes (test/uts/sample_trees.sh, test/smithwaterman/run.sh,
test/fib/fib.c) or with vectors produced by the reference's own UTS
sources compiled in place (scripts/gen_golden.py -> tests/golden/).
"""
import os

import pytest

from oracle import loader as L


def _words(hexstr):
    b = bytes.fromhex(hexstr)
    return [int.from_bytes(b[4 * k:4 * k + 4], "big") for k in range(5)]


def test_sha1_rng_vectors(golden):
    g = golden("uts_goldens.json")
    for v in g["sha1"]:
        root = L.rng_init(v["seed"])
        assert root == _words(v["root"])
        assert L.oracle().ora_rng_rand((__import__("ctypes").c_uint32 * 5)(*root)) == v["rand"]
        for i, h in v["children"].items():
            assert L.rng_spawn(root, int(i)) == _words(h)


@pytest.mark.parametrize("name", ["T1", "T2", "T3", "T4", "T5", "T3L"])
def test_num_children_vectors(golden, name):
    g = golden("uts_goldens.json")
    p = L.parse_uts_args(g["published"][name]["args"])
    for st, h, nc in g["num_children"][name]:
        assert L.uts_num_children(p, p.type, h, _words(st)) == nc, (name, st, h)


@pytest.mark.parametrize("name", ["T1", "T2", "T3", "T4", "T5"])
def test_uts_small_trees_published(golden, name):
    g = golden("uts_goldens.json")["published"][name]
    (n, lv, d), hist = L.uts_serial(L.parse_uts_args(g["args"]), max_levels=64)
    assert (n, d, lv) == (g["nodes"], g["depth"], g["leaves"])
    if name == "T1":
        levels = golden("uts_goldens.json")["levels"]["T1"]
        assert hist[: len(levels)] == levels


def test_uts_root_range_partition():
    p = L.parse_uts_args("-t 1 -a 3 -d 10 -b 4 -r 19")
    (n, lv, d), _ = L.uts_serial(p)
    parts = [L.uts_root_range(p, k, k + 1, k == 0) for k in range(5)]
    assert sum(x[0] for x in parts) == n
    assert sum(x[1] for x in parts) == lv
    assert max(x[2] for x in parts) == d


def _sw_inputs(size):
    from tests.conftest import GOLD

    a = open(os.path.join(GOLD, "sw", f"string1-{size}.txt"), "rb").read()
    b = open(os.path.join(GOLD, "sw", f"string2-{size}.txt"), "rb").read()
    return L.sw_map(a), L.sw_map(b)


@pytest.mark.parametrize("size", ["tiny", "medium", "large"])
def test_sw_published_scores(golden, size):
    g = golden("sw_goldens.json")["published"][size]
    s1, s2 = _sw_inputs(size)
    assert (len(s1), len(s2)) == (g["len1"], g["len2"])
    assert L.sw_score(s1, s2, g["tile_w"], g["tile_h"]) == g["score"]


def test_sw_64k_inputs_hash(golden):
    import hashlib

    g = golden("sw_goldens.json")["sw64k"]
    s1, s2 = _sw_inputs("huge")
    t1 = bytes(b"_ACGT"[x] for x in s1[:65536])
    t2 = bytes(b"_ACGT"[x] for x in s2[:65536])
    assert hashlib.sha256(t1).hexdigest() == g["sha256_1"]
    assert hashlib.sha256(t2).hexdigest() == g["sha256_2"]


def test_fib_table(golden):
    g = golden("fib_goldens.json")["values"]
    for n, v in g.items():
        assert L.fib_iter(int(n)) == v
    assert g["30"] == 832040


def test_forasync_flat_quirk():
    # domain {10,100,1,33} FLAT runs indices 10..108
    tile, counts = L.forasync1d_counts(10, 100, 1, 33, 0, 1, 0, 128)
    assert tile == 33
    assert counts[:10].sum() == 0 and (counts[10:109] == 1).all() and counts[109:].sum() == 0


def test_forasync_recursive_and_flat_cover_range():
    for mode in (0, 1):
        tile, counts = L.forasync1d_counts(0, 1024, 1, 33, mode, 8, 0, 1024)
        assert (counts == 1).all()
    tile, counts = L.forasync1d_counts(0, 1000, 1, -1, 1, 8, 0, 1000)
    assert tile == 125 and (counts == 1).all()


# ---- CPU work-stealing runtime restatement (the bench's cpu_baseline) ----
def test_cpu_runtime_fib():
    import ctypes as C

    lib = L.cpu_runtime()
    for w in (1, 4):
        for ddt in (0, 1):
            assert lib.ohc_fib(w, 20, ddt, None) == 6765


def test_cpu_runtime_uts_t1(golden):
    import ctypes as C

    lib = L.cpu_runtime()
    g = golden("uts_goldens.json")["published"]["T1"]
    p = L.parse_uts_args(g["args"])
    n, lv, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
    assert lib.ohc_uts(4, C.byref(p), C.byref(n), C.byref(lv), C.byref(d), None) == 0
    assert (n.value, lv.value, d.value) == (g["nodes"], g["leaves"], g["depth"])


def test_cpu_runtime_sw(golden):
    g = golden("sw_goldens.json")["published"]["medium"]
    s1, s2 = _sw_inputs("medium")
    assert L.cpu_runtime().ohc_sw(4, s1, len(s1), s2, len(s2), g["tile_w"], g["tile_h"], None) == g["score"]


def test_cpu_runtime_triad():
    import ctypes as C

    import numpy as np

    n = 1 << 16
    b = np.random.default_rng(1).random(n, dtype=np.float32)
    c = np.random.default_rng(2).random(n, dtype=np.float32)
    a = np.zeros(n, dtype=np.float32)
    f = C.POINTER(C.c_float)
    L.cpu_runtime().ohc_triad(4, a.ctypes.data_as(f), b.ctypes.data_as(f), c.ctypes.data_as(f),
                              C.c_float(3.0), n, -1, 0, None)
    exp = b + np.float32(3.0) * c
    assert np.array_equal(a, exp)
