"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU restatements in this directory. Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product package (hclib_amd) never does.

    liboracle.so    uts_oracle.c + sw_oracle.c  (serial restatements)
    libhclib_cpu.so hclib_cpu.c + workloads     (CPU work-stealing runtime)
    _ref/libref_uts.so  reference test/uts sources compiled in place
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
REF = os.path.join(HERE, "_ref")


class UtsParams(C.Structure):
    """ora_uts_params_t (uts_oracle.h); field meaning = UTS CLI flags."""

    _fields_ = [
        ("type", C.c_int),
        ("shape_fn", C.c_int),
        ("gen_mx", C.c_int),
        ("root_id", C.c_int),
        ("non_leaf_bf", C.c_int),
        ("compute_gran", C.c_int),
        ("b_0", C.c_double),
        ("non_leaf_prob", C.c_double),
        ("shift_depth", C.c_double),
    ]


class UtsResult(C.Structure):
    _fields_ = [("nodes", C.c_uint64), ("leaves", C.c_uint64), ("max_depth", C.c_uint64)]


def parse_uts_args(argv: str) -> UtsParams:
    """Parse a UTS argument string (test/uts/uts.c:362-425 semantics)."""
    lib = oracle()
    p = UtsParams()
    lib.ora_uts_default_params(C.byref(p))
    toks = argv.split()
    for i in range(0, len(toks), 2):
        flag, val = toks[i], toks[i + 1]
        c = flag[1]
        if c == "q":
            p.non_leaf_prob = float(val)
        elif c == "m":
            p.non_leaf_bf = int(val)
        elif c == "r":
            p.root_id = int(val)
        elif c == "t":
            p.type = int(val)
        elif c == "a":
            p.shape_fn = int(val)
        elif c == "b":
            p.b_0 = float(val)
        elif c == "d":
            p.gen_mx = int(val)
        elif c == "f":
            p.shift_depth = float(val)
        elif c == "g":
            p.compute_gran = max(1, int(val))
        elif c in "cixv":
            pass
        else:
            raise ValueError(f"unknown UTS flag {flag}")
    return p


_libs: dict = {}


def ensure_built() -> None:
    if not (os.path.exists(os.path.join(BUILD, "liboracle.so"))
            and os.path.exists(os.path.join(BUILD, "libhclib_cpu.so"))):
        subprocess.check_call(["make", "-s", "-C", HERE, "all"])


def _load(name: str, path: str):
    if name not in _libs:
        _libs[name] = C.CDLL(path)
    return _libs[name]


def oracle():
    ensure_built()
    lib = _load("oracle", os.path.join(BUILD, "liboracle.so"))
    lib.ora_sw_score.restype = C.c_int
    lib.ora_fib_iter.restype = C.c_long
    lib.ora_sw_map.restype = C.c_size_t
    return lib


def cpu_runtime():
    ensure_built()
    lib = _load("cpu", os.path.join(BUILD, "libhclib_cpu.so"))
    lib.ohc_fib.restype = C.c_long
    lib.ohc_sw.restype = C.c_int
    return lib


def ref_uts():
    """The reference's own UTS generator (oracle/_ref); None if not built."""
    path = os.path.join(REF, "libref_uts.so")
    if not os.path.exists(path):
        return None
    return _load("ref", path)


# ---------------------------------------------------------------- helpers
def uts_serial(p: UtsParams, max_levels: int = 0):
    lib = oracle()
    r = UtsResult()
    hist = (C.c_uint64 * max_levels)() if max_levels else None
    rc = lib.ora_uts_serial(C.byref(p), C.byref(r), hist, max_levels)
    assert rc == 0
    return (r.nodes, r.leaves, r.max_depth), (list(hist) if hist is not None else None)


def uts_root_range(p: UtsParams, first: int, last: int, count_root: bool):
    lib = oracle()
    r = UtsResult()
    assert lib.ora_uts_serial_root_range(C.byref(p), first, last, int(count_root), C.byref(r)) == 0
    return (r.nodes, r.leaves, r.max_depth)


def rng_init(seed: int):
    st = (C.c_uint32 * 5)()
    oracle().ora_rng_init(st, seed)
    return list(st)


def rng_spawn(parent, i: int):
    par = (C.c_uint32 * 5)(*parent)
    ch = (C.c_uint32 * 5)()
    oracle().ora_rng_spawn(par, ch, i)
    return list(ch)


def uts_num_children(p: UtsParams, node_type: int, height: int, st) -> int:
    s = (C.c_uint32 * 5)(*st)
    return oracle().ora_uts_num_children(C.byref(p), node_type, height, s)


def sw_map(text: bytes) -> bytes:
    out = C.create_string_buffer(len(text) + 1)
    n = oracle().ora_sw_map(text, len(text), out)
    return out.raw[:n]


def sw_score(s1: bytes, s2: bytes, tw: int, th: int, want_edges: bool = False):
    lib = oracle()
    W = (len(s1) // tw) * tw
    R = (len(s2) // th) * th
    lr = (C.c_int * (W + 1))() if want_edges else None
    lc = (C.c_int * (R + 1))() if want_edges else None
    score = lib.ora_sw_score(s1, len(s1), s2, len(s2), tw, th, lr, lc)
    if want_edges:
        return score, list(lr), list(lc)
    return score


def fib_iter(n: int) -> int:
    return oracle().ora_fib_iter(n)


def forasync1d_counts(low, high, stride, tile, mode, nworkers, base, ncounts):
    import numpy as np

    counts = np.zeros(ncounts, dtype=np.int32)
    tile_used = oracle().ora_forasync1d_counts(
        low, high, stride, tile, mode, nworkers, base,
        counts.ctypes.data_as(C.POINTER(C.c_int32)), ncounts)
    return tile_used, counts


def forasync_nd_counts(domains, mode, nworkers, bases, extents):
    """Visit counts of hclib_forasync for dim 1..3 (src/hclib.c:110-464):
    1-D uses the exact 1-D lowering (incl. the FLAT quirk); 2-D/3-D FLAT
    tiles each dimension with clamped tiles (src/hclib.c:353-416), RECURSIVE
    bisects each dimension (192-314); the runner restarts the stride at every
    tile's low bound. Returns (tiles_used, counts ndarray)."""
    import numpy as np

    dom = [list(d) for d in domains]
    for d in dom:
        if d[3] == -1:
            d[3] = ((d[1] - d[0]) + nworkers - 1) // nworkers
    if len(dom) == 1:
        t, c = forasync1d_counts(*dom[0], mode, nworkers, bases[0], extents[0])
        return [t], c

    def per_dim(low, high, stride, tile):
        idx = []
        if mode == 1:
            def rec(lo, hi):
                if hi - lo > tile:
                    mid = (hi + lo) // 2
                    rec(lo, mid)
                    rec(mid, hi)
                else:
                    idx.extend(range(lo, hi, stride))
            rec(low, high)
        else:
            lo = low
            while lo < high:
                hi = min(lo + tile, high)
                idx.extend(range(lo, hi, stride))
                lo += tile
        return idx

    sets = [per_dim(*d) for d in dom]
    counts = np.zeros(extents, dtype=np.int32)
    import itertools

    for tup in itertools.product(*sets):
        loc = tuple(v - b for v, b in zip(tup, bases))
        if all(0 <= l < e for l, e in zip(loc, extents)):
            counts[loc] += 1
    return [d[3] for d in dom], counts
