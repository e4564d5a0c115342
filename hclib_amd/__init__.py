"""hclib_amd — MI355X-native HClib task-scheduling hot path.

Python mirror of the module's C ABI (include/hclib_hip.h). The compute
entry points run only through the in-tree HIP library
hclib_amd/lib/libhclib_amd.so; there is no CPU fallback — if the library or
a gfx950 device is missing they raise HclibError.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

PKG = os.path.dirname(os.path.abspath(__file__))
# HCLIB_AMD_LIB selects a diagnostic variant (python -m hclib_amd.build --variant X)
LIB_PATH = os.environ.get("HCLIB_AMD_LIB") or os.path.join(PKG, "lib", "libhclib_amd.so")

HCLIB_HIP_OK = 0
FORASYNC_MODE_FLAT = 0       # inc/hclib.h:161
FORASYNC_MODE_RECURSIVE = 1  # inc/hclib.h:159
BODY_TRIAD_F32 = 1
BODY_IOTA_CHECK = 2
BODY_VISIT_COUNT = 3


class HclibError(RuntimeError):
    pass


class LoopDomain(C.Structure):
    """hclib_loop_domain_t, inc/hclib-task.h:53-58."""

    _fields_ = [("low", C.c_int), ("high", C.c_int), ("stride", C.c_int), ("tile", C.c_int)]


class TriadArgs(C.Structure):
    _fields_ = [("a", C.c_void_p), ("b", C.c_void_p), ("c", C.c_void_p), ("s", C.c_float)]


class IotaArgs(C.Structure):
    _fields_ = [("ran", C.c_void_p), ("errors", C.c_void_p)]


class VisitArgs(C.Structure):
    _fields_ = [("counts", C.c_void_p), ("base", C.c_int * 3), ("extent", C.c_int * 3)]


class UtsParams(C.Structure):
    """hclib_hip_uts_params_t — the UTS CLI flags of test/uts/uts.c:380-420."""

    _fields_ = [
        ("type", C.c_int), ("shape_fn", C.c_int), ("gen_mx", C.c_int), ("root_id", C.c_int),
        ("non_leaf_bf", C.c_int), ("compute_gran", C.c_int), ("b_0", C.c_double),
        ("non_leaf_prob", C.c_double), ("shift_depth", C.c_double),
    ]


class UtsResult(C.Structure):
    _fields_ = [
        ("nodes", C.c_uint64), ("leaves", C.c_uint64), ("max_depth", C.c_uint64),
        ("chunks_pushed", C.c_uint64), ("chunks_stolen", C.c_uint64), ("batches", C.c_uint64),
        ("kernel_ms", C.c_double), ("busy_frac", C.c_double), ("us_per_batch", C.c_double),
    ]


class UtsLaunch(C.Structure):
    _fields_ = [(k, C.c_int) for k in ("mode", "feat", "workers_per_group", "grid", "ring", "seeded",
                                       "seed_target", "spill_lo", "waves_per_cu")]


UTS_MODES = {0: "rules_global", 1: "rules_lds", 2: "bin", 3: "geo_fixed"}


class FibResult(C.Structure):
    _fields_ = [("tasks", C.c_uint64), ("joins", C.c_uint64), ("chunks_pushed", C.c_uint64),
                ("chunks_stolen", C.c_uint64), ("kernel_ms", C.c_double),
                ("busy_frac", C.c_double)]


class SwResult(C.Structure):
    _fields_ = [("tiles", C.c_uint64), ("releases", C.c_uint64), ("kernel_ms", C.c_double),
                ("cells_per_s", C.c_double), ("tile_us", C.c_double), ("release_us", C.c_double)]


# every symbol include/hclib_hip.h and include/hclib.h declare (checked by tests)
EXPORTS_HIP = [
    "hclib_hip_init", "hclib_hip_finalize", "hclib_hip_last_error", "hclib_hip_num_cus",
    "hclib_hip_version", "hclib_hip_forasync", "hclib_hip_forasync_triad_f32",
    "hclib_hip_num_workers", "hclib_hip_uts_search", "hclib_hip_uts_num_children_host",
    "hclib_hip_uts_bucket_check", "hclib_hip_sha1_calibrate",
    "hclib_hip_fib", "hclib_hip_sw", "hclib_hip_last_sched_counters", "hclib_hip_last_narrow_counters",
    "hclib_hip_last_phase_counters",
    "hclib_hip_sw_band_begin", "hclib_hip_sw_band_rows", "hclib_hip_sw_band_end",
]

_lib = None


def lib():
    """Load the HIP module library (never a fallback: raises if absent)."""
    global _lib
    if _lib is None:
        try:  # share ONE HIP runtime with torch (same soname libamdhip64.so.7)
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise HclibError(f"{LIB_PATH} is missing: run `python -m hclib_amd.build`")
        L = C.CDLL(LIB_PATH)
        L.hclib_hip_version.restype = C.c_char_p
        L.hclib_hip_last_error.restype = C.c_char_p
        L.hclib_hip_forasync_triad_f32.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float,
                                                   C.c_int64, C.c_void_p]
        L.hclib_hip_forasync.argtypes = [C.c_int, C.c_void_p, C.c_int, C.POINTER(LoopDomain),
                                         C.c_int, C.c_void_p]
        L.hclib_hip_uts_search.argtypes = [C.POINTER(UtsParams), C.c_int, C.c_int, C.c_int,
                                           C.POINTER(UtsResult), C.c_void_p, C.c_int]
        L.hclib_hip_uts_num_children_host.argtypes = [C.POINTER(UtsParams), C.c_int,
                                                      C.POINTER(C.c_uint32)]
        L.hclib_hip_fib.argtypes = [C.c_int, C.POINTER(C.c_int64), C.POINTER(FibResult)]
        L.hclib_hip_sw.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int,
                                   C.c_int, C.POINTER(C.c_int), C.POINTER(SwResult)]
        L.hclib_hip_sw_band_begin.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                              C.c_int, C.c_int, C.c_int, C.c_int,
                                              C.POINTER(C.c_void_p)]
        L.hclib_hip_sw_band_rows.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                             C.c_void_p]
        L.hclib_hip_sw_band_end.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int),
                                            C.POINTER(C.c_uint64)]
        L.hclib_hip_atomic_calibrate.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double),
                                                 C.POINTER(C.c_double)]
        L.hclib_hip_sha1_calibrate.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double),
                                               C.POINTER(C.c_double)]
        L.hclib_hip_uts_last_launch.argtypes = [C.POINTER(UtsLaunch)]
        L.hclib_hip_uts_bucket_check.argtypes = [C.POINTER(UtsParams), C.c_uint64, C.POINTER(C.c_uint64)]
        L.hclib_hip_global_bytes.restype = C.c_size_t
        L.hclib_hip_global_bytes.argtypes = [C.c_uint32]
        L.hclib_hip_global_init.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
        L.hclib_hip_global_alloc.argtypes = [C.c_uint32, C.c_int, C.POINTER(C.c_void_p)]
        L.hclib_hip_global_free.argtypes = [C.c_void_p]
        L.hclib_hip_global_attach.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
        L.hclib_hip_global_read.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.hclib_hip_ipc_export.argtypes = [C.c_void_p, C.c_void_p]
        L.hclib_hip_ipc_import.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.hclib_hip_ipc_close.argtypes = [C.c_void_p]
        L.hclib_hip_last_timeline.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32)]
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != HCLIB_HIP_OK:
        msg = lib().hclib_hip_last_error().decode(errors="replace")
        raise HclibError(f"{what} failed ({rc}): {msg}")


def version() -> str:
    return lib().hclib_hip_version().decode()


def init(device: int = 0) -> None:
    _check(lib().hclib_hip_init(device), "hclib_hip_init")


def num_cus() -> int:
    return lib().hclib_hip_num_cus()


def num_workers() -> int:
    return lib().hclib_hip_num_workers()


# ------------------------------------------------------------------ forasync
def forasync(body: int, args: C.Structure, domains, mode: int, stream: Optional[int] = None):
    """hclib_forasync at the GPU locale (src/hclib.c:452-464); domains is a
    list of (low, high, stride, tile). Returns the domains after the tile==-1
    write-back, as the reference does."""
    dims = (LoopDomain * len(domains))(*[LoopDomain(*d) for d in domains])
    _check(lib().hclib_hip_forasync(body, C.byref(args), len(domains), dims, mode, stream),
           "hclib_hip_forasync")
    return [(d.low, d.high, d.stride, d.tile) for d in dims]


def triad_f32(a_ptr: int, b_ptr: int, c_ptr: int, s: float, n: int, stream: Optional[int] = None):
    _check(lib().hclib_hip_forasync_triad_f32(a_ptr, b_ptr, c_ptr, s, n, stream),
           "hclib_hip_forasync_triad_f32")


# ----------------------------------------------------------------------- UTS
def parse_uts_args(argv: str) -> UtsParams:
    """UTS argument string -> params (test/uts/uts.c:362-425; T1 defaults)."""
    p = UtsParams(type=1, shape_fn=3, gen_mx=10, root_id=19, non_leaf_bf=4, compute_gran=1,
                  b_0=4.0, non_leaf_prob=15.0 / 64.0, shift_depth=0.5)
    toks = argv.split()
    if len(toks) % 2:
        raise ValueError("UTS arguments come in flag/value pairs")
    for flag, val in zip(toks[::2], toks[1::2]):
        c = flag[1]
        if c == "q": p.non_leaf_prob = float(val)
        elif c == "m": p.non_leaf_bf = int(val)
        elif c == "r": p.root_id = int(val)
        elif c == "t": p.type = int(val)
        elif c == "a": p.shape_fn = int(val)
        elif c == "b": p.b_0 = float(val)
        elif c == "d": p.gen_mx = int(val)
        elif c == "f": p.shift_depth = float(val)
        elif c == "g": p.compute_gran = max(1, int(val))
        elif c in "cixv": pass
        else: raise ValueError(f"unknown UTS flag {flag}")
    return p


def uts(params, shard: int = 0, nshards: int = 1, split_depth: int = 0, max_levels: int = 0):
    """Search a UTS tree on the GPU; returns a dict of counts and stats."""
    if isinstance(params, str):
        params = parse_uts_args(params)
    r = UtsResult()
    hist = (C.c_uint64 * max_levels)() if max_levels else None
    _check(lib().hclib_hip_uts_search(C.byref(params), shard, nshards, split_depth, C.byref(r),
                                      hist, max_levels), "hclib_hip_uts_search")
    out = {k: getattr(r, k) for k, _ in UtsResult._fields_}
    if hist is not None:
        out["levels"] = list(hist)
    return out


def uts_last_launch() -> dict:
    """The launch shape of this thread's last uts() (hclib_hip_uts_last_launch)."""
    r = UtsLaunch()
    _check(lib().hclib_hip_uts_last_launch(C.byref(r)), "hclib_hip_uts_last_launch")
    out = {k: getattr(r, k) for k, _ in UtsLaunch._fields_}
    out["mode"] = UTS_MODES.get(out["mode"], out["mode"])
    return out


def uts_bucket_check(params, nrandom: int = 1 << 20):
    """Host check (no GPU) of the bucketed numChildren lookup the fixed-shape
    GEO kernels use: (mismatches, values compared)."""
    if isinstance(params, str):
        params = parse_uts_args(params)
    n = C.c_uint64()
    bad = lib().hclib_hip_uts_bucket_check(C.byref(params), nrandom, C.byref(n))
    if bad < 0:
        raise HclibError(f"hclib_hip_uts_bucket_check failed ({bad}): "
                         f"{lib().hclib_hip_last_error().decode(errors='replace')}")
    return bad, n.value


def uts_num_children_host(params, height: int, state_words) -> int:
    if isinstance(params, str):
        params = parse_uts_args(params)
    st = (C.c_uint32 * 5)(*state_words)
    return lib().hclib_hip_uts_num_children_host(C.byref(params), height, st)


# ----------------------------------------------------------------------- fib
def global_bytes(cap: int) -> int:
    """Bytes of a cross-GPU work-sharing region with `cap` chunk slots."""
    n = lib().hclib_hip_global_bytes(cap)
    if n == 0:
        raise HclibError("global_bytes: cap must be a power of two >= 2")
    return n


GLOBAL_MEM_KINDS = {"uncached": 0, "fine": 1, "device": 2}


def global_alloc(cap: int, kind: str = "uncached") -> int:
    """Allocate a work-sharing region (hclib_hip_global_alloc); kind is one of
    GLOBAL_MEM_KINDS."""
    p = C.c_void_p()
    _check(lib().hclib_hip_global_alloc(cap, GLOBAL_MEM_KINDS[kind], C.byref(p)), "hclib_hip_global_alloc")
    return p.value


def global_free(region: Optional[int]) -> None:
    _check(lib().hclib_hip_global_free(region), "hclib_hip_global_free")


def global_init(region: int, cap: int, nranks: int) -> None:
    _check(lib().hclib_hip_global_init(region, cap, nranks), "hclib_hip_global_init")


def global_attach(region: Optional[int], cap: int = 0, rank: int = 0) -> None:
    _check(lib().hclib_hip_global_attach(region, cap, rank), "hclib_hip_global_attach")


def global_read(region: int) -> dict:
    out = (C.c_uint64 * 35)()
    _check(lib().hclib_hip_global_read(region, out), "hclib_hip_global_read")
    return {"active": out[0], "idle": out[1], "queued": out[2],
            "exported": [out[3 + 2 * r] for r in range(16)], "imported": [out[4 + 2 * r] for r in range(16)]}


def ipc_export(dev_ptr: int) -> bytes:
    h = (C.c_char * 64)()
    _check(lib().hclib_hip_ipc_export(dev_ptr, h), "hclib_hip_ipc_export")
    return bytes(h)


def ipc_import(handle: bytes) -> int:
    p = C.c_void_p()
    _check(lib().hclib_hip_ipc_import(C.c_char_p(handle), C.byref(p)), "hclib_hip_ipc_import")
    return p.value


def ipc_close(dev_ptr: int) -> None:
    _check(lib().hclib_hip_ipc_close(dev_ptr), "hclib_hip_ipc_close")


def fib(n: int):
    v = C.c_int64()
    r = FibResult()
    _check(lib().hclib_hip_fib(n, C.byref(v), C.byref(r)), "hclib_hip_fib")
    return v.value, {k: getattr(r, k) for k, _ in FibResult._fields_}


# ------------------------------------------------------------------------ SW
def sw(s1: bytes, s2: bytes, tile_w: int, tile_h: int):
    """Tiled Smith-Waterman DAG on the GPU; sequences coded 1..4."""
    score = C.c_int()
    r = SwResult()
    _check(lib().hclib_hip_sw(s1, len(s1), s2, len(s2), tile_w, tile_h, C.byref(score),
                              C.byref(r)), "hclib_hip_sw")
    return score.value, {k: getattr(r, k) for k, _ in SwResult._fields_}


class SwBand:
    """One rank's band of tile columns [j0, j1) of the SW tile grid
    (hclib_hip_sw_band_*, include/hclib_hip.h). rows() launches tile rows
    [i0, i1) on `stream` (a raw hipStream_t handle, e.g. torch's
    current_stream().cuda_stream); left_in / right_out are device pointers
    to nth*th int32 (H of matrix columns j0*tw and j1*tw, rows 1..)."""

    def __init__(self, s1: bytes, s2: bytes, tile_w: int, tile_h: int, j0: int, j1: int):
        self.ntw, self.nth = len(s1) // tile_w, len(s2) // tile_h
        self.tile_w, self.tile_h, self.j0, self.j1 = tile_w, tile_h, j0, j1
        h = C.c_void_p()
        _check(lib().hclib_hip_sw_band_begin(s1, len(s1), s2, len(s2), tile_w, tile_h, j0, j1,
                                             C.byref(h)), "hclib_hip_sw_band_begin")
        self._h = h

    def rows(self, i0: int, i1: int, left_in: int | None, right_out: int | None, stream: int):
        _check(lib().hclib_hip_sw_band_rows(self._h, i0, i1, left_in, right_out, stream),
               "hclib_hip_sw_band_rows")

    def end(self, stream: int):
        """Synchronise, free; returns (bottom-right cell of the band, tiles run)."""
        corner, tiles = C.c_int(), C.c_uint64()
        h, self._h = self._h, None
        _check(lib().hclib_hip_sw_band_end(h, stream, C.byref(corner), C.byref(tiles)),
               "hclib_hip_sw_band_end")
        return corner.value, tiles.value


def sw_map(text: bytes) -> bytes:
    """clear_whitespaces_do_mapping (smith_waterman.cpp:45-59): keep ACGT -> 1..4."""
    table = bytes.maketrans(b"ACGT", b"\x01\x02\x03\x04")
    return bytes(x for x in text if x in b"ACGT").translate(table)


ATOMIC_SCATTER_RET64 = 0  # include/hclib_hip.h
ATOMIC_HOT_WORD = 1
ATOMIC_COALESCED32 = 2


def atomic_calibrate(mode: int, iters: int = 256):
    """Saturated L2 atomic rate of one access shape: (Mops/s, kernel ms)."""
    r, ms = C.c_double(), C.c_double()
    _check(lib().hclib_hip_atomic_calibrate(mode, iters, C.byref(r), C.byref(ms)),
           "hclib_hip_atomic_calibrate")
    return r.value, ms.value


def sha1_calibrate(chains: int = 1, waves_per_cu: int = 8, iters: int = 2000):
    """The chip's UTS SHA-1 issue ceiling (SHA-1/s, kernel ms): the
    rng_spawn stream of k_uts_search back to back on every lane."""
    r, ms = C.c_double(), C.c_double()
    _check(lib().hclib_hip_sha1_calibrate(chains, waves_per_cu, iters, C.byref(r), C.byref(ms)),
           "hclib_hip_sha1_calibrate")
    return r.value, ms.value


def last_phase_counters():
    """HX_PHASES builds: main-loop batch phase cycles of the last launch
    (hclib_hip_last_phase_counters)."""
    out = (C.c_uint64 * 8)()
    lib().hclib_hip_last_phase_counters(out)
    return list(out)


def last_sched_counters():
    """Counters of the last megakernel launch (see include/hclib_hip.h)."""
    out = (C.c_uint64 * 16)()
    lib().hclib_hip_last_sched_counters(out)
    return list(out)


def last_narrow_counters():
    """Narrow-frontier loop of the last launch: batches, cycles, entries."""
    out = (C.c_uint64 * 4)()
    lib().hclib_hip_last_narrow_counters(out)
    return list(out)


TIMELINE_EVENTS = {1: "start", 2: "busy", 3: "idle", 4: "spill", 5: "term", 6: "end"}


def last_timeline():
    """Worker timelines of the last megakernel launch (a `--variant timeline`
    library run with HCLIB_HIP_TIMELINE=<events per worker>, hx_sched.h
    Timeline): per worker a list of (time in 10 ns ticks, event, value)."""
    per = C.c_uint32()
    nw = lib().hclib_hip_last_timeline(None, 0, C.byref(per))
    if nw <= 0 or per.value == 0:
        return []
    import numpy as np
    buf = np.zeros(nw * per.value, dtype=np.uint64)
    lib().hclib_hip_last_timeline(buf.ctypes.data, buf.size, C.byref(per))
    buf = buf.reshape(nw, per.value)
    out = []
    for w in range(nw):
        row = buf[w][buf[w] != 0]
        out.append([(int(v >> 24), int((v >> 20) & 0xF), int(v & 0xFFFFF)) for v in row])
    return out
