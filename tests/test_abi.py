"""CPU-side checks of the product's C ABI: the library builds for gfx950,
loads without a GPU, exports every declared symbol, and its host-side UTS
threshold tables agree with the reference's numChildren vectors.
No compute call runs here."""
import ctypes as C
import os
import re

import pytest

import hclib_amd as H
from tests.conftest import ROOT


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hclib_\w+)\s*\(", txt)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = H.lib()
    for header in ("hclib_hip.h", "hclib.h"):
        path = os.path.join(ROOT, "include", header)
        if not os.path.exists(path):
            continue
        for sym in _declared(header):
            assert hasattr(lib, sym), f"{sym} declared in {header} but not exported"
    for sym in H.EXPORTS_HIP:
        assert hasattr(lib, sym)
    assert "gfx950" in H.version()


def test_built_for_gfx950_only():
    out = os.popen(f"/opt/rocm/lib/llvm/bin/llvm-objdump --offloading {H.LIB_PATH} 2>/dev/null"
                   f" | grep -o 'gfx[0-9a-z]*' | sort -u").read().split()
    if not out:  # older objdump: fall back to the clang offload bundle marker
        data = open(H.LIB_PATH, "rb").read()
        out = sorted(set(m.decode() for m in re.findall(rb"gfx[0-9]{3}[a-z]?", data)))
    assert out and set(out) == {"gfx950"}, out


def _words(hexstr):
    b = bytes.fromhex(hexstr)
    return [int.from_bytes(b[4 * k:4 * k + 4], "big") for k in range(5)]


@pytest.mark.parametrize("name", ["T1", "T2", "T3", "T4", "T5", "T3L"])
def test_uts_device_tables_match_reference_vectors(golden, name):
    g = golden("uts_goldens.json")
    p = H.parse_uts_args(g["published"][name]["args"])
    for st, h, nc in g["num_children"][name]:
        if h == 0:
            continue  # root rule is checked below
        want = nc if nc > 0 else 0
        got = H.uts_num_children_host(p, h, _words(st))
        assert max(got, 0) == want, (name, st, h, got, nc)


@pytest.mark.parametrize("name", ["T1", "T1L", "T1XL", "T2", "T4", "T5", "T2L", "T3L"])
def test_uts_bucketed_num_children_is_exact(golden, name):
    """The fixed-shape GEO kernels count a node's children with 1,024 rand
    buckets and two compares (uts.hip uts_nc<kUtsGeoFixed>); the host mirror
    of that lookup equals #{k : thr[k] <= rand} at every threshold +-3, every
    bucket edge +-1 and 2^18 random values, for every published tree's first
    threshold table (BIN trees have none: nothing to check)."""
    g = golden("uts_goldens.json")
    bad, n = H.uts_bucket_check(g["published"][name]["args"], 1 << 18)
    assert bad == 0, (name, bad, n)
    assert n > (1 << 18) or name == "T3L"


@pytest.mark.parametrize("name", ["T1", "T3", "T3L", "T5"])
def test_uts_device_root_rule(golden, name):
    from oracle import loader as L

    g = golden("uts_goldens.json")
    args = g["published"][name]["args"]
    p = H.parse_uts_args(args)
    op = L.parse_uts_args(args)
    root = L.rng_init(op.root_id)
    assert H.uts_num_children_host(p, 0, root) == L.uts_num_children(op, op.type, 0, root)


def test_uts_tables_random_states_vs_oracle():
    """Random spawn states at every depth of T1/T2/T4/T5 vs the libm oracle."""
    import random

    from oracle import loader as L

    rng = random.Random(7)
    for args in ["-t 1 -a 3 -d 10 -b 4 -r 19", "-t 1 -a 2 -d 16 -b 6 -r 502",
                 "-t 2 -a 0 -d 16 -b 6 -r 1 -q 0.234375 -m 4 -r 1", "-t 1 -a 0 -d 20 -b 4 -r 34",
                 "-t 1 -a 1 -d 8 -b 3 -r 5"]:
        p = H.parse_uts_args(args)
        op = L.parse_uts_args(args)
        st = L.rng_init(op.root_id)
        for k in range(3000):
            st = L.rng_spawn(st, rng.randrange(100))
            h = rng.randrange(1, 40)
            want = max(0, L.uts_num_children(op, op.type, h, st))
            assert max(0, H.uts_num_children_host(p, h, st)) == want, (args, h)


def test_compute_entry_points_fail_loudly_without_gpu():
    """No CPU fallback: without a gfx950 device the compute calls raise."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(H.HclibError):
        H.fib(10)
    with pytest.raises(H.HclibError):
        H.uts("-t 1 -a 3 -d 10 -b 4 -r 19")
    with pytest.raises(H.HclibError):
        H.atomic_calibrate(H.ATOMIC_SCATTER_RET64, 16)


def test_atomic_calibrate_rejects_bad_arguments():
    """Argument checks run before any device call (no GPU needed)."""
    with pytest.raises(H.HclibError):
        H.atomic_calibrate(3, 16)
    with pytest.raises(H.HclibError):
        H.atomic_calibrate(H.ATOMIC_HOT_WORD, 1)


def test_dag_begin_checks_arguments_then_needs_a_gpu():
    """hclib_hip_dag_begin validates the graph on the host (out-of-range
    promise ids, non-monotone CSR) before touching a device, and without a
    gfx950 device a valid graph fails with ENODEV — no CPU fallback."""
    import ctypes as C

    import torch

    lib = C.CDLL(H.LIB_PATH)
    out = (C.c_char * 64)()
    off = (C.c_uint32 * 3)(0, 1, 2)
    bad_ids = (C.c_uint32 * 2)(0, 7)  # promise 7 of 2
    fn = lib.hclib_hip_dag_begin
    fn.restype = C.c_int
    rc = fn(C.c_uint32(2), C.c_uint32(2), C.c_uint32(0), None, off, bad_ids, None, None, 4,
            C.c_uint32(100), C.byref(out))
    assert rc == -2  # EINVAL, with or without a GPU
    nonmono = (C.c_uint32 * 3)(0, 2, 1)
    ids = (C.c_uint32 * 2)(0, 1)
    rc = fn(C.c_uint32(2), C.c_uint32(2), C.c_uint32(0), None, nonmono, ids, None, None, 4,
            C.c_uint32(100), C.byref(out))
    assert rc == -2
    if torch.cuda.is_available():
        return
    rc = fn(C.c_uint32(2), C.c_uint32(2), C.c_uint32(0), None, off, ids, None, None, 4,
            C.c_uint32(100), C.byref(out))
    assert rc == -1  # ENODEV: a valid graph needs the GPU


def test_sw_band_checks_arguments_then_needs_a_gpu():
    """hclib_hip_sw_band_*: bands outside the tile grid, uncoded sequences and
    a missing left column are rejected on the host; without a gfx950 device a
    valid band fails with ENODEV — no CPU fallback."""
    import torch

    s = bytes([1, 2, 3, 4] * 64)
    with pytest.raises(H.HclibError, match="outside"):
        H.SwBand(s, s, 64, 64, 2, 5)  # 4 tile columns
    with pytest.raises(H.HclibError, match="outside"):
        H.SwBand(s, s, 64, 64, 1, 1)
    with pytest.raises(H.HclibError, match="coded"):
        H.SwBand(bytes(256), s, 64, 64, 0, 4)
    with pytest.raises(H.HclibError, match="invalid"):
        H._check(H.lib().hclib_hip_sw_band_rows(None, 0, 1, None, None, None), "rows")
    with pytest.raises(H.HclibError, match="null"):
        H._check(H.lib().hclib_hip_sw_band_end(None, None, None, None), "end")
    if not torch.cuda.is_available():
        with pytest.raises(H.HclibError):
            H.SwBand(s, s, 64, 64, 1, 3)


def test_global_region_layout_and_no_gpu_failures():
    """Cross-GPU sharing region (hclib_hip_global_*): its size is a host-side
    function of the slot count (header + {seq, cnt} pairs + 2-KiB chunk
    payloads), bad capacities are refused, and without a GPU the calls that
    touch a device fail with an error instead of falling back."""
    import torch

    n = H.global_bytes(1024)
    assert n >= 1024 * 8 + 1024 * 64 * 8 * 4 and n % 256 == 0
    assert H.global_bytes(2048) - H.global_bytes(1024) == 1024 * (8 + 64 * 8 * 4)
    with pytest.raises(H.HclibError):
        H.global_bytes(1000)  # not a power of two
    with pytest.raises(H.HclibError):
        H.global_init(0, 1024, 2)  # no region
    with pytest.raises(KeyError):
        H.global_alloc(1024, "host")  # no such region memory
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(H.HclibError):
        H.global_attach(None)
    with pytest.raises(H.HclibError):
        H.ipc_import(b"\0" * 64)
    with pytest.raises(H.HclibError):
        H.global_alloc(1024)
