"""The drop-in boundary: C programs written against include/hclib.h (the
reference's C API) compiled with gcc and linked to libhclib_amd.so.

tests/c/*.c restate reference test programs (test/c/forasync1DCh.c,
test/c/promise/asyncAwait1.c, test/c/promise/future0.c, test/fib/fib.c,
test/uts/UTS.cpp's driver) and assert like them ("Check results: OK").
"""
import os
import subprocess

import pytest

import hclib_amd as H
from tests.conftest import ROOT

CDIR = os.path.join(ROOT, "tests", "c")


def _build(name, tmp_path_factory=None):
    out = os.path.join("/tmp", f"hclib_capi_{name}_{os.getpid()}")
    cmd = ["gcc", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
           os.path.join(CDIR, name + ".c"), "-o", out, "-L", os.path.dirname(H.LIB_PATH),
           "-lhclib_amd", "-Wl,-rpath," + os.path.dirname(H.LIB_PATH)]
    subprocess.check_call(cmd)
    return out


def _run(exe, *args, timeout=300, env=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    return subprocess.run([exe, *map(str, args)], capture_output=True, text=True,
                          timeout=timeout, env=e)


@pytest.mark.parametrize("name", ["promise_chain", "fib_gpu", "forasync1DCh_gpu", "uts_gpu", "mem_locale",
                                  "locale_idle"])
def test_c_programs_compile_against_hclib_h(name):
    assert os.path.exists(_build(name))


def test_host_promise_semantics():
    r = _run(_build("promise_chain"))
    assert r.returncode == 0, r.stderr
    assert "Check results: OK" in r.stdout


def test_locale_tasks_idle_functions_and_harness_timer():
    """locale_num_tasks / locale_register_idle_task / locale_run_idle_tasks
    (inc/hclib-locality-graph.h:102-105) and hclib_user_harness_timer
    (inc/hclib-rt.h:153): link, call, reference semantics."""
    r = _run(_build("locale_idle"), env={"HCLIB_STATS": "1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "User harness timer: 1.250000 s" in r.stdout


def test_host_locale_memory_operations():
    """hclib_allocate_at / reallocate_at / memset_at / async_copy / free_at at
    the host locale (src/hclib-mem.c:23-241) and locale types."""
    r = _run(_build("mem_locale"))
    assert r.returncode == 0, r.stderr
    assert "Check results: OK" in r.stdout


@pytest.mark.gpu
def test_gpu_locale_memory_operations():
    """The same at the GPU locale: the hip plug-in module's hipMalloc /
    hipMemsetAsync / hipMemcpyAsync callbacks (registered in its post-init,
    like modules/cuda/src/hclib_cuda.cpp:169-174), host<->GPU round trip, realloc keeping the prefix, a copy whose
    source is a future (HCLIB_ASYNC_COPY_USE_FUTURE_AS_SRC)."""
    r = _run(_build("mem_locale"), "gpu")
    assert r.returncode == 0, r.stderr
    assert "Check results: OK" in r.stdout
    # every GPU-locale operation ran the hip plug-in module's callbacks
    assert "hip module callbacks: alloc 1, realloc 1, free 1, memset 1, copy 5" in r.stdout


def test_device_kinds_fail_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = _run(_build("fib_gpu"), 10)
    assert r.returncode != 0
    assert "hip module could not bind" in r.stderr


@pytest.mark.gpu
def test_fib_c_program_on_gpu():
    r = _run(_build("fib_gpu"), 30)
    assert r.returncode == 0, r.stderr
    assert "Fib(30) = 832040 = 832040" in r.stdout and "Check results: OK" in r.stdout


@pytest.mark.gpu
def test_forasync1DCh_c_program_on_gpu():
    r = _run(_build("forasync1DCh_gpu"))
    assert r.returncode == 0, r.stderr
    assert "Check results: OK" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["T1", "T3", "T3L"])
def test_uts_c_program_on_gpu(golden, name):
    g = golden("uts_goldens.json")["published"][name]
    r = _run(_build("uts_gpu"), *g["args"].split())
    assert r.returncode == 0, r.stderr
    want = (f"Tree size = {g['nodes']}, tree depth = {g['depth']}, "
            f"num leaves = {g['leaves']}")
    assert want in r.stdout, r.stdout


def test_hclib_stats_report_layout():
    """HCLIB_STATS=1 prints the reference's report layout at finalize
    (src/hclib-runtime.c:1370-1410): the banner, a per-worker line, totals."""
    r = _run(_build("promise_chain"), env={"HCLIB_STATS": "1"})
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "===== HClib statistics: =====" in out
    assert "  Worker 0: " in out and " tasks executed, " in out
    assert "Total: " in out and " end finishes, " in out and " future waits, " in out


@pytest.mark.gpu
def test_hclib_stats_per_wave_device_lines(golden):
    """HCLIB_STATS=1 after a device UTS task (tests/c/uts_gpu.c, T1): one
    "Device wave" line per megakernel wave, each written by the wave itself
    (hclib_hip_last_wave_stats), in the reference's per-worker layout
    (src/hclib-runtime.c:1370-1410). Their sums equal the launch-wide
    scheduler counters on the aggregate line, and the tasks they executed
    are the tree's nodes below the root (the root is counted by roots())."""
    import re

    g = golden("uts_goldens.json")["published"]["T1"]
    r = _run(_build("uts_gpu"), *g["args"].split(), env={"HCLIB_STATS": "1"})
    assert r.returncode == 0, r.stderr
    pat = re.compile(r"  Device wave (\d+) \(XCD (\d)\): (\d+) tasks executed, (\d+) tasks spawned, "
                     r"(\d+) batches, (\d+) chunks pushed, (\d+) steals, (\d+) stolen tasks, [\d.]+ tasks per "
                     r"steal, stolen from = \[ ((?:\d+ ){8})\]")
    waves = [tuple(int(x) for x in m.groups()[:8]) + (list(map(int, m.group(9).split())),)
             for m in pat.finditer(r.stdout)]
    assert len(waves) >= 256 and [w[0] for w in waves] == list(range(len(waves)))
    agg = re.search(r"  Device \((\d+) waves\): (\d+) device items executed in (\d+) batches, (\d+) chunks "
                    r"pushed, (\d+) chunks stolen", r.stdout)
    assert agg, r.stdout[-2000:]
    nw, items, batches, pushed, stolen = map(int, agg.groups())
    assert nw == len(waves) and items == g["nodes"]
    assert sum(w[4] for w in waves) == batches
    assert sum(w[5] for w in waves) == pushed
    assert sum(w[6] for w in waves) == stolen
    assert sum(sum(w[8]) for w in waves) == stolen
    assert sum(w[2] for w in waves) == g["nodes"] - 1
    assert len({w[1] for w in waves}) == 8  # waves ran on all eight XCDs
