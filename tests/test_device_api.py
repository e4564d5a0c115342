"""The device side of the C++ API (include/hclib_hip_cpp.h): a HIP program of
the caller's own (tests/hip/device_api.hip, built by
`python -m hclib_amd.build` / __graft_entry__.build into hclib_amd/lib/tests)
runs forasync{1,2,3}D with __device__ lambdas against the reference's tiling
and two user-defined task kinds (fib call tree, N-Queens) on the megakernel."""
import os
import subprocess

import pytest

import hclib_amd as H

EXE = os.path.join(os.path.dirname(H.LIB_PATH), "tests", "device_api")


def test_device_api_program_is_built():
    assert os.path.exists(EXE), "run python -m hclib_amd.build"


def test_device_api_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "hclib_hip_init" in r.stderr


@pytest.mark.gpu
def test_device_api_on_gpu():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "fib(25) = 75025" in r.stdout and "queens(12) = 14200 solutions" in r.stdout
    assert "worker identity: 150049 tasks on" in r.stdout


DAG_EXE = os.path.join(os.path.dirname(H.LIB_PATH), "tests", "device_dag")


def test_device_dag_program_is_built():
    assert os.path.exists(DAG_EXE), "run python -m hclib_amd.build"


@pytest.mark.gpu
def test_device_promise_dag_on_gpu():
    """Device promises/futures with dependency-counter release
    (include/hclib_hip/hx_dag.h): chain, SW-style wavefront with plain-data
    hand-offs, random DAG with > MAX_NUM_WAITS futures, 30,000-way fan-out,
    all bit-exact against serial host evaluation; a double put and an
    unsatisfiable future return HCLIB_HIP_EDEVICE instead of hanging."""
    r = subprocess.run([DAG_EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "single assignment" in r.stdout and "deadlock" in r.stdout


FIN_EXE = os.path.join(os.path.dirname(H.LIB_PATH), "tests", "device_finish")


def test_device_finish_program_is_built():
    assert os.path.exists(FIN_EXE), "run python -m hclib_amd.build"


@pytest.mark.gpu
def test_device_nested_finish_on_gpu():
    """Nested finish inside device tasks (include/hclib_hip/hx_finish.h):
    fib as test/fib/fib.c writes it (FINISH + continuation) as a user kind
    through run_tasks, fib(0..27) against fib_iter with exact task and
    continuation counts; test/cpp/nested_finish.cpp's 100 iterations x 4
    nested finishes, every finish ending after everything inside it."""
    r = subprocess.run([FIN_EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "fib(27) = 196418" in r.stdout and "nested finish: 100 iterations x 4" in r.stdout


KT_EXE = os.path.join(os.path.dirname(H.LIB_PATH), "tests", "kind_table")


def test_kind_table_program_is_built():
    """tests/hip/kind_table.hip (device kinds of the program's own) linked
    into the C program tests/c/kind_table_main.c."""
    assert os.path.exists(KT_EXE), "run python -m hclib_amd.build"


def test_kind_table_refuses_unknown_builtin_kinds():
    """A kind id outside the table is refused, naming the way to register a
    kind of the program's own (no GPU needed: it fails before any launch)."""
    r = subprocess.run([KT_EXE, "bad"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "unknown kind 99" in r.stderr and "hclib_hip_register_device_async" in r.stderr
    assert "accepted" not in r.stdout


@pytest.mark.gpu
def test_kind_table_device_kinds_from_the_programs_hip_object():
    """The C drop-in runs hclib_async(fib, ...) through the program's own
    device kind (nested-finish fib on the megakernel) and hclib_forasync of
    the program's own device loop body over GPU-locale memory (FLAT and
    RECURSIVE), both checked against host evaluation."""
    r = subprocess.run([KT_EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "Fib(25) = 75025 = 75025" in r.stdout
    assert "forasync (FLAT) of the device body: 100000 indices OK" in r.stdout
    assert "forasync (RECURSIVE) of the device body: 100000 indices OK" in r.stdout
    assert "forasync_future + end_finish_nonblocking with device work: OK" in r.stdout


DYN_EXE = os.path.join(os.path.dirname(H.LIB_PATH), "tests", "device_dyn")


def test_device_dyn_program_is_built():
    assert os.path.exists(DYN_EXE), "run python -m hclib_amd.build"


@pytest.mark.gpu
def test_dynamic_device_dataflow_on_gpu():
    """Device tasks that create promises and async_await tasks while the
    launch runs (include/hclib_hip/hx_dyn.h): fib with data-driven tasks
    (test/fib/fib.c:113-141) for n = 0..22 with the exact task / promise /
    put counts, the smith_waterman.cpp:171-232 tile program (a root task
    creating 3 promises and one async_await per tile) against a serial host
    DP, and a double put / a never-put future returning HCLIB_HIP_EDEVICE."""
    r = subprocess.run([DYN_EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "fib(22) = 17711 with data-driven device tasks" in r.stdout
    assert "as device async_awaits: score" in r.stdout
    assert "single assignment" in r.stdout and "deadlock" in r.stdout
