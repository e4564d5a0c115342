"""The plug-in boundary: task records and spawn*, worker state,
modules loaded from `deps`, per-worker module state, locale metadata and
locality files — all through the C-ABI library, no GPU needed.

* tests/c/spawn_api.c drives spawn / spawn_at / spawn_await / spawn_await_at
  with caller-built 96-byte hclib_task_t records (inc/hclib-async-struct.h:
  49-54, inc/hclib-task.h:32-44), current_ws(), a module's pre/post/finalize
  hooks, per-worker module state and locale metadata (inc/hclib-module.h:
  79-106, src/hclib_module.c:49-160).
* The reference's own modules/system/src/hclib_system.cpp is compiled,
  unmodified, against include/ into libhclib_system.so; a program launched
  with deps {"system"} loads it (src/hclib-runtime.c:294-317) and runs on its
  locale types and memory callbacks; the reference's own module tests
  (modules/system/test/init.cpp) runs against it too. Skipped
  where /root/reference is absent (the GPU box).
* tests/c/locality_file.c loads the reference's locality_graphs/davinci.json
  (a data fixture, tests/golden/locality/) with HCLIB_LOCALITY_FILE.
"""
import os
import subprocess

import pytest

import hclib_amd as H
from tests.conftest import GOLD, ROOT

REF_SYSTEM = "/root/reference/modules/system"
LIBDIR = os.path.dirname(H.LIB_PATH)
INC = os.path.join(ROOT, "include")


def _link():
    return ["-L", LIBDIR, "-lhclib_amd", "-Wl,-rpath," + LIBDIR]


def _build_c(name, out_dir):
    exe = os.path.join(out_dir, name)
    subprocess.check_call(["gcc", "-std=gnu11", "-O1", "-Wall", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "c", name + ".c"), "-o", exe] + _link())
    return exe


def _run(exe, *args, env=None):
    e = dict(os.environ)
    e.pop("HCLIB_LOCALITY_FILE", None)
    e.pop("HCLIB_WORKERS", None)
    if env:
        e.update(env)
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=120, env=e)


def test_task_record_spawn_and_module_state(tmp_path):
    r = _run(_build_c("spawn_api", str(tmp_path)))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout


def test_library_exports_the_plugin_boundary():
    import ctypes

    lib = ctypes.CDLL(H.LIB_PATH)
    for sym in ("spawn", "spawn_at", "spawn_await", "spawn_await_at", "current_ws", "ws_key",
                "hclib_add_locale_metadata_functions", "hclib_add_per_worker_module_state",
                "hclib_get_curr_worker_module_state", "hclib_release_per_worker_module_state",
                "hclib_call_module_pre_init_functions", "hclib_call_module_post_init_functions",
                "hclib_call_finalize_functions", "load_locality_info", "generate_locality_info",
                "print_locality_graph", "print_worker_paths"):
        assert hasattr(lib, sym), sym


def test_locality_file_with_gpu_locales(tmp_path):
    exe = _build_c("locality_file", str(tmp_path))
    f = os.path.join(GOLD, "locality", "davinci.json")
    r = _run(exe, env={"HCLIB_LOCALITY_FILE": f})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout
    assert "GPU0 (type GPU): sysmem" in r.stderr  # print_locality_graph
    assert "Worker 1\n  pop path: L2_0_1 L3_0 sysmem" in r.stderr


def test_locality_file_gpu_type_comes_from_the_hip_module(tmp_path):
    """Without "hip" in deps nothing registers the GPU locale type, so the
    file's GPU locales are unknown, as in the reference without
    modules/cuda (src/hclib-locality-graph.c:322-367)."""
    exe = _build_c("locality_file", str(tmp_path))
    f = os.path.join(GOLD, "locality", "davinci.json")
    r = _run(exe, "nohip", env={"HCLIB_LOCALITY_FILE": f})
    assert r.returncode == 1
    assert 'Unknown locale type for locale "GPU0"' in r.stderr


def test_hip_module_library_exports():
    import ctypes

    so = os.path.join(LIBDIR, "libhclib_hip.so")
    assert os.path.exists(so)
    lib = ctypes.CDLL(so)
    for sym in ("hclib_hip_module_counts", "hclib_hip_module_gpu_type"):
        assert hasattr(lib, sym), sym


@pytest.mark.gpu
def test_locality_file_gpu_locale_memory_through_the_module(tmp_path):
    """hclib_allocate_at / memset_at / async_copy / free_at at the GPU0
    locale that davinci.json declares, run by the hip plug-in module's
    registered callbacks (asserted through its counters)."""
    exe = _build_c("locality_file", str(tmp_path))
    f = os.path.join(GOLD, "locality", "davinci.json")
    r = _run(exe, "gpu", env={"HCLIB_LOCALITY_FILE": f})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout and "hip module callbacks: alloc 1" in r.stdout


def test_locality_file_unknown_locale_type_is_fatal(tmp_path):
    exe = _build_c("locality_file", str(tmp_path))
    f = os.path.join(GOLD, "locality", "davinci.json")
    r = _run(exe, "nointerconnect", env={"HCLIB_LOCALITY_FILE": f})
    assert r.returncode == 1
    assert 'Unknown locale type for locale "Interconnect"' in r.stderr


def test_locality_file_missing_is_fatal(tmp_path):
    exe = _build_c("locality_file", str(tmp_path))
    r = _run(exe, env={"HCLIB_LOCALITY_FILE": str(tmp_path / "nope.json")})
    assert r.returncode == 1 and "Failed loading locality graph" in r.stderr


@pytest.fixture(scope="module")
def system_module(tmp_path_factory):
    if not os.path.isdir(REF_SYSTEM):
        pytest.skip("reference sources not present")
    out = str(tmp_path_factory.mktemp("sysmod"))
    so = os.path.join(out, "libhclib_system.so")
    # compiled from where it lies, unmodified: only include/ and the
    # module's own inc/ on the include path
    r = subprocess.run(["g++", "-std=c++14", "-O1", "-fPIC", "-shared", "-I", os.path.join(REF_SYSTEM, "inc"),
                        "-I", INC, os.path.join(REF_SYSTEM, "src", "hclib_system.cpp"), "-o", so] + _link(),
                       capture_output=True, text=True)
    assert r.returncode == 0, "modules/system does not compile against include/:\n" + r.stderr[-3000:]
    return out


def test_reference_system_module_compiles_and_loads(system_module, tmp_path):
    exe = str(tmp_path / "system_module")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", INC,
                           os.path.join(ROOT, "tests", "cpp", "system_module.cpp"), "-o", exe,
                           "-L", system_module, "-lhclib_system", "-Wl,-rpath," + system_module] + _link())
    r = _run(exe, env={"HCLIB_MODULE_PATH": system_module})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout


def test_system_module_is_found_through_deps_only(system_module, tmp_path):
    """Not linked: found by hclib_launch's dlopen of HCLIB_ROOT/lib/libhclib_system.so."""
    root = tmp_path / "root"
    (root / "lib").mkdir(parents=True)
    os.symlink(os.path.join(system_module, "libhclib_system.so"), root / "lib" / "libhclib_system.so")
    src = tmp_path / "probe.c"
    src.write_text(
        '#include <assert.h>\n#include <stdio.h>\n#include <string.h>\n#include "hclib.h"\n'
        'static void body(void *a) { (void)a; char *p = hclib_future_wait(hclib_allocate_at(64, '
        'hclib_get_central_place()));\n assert(p[0] == 42); assert(strcmp(hclib_get_closest_locale()->lbl, "L10") == 0);'
        ' printf("Check results: OK\\n"); }\n'
        'int main(void) { const char *deps[] = {"system"}; hclib_launch(body, NULL, deps, 1); return 0; }\n')
    exe = str(tmp_path / "probe")
    subprocess.check_call(["gcc", "-std=gnu11", "-O1", "-I", INC, str(src), "-o", exe] + _link())
    r = _run(exe, env={"HCLIB_ROOT": str(root)})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Check results: OK" in r.stdout


@pytest.mark.parametrize("prog", ["init"])
def test_reference_system_module_tests(system_module, tmp_path, prog):
    """modules/system/test/init.cpp, unmodified. (Its allocate.cpp uses an
    untyped hclib::future_t that the reference's own inc/hclib_future.h no
    longer declares, so it is stale against the reference too; what it
    exercises is covered by tests/cpp/system_module.cpp.)"""
    exe = str(tmp_path / prog)
    r = subprocess.run(["g++", "-std=c++14", "-O1", "-w", "-I", os.path.join(REF_SYSTEM, "inc"), "-I", INC,
                        os.path.join(REF_SYSTEM, "test", prog + ".cpp"), "-o", exe, "-L", system_module,
                        "-lhclib_system", "-Wl,-rpath," + system_module] + _link(), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _run(exe, env={"HCLIB_MODULE_PATH": system_module})
    assert r.returncode == 0, r.stdout + r.stderr
