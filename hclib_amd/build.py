"""Build the MI355X module library in-tree with hipcc (gfx950 only).

    python -m hclib_amd.build        -> hclib_amd/lib/libhclib_amd.so
    python -m hclib_amd.build --variant stamps
                                     -> hclib_amd/lib/stamps/libhclib_amd.so (-DHX_STAMPS=1,
                                        diagnostic per-phase cycle stamps; load it with
                                        HCLIB_AMD_LIB=<path>; never benchmark it)

The library holds every hand-written HIP kernel plus the C ABI of
include/hclib_hip.h (modules/hip) and include/hclib.h (the HClib C API).
Sources compile in parallel; an unchanged source is not rebuilt.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "lib")
LIB = os.path.join(OUT, "libhclib_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["module.hip", "forasync.hip", "uts.hip", "fib.hip", "sw.hip", "dag.hip", "hclib_api.hip", "locality.hip",
           "calib.hip"]
CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result",
    "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
]


# per-source additions: the UTS megakernel under the iterative ILP machine
# scheduler (T3L 27.00-27.12 -> 26.80-26.82 ms, T1 / T1XL even,
# profiles/r06/ab_sched_nf.log; per-source: 26.85-27.10 -> 26.72-26.95, T3
# 2.61 -> 2.58, T1XL +0.2 %, ab_ilp.log; the other sources keep the default:
# the SW kernels are slower under it, 6.46 -> 6.90 ms, ab_sched_sw.log, and
# fib(30) even, 0.380 / 0.380 ms, ab_fibilp.log)
SOURCE_FLAGS = {"uts.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}

VARIANTS = {
    # diagnostic builds (never benchmarked): per-phase cycle stamps, the SW
    # DAG's critical-path trace, worker timelines, main-loop batch phases
    "stamps": ["-DHX_STAMPS=1"], "trace": ["-DHX_TRACE=1"], "timeline": ["-DHX_TIMELINE=1"],
    "phases": ["-DHX_PHASES=1"],
    # memory-model alternatives: the formal agent release/acquire fences
    # around every hand-off (chunks; the seeding's levels), measured slower
    "strict": ["-DHX_STRICT_HANDOFF=1"], "seedfence1": ["-DHX_SEED_FENCES=1"],
    # compiler machine-scheduler strategies (within noise on T3L)
    "sched_minreg": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"],
    "sched_ilp": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "base": [],
}


def _hash(paths, cflags):
    h = hashlib.sha1()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(cflags).encode())
    return h.hexdigest()[:16]


def _headers():
    hs = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".h")]
    inc = os.path.join(ROOT, "include")
    for d, _, fs in sorted(os.walk(inc)):
        hs += [os.path.join(d, f) for f in sorted(fs) if f.endswith(".h")]
    return hs


def _compile(src: str, hdrs, out: str, cflags) -> str:
    path = os.path.join(CSRC, src)
    obj = os.path.join(out, src.replace(".hip", "") + "." + _hash([path] + hdrs, cflags) + ".o")
    if not os.path.exists(obj):
        cmd = [HIPCC] + cflags + ["-c", "-x", "hip", path, "-o", obj + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
        os.replace(obj + ".tmp", obj)
    return obj


def build(verbose: bool = True, variant: str = "") -> str:
    out = os.path.join(OUT, variant) if variant else OUT
    lib = os.path.join(out, "libhclib_amd.so")
    cflags = CFLAGS + VARIANTS[variant] if variant else CFLAGS
    os.makedirs(out, exist_ok=True)
    hdrs = _headers()
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdrs, out, cflags + SOURCE_FLAGS.get(s, [])), srcs))
    stamp = os.path.join(out, ".stamp")
    key = "|".join(objs)
    if not os.path.exists(lib) or not os.path.exists(stamp) or open(stamp).read() != key:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs + [
            "-lpthread", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(lib + ".tmp", lib)
        with open(stamp, "w") as f:
            f.write(key)
    # drop stale objects, and the per-object offload-bundle files the link
    # step leaves beside the library (libhclib_amd.so.<n>.<target>)
    keep = set(objs)
    for f in os.listdir(out):
        p = os.path.join(out, f)
        if (f.endswith(".o") and p not in keep) or (f.startswith("libhclib_amd.so.") and not f.endswith(".stamp")):
            os.remove(p)
    if verbose:
        print("built", lib)
    build_modules(out, lib, cflags, verbose)
    return lib


MODULES = {"hip": "modules/hclib_hip_module.hip"}


def build_modules(out: str, lib: str, cflags, verbose: bool = True) -> list:
    """The plug-in modules (libhclib_<name>.so beside libhclib_amd.so, where
    hclib_launch's dlopen of `deps` finds them; src/hclib-runtime.c:294-317):
    "hip" registers the GPU locale type and its memory callbacks."""
    built = []
    for name, src in MODULES.items():
        so = os.path.join(out, f"libhclib_{name}.so")
        path = os.path.join(CSRC, src)
        key = _hash([path] + _headers() + [lib], cflags)
        stamp = so + ".stamp"
        if not (os.path.exists(so) and os.path.exists(stamp) and open(stamp).read() == key):
            cmd = [HIPCC] + cflags + ["-shared", "-x", "hip", path, "-o", so + ".tmp", "-L" + out, "-lhclib_amd",
                                      "-Wl,-rpath,$ORIGIN"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"module {name} failed:\n{r.stderr[-6000:]}")
            os.replace(so + ".tmp", so)
            with open(stamp, "w") as fh:
                fh.write(key)
        for f in os.listdir(out):  # offload-bundle leftovers of the link step
            if f.startswith(f"libhclib_{name}.so.") and not f.endswith(".stamp"):
                os.remove(os.path.join(out, f))
        built.append(so)
        if verbose:
            print("built", so)
    return built


def build_tests(verbose: bool = True) -> list:
    """Compile the HIP C++ API test programs (tests/hip/*.hip) into
    hclib_amd/lib/tests/ — HIP translation units of the caller's own, linked to
    libhclib_amd.so through an $ORIGIN rpath so they run from any checkout.
    Built here, on the CPU, never inside a GPU test."""
    build(verbose=False)
    tdir = os.path.join(ROOT, "tests", "hip")
    out = os.path.join(OUT, "tests")
    os.makedirs(out, exist_ok=True)
    exes = []
    for f in sorted(os.listdir(tdir)):
        if not f.endswith(".hip"):
            continue
        src = os.path.join(tdir, f)
        exe = os.path.join(out, f[:-4])
        # a HIP object of device kinds linked into a C program of its own
        # (tests/c/<name>_main.c, compiled with gcc against include/hclib.h)
        cmain = os.path.join(ROOT, "tests", "c", f[:-4] + "_main.c")
        deps = [src] + ([cmain] if os.path.exists(cmain) else [])
        key = _hash(deps + _headers() + [LIB], CFLAGS)
        stamp = exe + ".stamp"
        if not (os.path.exists(exe) and os.path.exists(stamp) and open(stamp).read() == key):
            hip = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off",
                   "-I" + os.path.join(ROOT, "include")]
            link = ["-L" + OUT, "-lhclib_amd", "-Wl,-rpath,$ORIGIN/.."]
            if os.path.exists(cmain):
                steps = [hip + ["-c", src, "-o", exe + ".kinds.o"],
                         ["gcc", "-std=gnu11", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), "-c", cmain,
                          "-o", exe + ".main.o"],
                         [HIPCC, f"--offload-arch={ARCH}", exe + ".main.o", exe + ".kinds.o", "-o", exe + ".tmp"] + link]
            else:
                steps = [hip + [src, "-o", exe + ".tmp"] + link]
            for cmd in steps:
                r = subprocess.run(cmd, capture_output=True, text=True)
                if r.returncode != 0:
                    raise RuntimeError(f"build failed for {f}:\n{r.stderr[-6000:]}")
            for tmp in (exe + ".kinds.o", exe + ".main.o"):
                if os.path.exists(tmp):
                    os.remove(tmp)
            os.replace(exe + ".tmp", exe)
            with open(stamp, "w") as fh:
                fh.write(key)
        exes.append(exe)
        if verbose:
            print("built", exe)
    return exes


if __name__ == "__main__":
    v = sys.argv[sys.argv.index("--variant") + 1] if "--variant" in sys.argv else ""
    build(variant=v)
    if not v:
        build_tests()
    sys.exit(0)
