"""The C++ drop-in: programs written against include/hclib_cpp.h (the
reference's namespace-hclib API: launch / async / async_await / finish /
promise_t / future_t / forasync{1,2,3}D) compiled with g++ and linked to
libhclib_amd.so. Host lambdas run on the host control thread, so these run
without a GPU. tests/cpp/*.cpp restate reference test programs
(test/cpp/finish1.cpp, forasync{1,2,3}D{Ch,Rec}.cpp,
nested_finish_async_await.cpp, promise/asyncAwait0Vector.cpp,
promise/future3.cpp) and assert like them ("Check results: OK")."""
import os
import subprocess

import pytest

import hclib_amd as H
from tests.conftest import ROOT

CDIR = os.path.join(ROOT, "tests", "cpp")


def _build(name):
    out = os.path.join("/tmp", f"hclib_cpp_{name}_{os.getpid()}")
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(CDIR, name + ".cpp"), "-o", out, "-L", os.path.dirname(H.LIB_PATH),
           "-lhclib_amd", "-Wl,-rpath," + os.path.dirname(H.LIB_PATH)]
    subprocess.check_call(cmd)
    return out


@pytest.mark.parametrize("name", ["finish_async", "forasync_nd", "promise_api"])
def test_cpp_programs_on_host_lambdas(name):
    r = subprocess.run([_build(name)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Check results: OK" in r.stdout
