"""Native C++ tests (tests/cpp/test_native.cpp; the reference's tests/cpp_tests analogue): LCG
stream, string/bitset utilities, shared metric math, C API train -> batch / single-row-fast
predict -> model text round trip -> streaming push rows. Also run under AddressSanitizer +
UBSan when `make asan` has built that binary."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "data")


def _run(binary):
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([binary, DATA], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "all passed" in r.stdout


def test_native_cpp_suite():
    binary = os.path.join(ROOT, "build", "test_native")
    if not os.path.exists(binary):
        subprocess.run(["make", "-j8", "cpptest"], cwd=ROOT, check=True, capture_output=True)
    _run(binary)


def test_native_cpp_suite_under_asan_ubsan():
    binary = os.path.join(ROOT, "build", "asan", "test_native")
    if not os.path.exists(binary):
        pytest.skip("build/asan/test_native not built (make asan; __graft_entry__.build() builds it)")
    _run(binary)
