"""The C++ mirror (include/chordx.hpp) runs the reference's gtest cases for the
lookup path (tests/cpp/test_chordx_api.cpp) on the GPU."""
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "test_chordx_api")


def test_cpp_driver_builds_and_links():
    assert os.path.exists(BIN), "build() compiles tests/cpp/test_chordx_api"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libchordx.so" in out


@pytest.mark.gpu
def test_cpp_reference_cases_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout + r.stderr
