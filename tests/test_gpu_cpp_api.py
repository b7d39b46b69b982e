"""Compile and run the C++ API check (tests/cpp/test_stereo_api.cpp) on the GPU box."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cpp_stereo_api(tmp_path):
    exe = str(tmp_path / "test_stereo_api")
    lib = os.path.join(ROOT, "tea_stereo_matching_amd", "lib")
    subprocess.run(["g++", "-std=c++20", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_stereo_api.cpp"), "-o", exe,
                    f"-L{lib}", "-ltsm_adcensus", f"-Wl,-rpath,{lib}", "-L/opt/rocm/lib",
                    "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
