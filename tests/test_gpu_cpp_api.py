"""Compile and run the C++ API checks on the GPU box; each program's disparity is then
compared with the oracle's, bit for bit.

* tests/cpp/test_stereo_api.cpp: include/stereo.h without OpenCV (ImageView virtual),
  plus the f2-f4 calls.
* tests/cpp/test_stereo_api_cvmat.cpp: include/stereo.h with a cv::Mat on the include path
  (tests/cpp/cvshim), so StereoMatching's pure virtual is the reference's
  compute(const cv::Mat&, const cv::Mat&, cv::Mat&) (reference stereo.h:325-331) and the
  matcher is called through a StereoMatching&, on ROI (non-continuous) inputs.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, host_threads

pytestmark = pytest.mark.gpu

LIB = os.path.join(ROOT, "tea_stereo_matching_amd", "lib")


def compile_program(src, exe, opencv):
    cmd = ["g++", "-std=c++20", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include")]
    if opencv:
        cmd += ["-I", os.path.join(ROOT, "tests", "cpp", "cvshim")]
    cmd += [os.path.join(ROOT, "tests", "cpp", src), "-o", exe, f"-L{LIB}", "-ltsm_adcensus",
            f"-Wl,-rpath,{LIB}", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)


@pytest.mark.parametrize("src,opencv", [("test_stereo_api.cpp", False),
                                        ("test_stereo_api_cvmat.cpp", True)])
def test_cpp_stereo_api(tmp_path, src, opencv):
    exe = str(tmp_path / "prog")
    compile_program(src, exe, opencv)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
    # the C++ class's disparity of its own 48x80 pair, bit-exact against the oracle
    # (RGB, D = [0, 16], serial scanline: the class's settings in the program)
    from oracle import oracle as O
    H, W = 48, 80
    left = np.fromfile(tmp_path / "left.bgr", np.uint8).reshape(H, W, 3)
    right = np.fromfile(tmp_path / "right.bgr", np.uint8).reshape(H, W, 3)
    got = np.fromfile(tmp_path / "disp.f32", np.float32).reshape(H, W)
    want, _ = O.compute(left, right, O.default_params(O.RGB, 0, 16, num_threads=host_threads()))
    assert np.array_equal(got, want)
